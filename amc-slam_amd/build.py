"""Build libamc_lba.so in-tree with hipcc for gfx950 (no CMake), and the LocalGPBA host
adapter libamc_lba_map.so (plain C++, g++) on top of it.

    python amc-slam_amd/build.py            # rebuild what is stale
    python amc-slam_amd/build.py --force

Staleness is decided by content, not mtime: each library gets a `<lib>.stamp` holding the sha256 of
its compiler line and every source and header it is built from.  A prebuilt .so that travelled to a
GPU box with newer sources (gpurun copies both) is therefore rebuilt by build(), and refused by
`stale()` / the loaders in amc_lba (they compare the stamp with the sources before dlopen).
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib", "libamc_lba.so")
SOURCES = ["lba_kernels.hip", "lba_host.hip", "lba_track.hip", "lba_debug.hip"]
HEADERS = ["lba_device.hpp", "lba_math.hpp", "lba_plan.hpp", os.path.join("..", "..", "include", "amc_lba.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall"]
HOST = os.path.join(HERE, "host")
MAP_LIB = os.path.join(HERE, "lib", "libamc_lba_map.so")
MAP_SOURCES = ["lba_map.cpp", "optimizer.cpp", "bundle_adjustment.cpp", "capi.cpp"]
MAP_HEADERS = ["lba_map.hpp", "optimizer.hpp", os.path.join("..", "..", "include", "amc_lba_map.h"),
               os.path.join("..", "..", "include", "amc_lba.h"), os.path.join("..", "csrc", "lba_math.hpp")]
CXX = os.environ.get("CXX", "g++")
# -ffp-contract=off: the adapter's float conversions follow the reference's rounding step by step
MAP_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", "-Wextra", "-ffp-contract=off"]


def _digest(cmd_flags, files, extra=b""):
    h = hashlib.sha256()
    h.update(" ".join(cmd_flags).encode())
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(extra)
    return h.hexdigest()


def lib_digest():
    return _digest(FLAGS, [os.path.join(CSRC, f) for f in SOURCES + HEADERS])


def map_digest():
    # the adapter links the engine: a new engine stamp re-stamps the adapter
    return _digest(MAP_FLAGS, [os.path.join(HOST, f) for f in MAP_SOURCES + MAP_HEADERS], lib_digest().encode())


def _stamp_ok(path, digest):
    try:
        with open(path + ".stamp") as fh:
            return os.path.exists(path) and fh.read().strip() == digest
    except OSError:
        return False


def _write_stamp(path, digest):
    with open(path + ".stamp", "w") as fh:
        fh.write(digest + "\n")


def stale(which="engine"):
    """None if the library matches its sources, else a one-line reason (used by the loaders)."""
    path, dig = (LIB, lib_digest) if which == "engine" else (MAP_LIB, map_digest)
    if not os.path.exists(path):
        return f"{path} not built"
    if not _stamp_ok(path, dig()):
        return f"{path} does not match its sources (stamp {path}.stamp)"
    return None


def needs_build():
    return not _stamp_ok(LIB, lib_digest())


def map_needs_build():
    return not _stamp_ok(MAP_LIB, map_digest())


def build(force=False, verbose=True):
    if force or needs_build():
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        cmd = [HIPCC] + FLAGS + [os.path.join(CSRC, s) for s in SOURCES] + ["-o", LIB, "-lrccl"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        _write_stamp(LIB, lib_digest())
    if force or map_needs_build():
        cmd = [CXX] + MAP_FLAGS + [os.path.join(HOST, s) for s in MAP_SOURCES] + [
            "-o", MAP_LIB, "-L" + os.path.dirname(LIB), "-lamc_lba", "-Wl,-rpath,$ORIGIN"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        _write_stamp(MAP_LIB, map_digest())
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
