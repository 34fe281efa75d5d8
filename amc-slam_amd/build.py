"""Build libamc_lba.so in-tree with hipcc for gfx950 (no CMake), and the LocalGPBA host
adapter libamc_lba_map.so (plain C++, g++) on top of it.

    python amc-slam_amd/build.py            # incremental
    python amc-slam_amd/build.py --force
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib", "libamc_lba.so")
SOURCES = ["lba_kernels.hip", "lba_host.hip", "lba_track.hip"]
HEADERS = ["lba_device.hpp", "lba_math.hpp", os.path.join("..", "..", "include", "amc_lba.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall"]
HOST = os.path.join(HERE, "host")
MAP_LIB = os.path.join(HERE, "lib", "libamc_lba_map.so")
MAP_SOURCES = ["lba_map.cpp", "optimizer.cpp", "capi.cpp"]
MAP_HEADERS = ["lba_map.hpp", "optimizer.hpp", os.path.join("..", "..", "include", "amc_lba_map.h"),
               os.path.join("..", "..", "include", "amc_lba.h"), os.path.join("..", "csrc", "lba_math.hpp")]
CXX = os.environ.get("CXX", "g++")
# -ffp-contract=off: the adapter's float conversions follow the reference's rounding step by step
MAP_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra", "-ffp-contract=off"]


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS)


def map_needs_build():
    if not os.path.exists(MAP_LIB) or os.path.getmtime(MAP_LIB) < os.path.getmtime(LIB):
        return True
    t = os.path.getmtime(MAP_LIB)
    return any(os.path.getmtime(os.path.join(HOST, f)) > t for f in MAP_SOURCES + MAP_HEADERS)


def build(force=False, verbose=True):
    if force or needs_build():
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        cmd = [HIPCC] + FLAGS + [os.path.join(CSRC, s) for s in SOURCES] + ["-o", LIB, "-lrccl"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    if force or map_needs_build():
        cmd = [CXX] + MAP_FLAGS + [os.path.join(HOST, s) for s in MAP_SOURCES] + [
            "-o", MAP_LIB, "-L" + os.path.dirname(LIB), "-lamc_lba", "-Wl,-rpath,$ORIGIN"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
