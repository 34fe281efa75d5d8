"""The drop-in boundary: libamc_lba.so loads, exports every function include/amc_lba.h declares,
the numpy/ctypes mirrors of the structs have the C layout, and the product fails loudly (no
silent CPU fallback) when the library or the GPU is missing.  No compute calls here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import amc_lba
from amc_lba import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "amc_lba.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|void|const char\*)\s+(lba_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for n in ("lba_create", "lba_set_problem", "lba_optimize", "lba_get_state", "lba_eval", "lba_linearize",
              "lba_solve_step", "lba_destroy"):
        assert n in names


def test_library_exports_every_declared_symbol():
    L = amc_lba.lib()
    exported = subprocess.run(["nm", "-D", "--defined-only", amc_lba.LIB_PATH], capture_output=True,
                              text=True).stdout
    for n in declared_functions():
        assert hasattr(L, n), n
        assert re.search(rf"\bT {n}\b", exported), n
    assert set(amc_lba.exported_symbols()) <= set(declared_functions())
    assert L.lba_abi_version() == 5


def _c_sizeof(struct):
    code = f'#include "{HEADER}"\n#include <stdio.h>\n#include <stddef.h>\nint main(void){{printf("%zu", sizeof({struct}));return 0;}}'
    exe = "/tmp/_abi_sz"
    subprocess.run(["gcc", "-x", "c", "-", "-o", exe], input=code, text=True, check=True)
    return int(subprocess.run([exe], capture_output=True, text=True, check=True).stdout)


@pytest.mark.parametrize("struct,dtype", [("lba_kf", abi.KF_DTYPE), ("lba_obs", abi.OBS_DTYPE),
                                          ("lba_prior", abi.PRIOR_DTYPE), ("lba_cam", abi.CAM_DTYPE)])
def test_struct_layouts_match_header(struct, dtype):
    assert _c_sizeof(struct) == dtype.itemsize


def test_track_structs_match_header():
    from amc_lba.track import TRACK_FRAME_DTYPE, TRACK_OBS_DTYPE
    assert _c_sizeof("lba_track_obs") == TRACK_OBS_DTYPE.itemsize
    assert _c_sizeof("lba_track_frame") == TRACK_FRAME_DTYPE.itemsize


def test_ctypes_structs_match_header():
    assert _c_sizeof("lba_config") == ctypes.sizeof(abi.LbaConfig)
    assert _c_sizeof("lba_stats") == ctypes.sizeof(abi.LbaStats)


def test_create_without_gpu_fails_cleanly():
    """No GPU in the build container: lba_create must return an error code, never crash."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    h = ctypes.c_void_p()
    cfg = abi.make_config()
    rc = amc_lba.lib().lba_create(ctypes.byref(h), ctypes.byref(cfg))
    assert rc in (abi.LBA_E_HIP, abi.LBA_E_ARG)
    assert not h.value


def test_missing_library_fails_loudly(monkeypatch):
    monkeypatch.setattr(amc_lba, "_lib", None)
    monkeypatch.setattr(amc_lba, "LIB_PATH", "/nonexistent/libamc_lba.so")
    with pytest.raises(RuntimeError):
        amc_lba.lib()


def test_null_arguments_rejected():
    L = amc_lba.lib()
    assert L.lba_create(None, None) == abi.LBA_E_ARG
    assert L.lba_optimize(None, 1, None, None) == abi.LBA_E_ARG
    assert L.lba_get_state(None, None, None) == abi.LBA_E_ARG


def _layout(threads, window="make_config_window('cfg1_local_50kf')"):
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, 'amc-slam_amd'); import amc_lba; "
            "from amc_lba.synth import make_config_window, make_window; "
            f"ms, c = amc_lba.setup_host_profile({window}); print(*c)")
    env = dict(os.environ, LBA_SETUP_THREADS=str(threads))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    return out.stdout.split()


def test_set_problem_host_layout_independent_of_threads():
    """lba_setup_host_profile (the host preprocessing of lba_set_problem, no GPU): the tiling and slab
    layout of config 1 is the same with 1 and 8 set-up threads (fixed work pieces)."""
    one, eight = _layout(1), _layout(8)
    assert one == eight
    n_lm, n_pb, np_, tiles, _ = (int(x) for x in one)
    assert n_lm == 20000 and n_pb == 50 and np_ == 600 and 900 < tiles < 1200


def test_set_problem_host_layout_small_window_independent_of_threads():
    """The same for a LocalGPBA-sized window (3000 landmarks: below 256 per piece, so its tiles are cut in one piece
    and their lists built in parallel runs of tiles) -- the layout fingerprint covers every tile list."""
    w = "make_window(n_opt_kf=11, n_lm=3000, obs_per_lm=6, n_cam=4, gp=True, seed=21)"
    one, eight = _layout(1, w), _layout(8, w)
    assert one == eight
    n_lm, n_pb, np_, tiles, _ = (int(x) for x in one)
    assert n_lm == 3000 and tiles > 16   # more tiles than set-up pieces: the runs split the list building


def _pool_stress(threads, passes, pieces):
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, 'amc-slam_amd'); import amc_lba; "
            f"print(amc_lba.lib().lba_debug_pool_stress({passes}, {pieces}))")
    env = dict(os.environ, LBA_SETUP_THREADS=str(threads))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True,
                         cwd=ROOT)
    return int(out.stdout.split()[-1])


@pytest.mark.parametrize("threads", [2, 8])
def test_setup_pool_back_to_back_passes(threads):
    """lba_set_problem's host thread pool (SetupPool): many short passes back to back, each with a different
    piece count (a pass with more pieces right after one with fewer is where a late worker of the old pass
    could claim a piece of the new one): every piece runs exactly once, inside its own pass."""
    assert _pool_stress(threads, 20000, 64) == 0


def test_header_constants_match_the_python_mirror():
    """Every LBA_FLAG_* bit, status code and observation kind the header defines has the same value in amc_lba.abi
    (a caller of either side sets the same bits)."""
    src = open(HEADER).read()
    macros = {m: int(v) for m, v in re.findall(r"^#define\s+(LBA_\w+)\s+(-?\d+)", src, flags=re.M)}
    flags = {m: v for m, v in macros.items() if m.startswith("LBA_FLAG_")}
    assert "LBA_FLAG_F32_RESIDUAL" in flags
    for m, v in flags.items():
        assert getattr(abi, m[len("LBA_"):]) == v, m
    assert len(set(flags.values())) == len(flags) and all(v & (v - 1) == 0 for v in flags.values())   # one bit each
    for m in ("LBA_OK", "LBA_E_EMPTY", "LBA_E_SOLVE", "LBA_E_DIVERGED", "LBA_E_ARG", "LBA_E_HIP", "LBA_E_LIMIT", "LBA_E_TIMEOUT"):
        assert getattr(abi, m) == macros[m], m
    for m in ("LBA_MONO_GP", "LBA_STEREO_GP", "LBA_MONO", "LBA_STEREO"):
        assert getattr(abi, m[len("LBA_"):]) == macros[m], m
