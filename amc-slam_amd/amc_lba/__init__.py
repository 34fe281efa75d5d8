"""Python binding of the MI355X local-BA C ABI (include/amc_lba.h) via ctypes.

The binding mirrors the drop-in boundary one to one: `Problem` owns an `lba_problem*`, takes the
flat window arrays (numpy structured arrays with the dtypes of `abi`) and calls the HIP library.
There is no CPU fallback: importing works anywhere, but every call goes to libamc_lba.so and
fails loudly when the library or a GPU is missing.
"""
import ctypes
import os

import numpy as np

from . import abi as _abi
from .abi import (CAM_DTYPE, KF_DTYPE, OBS_DTYPE, PRIOR_DTYPE, LbaConfig, LbaStats, make_config,  # noqa: F401
                  ptr)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# AMC_LBA_LIB: another build of the library (kernel experiments; scripts/exp_build.sh)
LIB_PATH = os.environ.get("AMC_LBA_LIB") or os.path.join(PKG_DIR, "lib", "libamc_lba.so")

_dp = ctypes.POINTER(ctypes.c_double)
_lib = None


class LbaError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"lba error {code}: {msg}")
        self.code = code


def check_fresh(which="engine"):
    """Raise if the in-tree library is missing or was built from other sources than the ones beside it
    (build.py's content stamp): a stale binary is never loaded silently."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_amc_lba_build", os.path.join(PKG_DIR, "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    why = b.stale(which)
    if why:
        raise RuntimeError(f"{why}: run python -c 'import __graft_entry__ as g; g.build()'")


def lib_digest(path=None):
    """sha256 (first 16 hex digits) of the engine library file: profiles measured on one build carry it,
    so a summary of another build is not taken for this one's."""
    import hashlib
    with open(path or LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def lib():
    """Load libamc_lba.so (built by __graft_entry__.build()); raises if it is missing or stale."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run python -c 'import __graft_entry__ as g; g.build()'")
        if not os.environ.get("AMC_LBA_LIB"):
            check_fresh("engine")
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.lba_abi_version.restype = ctypes.c_int
        L.lba_create.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(LbaConfig)]
        L.lba_destroy.argtypes = [vp]
        L.lba_destroy.restype = None
        L.lba_last_error.argtypes = [vp]
        L.lba_last_error.restype = ctypes.c_char_p
        L.lba_pose_dim.argtypes = [vp]
        L.lba_set_problem.argtypes = [vp, vp, ctypes.c_int32, vp, ctypes.c_int32, vp, ctypes.c_int32, vp,
                                      ctypes.c_int32, vp, ctypes.c_int32, vp, ctypes.c_int32]
        L.lba_optimize.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(LbaStats)]
        L.lba_get_state.argtypes = [vp, vp, _dp]
        L.lba_set_state.argtypes = [vp, vp, _dp]
        L.lba_eval.argtypes = [vp, _dp, _dp, vp]
        L.lba_trial_chi2.argtypes = [vp, _dp]
        L.lba_linearize.argtypes = [vp, _dp, _dp, _dp, _dp]
        L.lba_solve_step.argtypes = [vp, ctypes.c_double, _dp]
        L.lba_set_config.argtypes = [vp, ctypes.POINTER(LbaConfig)]
        L.lba_set_partition.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, vp]
        L.lba_rccl_unique_id.argtypes = [ctypes.c_char_p]
        L.lba_set_partition_rccl.argtypes = [vp, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32]
        L.lba_group_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int32]
        L.lba_group_destroy.argtypes = [vp]
        L.lba_group_destroy.restype = None
        L.lba_set_partition_group.argtypes = [vp, vp, ctypes.c_int32]
        L.lba_get_cams.argtypes = [vp, vp]
        _ip = ctypes.POINTER(ctypes.c_int32)
        _lp = ctypes.POINTER(ctypes.c_int64)
        L.lba_set_farm.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, vp]
        L.lba_set_farm_rccl.argtypes = [vp, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32]
        L.lba_set_farm_group.argtypes = [vp, vp, ctypes.c_int32]
        L.lba_farm_plan.argtypes = [vp, _lp, _ip, _lp, _ip, _ip]
        L.lba_farm_exchange.argtypes = [vp]
        L.lba_solver_info.argtypes = [vp, _ip]
        if hasattr(L, "lba_trial_state"):   # (absent from builds before it: A/B runs of older libraries)
            L.lba_trial_state.argtypes = [vp, vp, _dp]
            L.lba_debug_inject_fault.argtypes = [vp, ctypes.c_int32]
        L.lba_kernel_modes.argtypes = [vp, _ip]
        if hasattr(L, "lba_debug_pool_stress"):
            L.lba_debug_pool_stress.argtypes = [ctypes.c_int32, ctypes.c_int32]
            L.lba_debug_lie.argtypes = [ctypes.c_int32, ctypes.c_int32, _dp, _dp]
        if hasattr(L, "lba_solver_flops"):   # (absent from builds before it: A/B runs of older libraries)
            L.lba_solver_flops.argtypes = [vp, _dp]
        L.lba_device_bytes.argtypes = [vp]
        L.lba_device_bytes.restype = ctypes.c_int64
        L.lba_setup_phases.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int32]
        L.lba_setup_phases.restype = ctypes.c_int32
        L.lba_setup_host_profile.argtypes = [ctypes.POINTER(LbaConfig), vp, ctypes.c_int32, vp, ctypes.c_int32, vp,
                                             ctypes.c_int32, vp, ctypes.c_int32, vp, ctypes.c_int32, vp, ctypes.c_int32,
                                             _dp, _ip]
        L.lba_farm_match.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _lp, _lp, _ip, ctypes.c_int32, _ip]
        if hasattr(L, "lba_partition_assign"):   # (absent from builds before it: A/B runs of older libraries)
            L.lba_partition_assign.argtypes = [ctypes.POINTER(LbaConfig), vp, ctypes.c_int32, ctypes.c_int32, vp,
                                               ctypes.c_int32, vp, ctypes.c_int32, vp, ctypes.c_int32, ctypes.c_int32,
                                               _ip, _ip, _ip, _ip, _ip]
            L.lba_kf_owner.argtypes = [vp, _ip]
            L.lba_split_info.argtypes = [vp, _dp]
        _lib = L
    return _lib


def exported_symbols():
    return ["lba_abi_version", "lba_live_problems", "lba_create", "lba_destroy", "lba_last_error", "lba_set_config", "lba_set_problem",
            "lba_optimize", "lba_get_state", "lba_set_state", "lba_eval", "lba_trial_chi2", "lba_linearize", "lba_solve_step",
            "lba_pose_dim", "lba_set_partition", "lba_rccl_unique_id", "lba_set_partition_rccl", "lba_group_create",
            "lba_group_destroy", "lba_set_partition_group", "lba_get_cams", "lba_set_farm", "lba_set_farm_rccl",
            "lba_set_farm_group", "lba_farm_plan", "lba_farm_exchange", "lba_farm_match", "lba_solver_info", "lba_solver_flops", "lba_device_bytes", "lba_setup_phases",
            "lba_kernel_modes", "lba_setup_host_profile", "lba_debug_pool_stress", "lba_debug_lie", "lba_partition_assign", "lba_kf_owner", "lba_split_info"]


def setup_host_profile(win, **cfg_over):
    """lba_setup_host_profile: the host preprocessing of lba_set_problem on the CPU (no GPU).  Returns
    (phase ms [order/pairs, tiles, slots/state], counts [device landmarks, pose blocks, np, tiles, layout hash])."""
    kw = dict(win.cfg)
    kw.update(cfg_over)
    cfg = make_config(**kw)
    kfs = np.ascontiguousarray(win.kfs, dtype=KF_DTYPE)
    lm = np.ascontiguousarray(win.lm, dtype=np.float64)
    obs = np.ascontiguousarray(win.obs, dtype=OBS_DTYPE)
    pri = np.ascontiguousarray(win.priors, dtype=PRIOR_DTYPE)
    vel = np.ascontiguousarray(win.vel_kfs, dtype=np.int32)
    cams = np.ascontiguousarray(win.cams, dtype=CAM_DTYPE)
    ms = np.zeros(3)
    cnt = np.zeros(5, dtype=np.int32)
    rc = lib().lba_setup_host_profile(ctypes.byref(cfg), ptr(kfs), len(kfs), ptr(lm), len(lm), ptr(obs), len(obs),
                                      ptr(pri), len(pri), ptr(vel), len(vel), ptr(cams), len(cams), _d(ms),
                                      cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    if rc != 0:
        raise LbaError(rc, "lba_setup_host_profile failed")
    return ms, cnt


def debug_lie(xi, q=None, t=None, device=0):
    """lba_debug_lie: the kernels' se3 exp / log and right Jacobians (and inverse) evaluated on the GPU.  xi: (n, 6)
    tangents, (q, t): (n, 4) / (n, 3) poses to take the log of (default: exp(xi) is not needed, identity).
    Returns dict(q, t, log, Jr, Jr_inv)."""
    xi = np.atleast_2d(np.asarray(xi, dtype=np.float64))
    n = len(xi)
    inp = np.zeros((n, 13))
    inp[:, :6] = xi
    inp[:, 6:10] = [0, 0, 0, 1] if q is None else np.atleast_2d(q)
    inp[:, 10:13] = 0 if t is None else np.atleast_2d(t)
    out = np.zeros((n, 85))
    rc = lib().lba_debug_lie(device, n, _d(np.ascontiguousarray(inp)), _d(out))
    if rc != 0:
        raise LbaError(rc, "lba_debug_lie failed")
    return {"q": out[:, 0:4], "t": out[:, 4:7], "log": out[:, 7:13], "Jr": out[:, 13:49].reshape(n, 6, 6),
            "Jr_inv": out[:, 49:85].reshape(n, 6, 6)}


def partition_assign(win, nranks, kf=False, **cfg_over):
    """lba_partition_assign (host only): the landmark / motion-prior / velocity-edge split of `win` for the
    distributed factorisation (LBA_FLAG_SUBTREE_SOLVE).  Returns (lm_rank, prior_rank, vel_rank, panels) with
    panels = [panels of the system, panels in the top, columns of the largest subtree]; with kf=True also the
    keyframes' ranks (-1: the top or fixed)."""
    if np.any(np.asarray(win.cams["ext_free"]) != 0):
        # (the C call sees no cameras and plans the keyframe-only pattern; a partitioned set-up rejects free extrinsics)
        raise LbaError(_abi.LBA_E_LIMIT, "partition_assign: free extrinsics (lba_cam.ext_free) are not supported in a "
                                    "partitioned problem")
    kw = dict(win.cfg)
    kw.update(cfg_over)
    cfg = make_config(**kw)
    kfs = np.ascontiguousarray(win.kfs, dtype=KF_DTYPE)
    obs = np.ascontiguousarray(win.obs, dtype=OBS_DTYPE)
    pri = np.ascontiguousarray(win.priors, dtype=PRIOR_DTYPE)
    vel = np.ascontiguousarray(win.vel_kfs, dtype=np.int32)
    out = [np.zeros(max(n, 1), np.int32) for n in (len(win.lm), len(pri), len(vel))]
    panels = np.zeros(3, np.int32)
    kfr = np.zeros(max(len(kfs), 1), np.int32)
    ip = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))   # noqa: E731
    rc = lib().lba_partition_assign(ctypes.byref(cfg), ptr(kfs), len(kfs), len(win.lm), ptr(obs), len(obs), ptr(pri),
                                    len(pri), ptr(vel), len(vel), nranks, ip(out[0]), ip(out[1]), ip(out[2]), ip(panels),
                                    ip(kfr))
    if rc != 0:
        raise LbaError(rc, "lba_partition_assign failed")
    res = (out[0][:len(win.lm)], out[1][:len(pri)], out[2][:len(vel)], panels)
    return res + (kfr[:len(kfs)],) if kf else res


def _i32(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def _i64(a):
    a = np.ascontiguousarray(a, dtype=np.int64)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


def farm_match(rank, nranks, cap, pub_gid, gid, owner):
    """lba_farm_match (host only): source slot owner * cap + position of every received vertex, -1 for
    the rest; returns (src, unmatched)."""
    pg, pgp = _i64(np.asarray(pub_gid).reshape(-1))
    g, gp = _i64(gid)
    o, op = _i32(owner)
    src = np.full(len(g), -1, dtype=np.int32)
    rc = lib().lba_farm_match(rank, nranks, cap, pgp, gp, op, len(g), src.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    if rc < 0:
        raise LbaError(rc, "lba_farm_match failed")
    return src, rc


class Group:
    """In-process all-reduce group of `n` problems on one device (lba_group): the partitioned global
    BA of several ranks driven from threads of one process (tests, single-GPU rehearsal)."""

    def __init__(self, n):
        self.h = ctypes.c_void_p()
        rc = lib().lba_group_create(ctypes.byref(self.h), n)
        if rc != 0:
            raise LbaError(rc, "lba_group_create failed")
        self.n = n

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().lba_group_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        self.close()


def rccl_unique_id():
    """128-byte RCCL unique id (one rank creates it, the caller shares it, e.g. via torch.distributed)."""
    buf = ctypes.create_string_buffer(128)
    rc = lib().lba_rccl_unique_id(buf)
    if rc != 0:
        raise LbaError(rc, "lba_rccl_unique_id failed")
    return buf.raw


def _d(a):
    return None if a is None else a.ctypes.data_as(_dp)


class Problem:
    """One local-BA window resident on one GPU (lba_create + lba_set_problem)."""

    def __init__(self, win, cfg=None, device=0, group=None, rank=0, rccl_id=None, nranks=1, **cfg_over):
        """group / rank: partitioned problem in an in-process Group; rccl_id / rank / nranks: partitioned
        across processes over RCCL.  Construction is then collective (set_problem agrees on the
        union envelope), so the ranks' constructors must run concurrently."""
        L = lib()
        if cfg is None:
            kw = dict(win.cfg)
            kw.update(cfg_over)
            kw.setdefault("device", device)
            cfg = make_config(**kw)
        self.cfg = cfg
        self.h = ctypes.c_void_p()
        self._check(L.lba_create(ctypes.byref(self.h), ctypes.byref(cfg)), created=False)
        self.win = win
        self.n_obs, self.n_lm, self.n_kf = len(win.obs), len(win.lm), len(win.kfs)
        self._keep = tuple(np.ascontiguousarray(a) for a in (win.kfs, win.lm, win.obs, win.priors, win.vel_kfs,
                                                              win.cams))
        kfs, lm, obs, pri, vel, cams = self._keep
        self.group = group
        if group is not None:
            self._check(L.lba_set_partition_group(self.h, group.h, rank))
        elif rccl_id is not None and nranks > 1:
            self._check(L.lba_set_partition_rccl(self.h, rccl_id, rank, nranks))
        self._check(L.lba_set_problem(self.h, ptr(kfs), len(kfs), ptr(lm), len(lm), ptr(obs), len(obs), ptr(pri),
                                      len(pri), ptr(vel), len(vel), ptr(cams), len(cams)))

    def set_window(self, win):
        """lba_set_problem with another window on the same engine (its device buffers and plan cache reused), as the
        mapping thread's one problem per thread does; unpartitioned problems only."""
        if self.group is not None:
            raise ValueError("set_window: partitioned problems are set up collectively")
        kw = dict(win.cfg)
        kw.setdefault("device", self.cfg.device)
        cfg = make_config(**kw)   # the window's own configuration, as the adapter sets it per call (lba_set_config)
        self._check(lib().lba_set_config(self.h, ctypes.byref(cfg)))
        self.cfg = cfg
        keep =tuple(np.ascontiguousarray(a) for a in (win.kfs, win.lm, win.obs, win.priors, win.vel_kfs, win.cams))
        kfs, lm, obs, pri, vel, cams = keep
        self._check(lib().lba_set_problem(self.h, ptr(kfs), len(kfs), ptr(lm), len(lm), ptr(obs), len(obs), ptr(pri),
                                          len(pri), ptr(vel), len(vel), ptr(cams), len(cams)))
        self.win, self._keep = win, keep
        self.n_obs, self.n_lm, self.n_kf = len(win.obs), len(win.lm), len(win.kfs)

    def _check(self, rc, created=True):
        if rc < 0:
            msg = lib().lba_last_error(self.h).decode() if created and self.h else "lba_create failed"
            raise LbaError(rc, msg)
        return rc

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().lba_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        self.close()

    @property
    def pose_dim(self):
        return lib().lba_pose_dim(self.h)

    @property
    def lm_dim(self):
        return 3 * int(np.unique(self.win.obs["lm"]).size)

    def optimize(self, iters, stop_flag=None):
        st = LbaStats()
        flag = None if stop_flag is None else ctypes.byref(stop_flag)
        n = self._check(lib().lba_optimize(self.h, iters, flag, ctypes.byref(st)))
        return n, st

    def state(self):
        kfs = np.zeros(self.n_kf, KF_DTYPE)
        lm = np.zeros((self.n_lm, 3))
        self._check(lib().lba_get_state(self.h, ptr(kfs), _d(lm)))
        return kfs, lm

    def cams(self):
        """Camera records with the current extrinsic estimates (lba_get_cams)."""
        c = np.zeros(len(self.win.cams), CAM_DTYPE)
        self._check(lib().lba_get_cams(self.h, ptr(c)))
        return c

    # ---- window farm (lba_set_farm_*, lba_farm_plan, lba_farm_exchange)
    def set_farm_group(self, group, rank):
        self._check(lib().lba_set_farm_group(self.h, group.h, rank))

    def set_farm_rccl(self, rccl_id, rank, nranks):
        self._check(lib().lba_set_farm_rccl(self.h, rccl_id, rank, nranks))

    def farm_plan(self, kf_gid, kf_owner, lm_gid, lm_owner):
        """Collective: returns (kf published, lm published, kf received, lm received, unmatched)."""
        kg, kgp = _i64(kf_gid)
        ko, kop = _i32(kf_owner)
        lg, lgp = _i64(lm_gid)
        lo, lop = _i32(lm_owner)
        out = np.zeros(5, dtype=np.int32)
        self._check(lib().lba_farm_plan(self.h, kgp, kop, lgp, lop, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return tuple(int(v) for v in out)

    def kf_owner(self):
        """lba_kf_owner: per keyframe, the rank whose subtree holds it in the distributed factorisation (-1: all)."""
        out = np.zeros(max(self.n_kf, 1), np.int32)
        self._check(lib().lba_kf_owner(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return out[:self.n_kf]

    def split_info(self):
        """lba_split_info: dict(rank_flops, system_flops, allreduce_bytes, replicated_allreduce_bytes, own_panels,
        top_panels)."""
        out = np.zeros(6)
        self._check(lib().lba_split_info(self.h, _d(out)))
        return dict(zip(("rank_flops", "system_flops", "allreduce_bytes", "replicated_allreduce_bytes",
                         "own_panels", "top_panels"), out.tolist()))

    def solver_info(self):
        """lba_solver_info: dict(tail, panels, tiles (of L, fill-in included), band, chain, levels, s_tiles
        (the pattern of S), fill (tiles of L that are zero in S))."""
        out = np.zeros(8, dtype=np.int32)
        self._check(lib().lba_solver_info(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return dict(zip(("tail", "panels", "tiles", "band", "chain", "levels", "s_tiles", "fill"),
                        (int(v) for v in out)))

    def kernel_modes(self):
        """lba_kernel_modes: dict(fuse_eval, fuse_asm, f32res, update_grid)."""
        out = np.zeros(4, dtype=np.int32)
        self._check(lib().lba_kernel_modes(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return dict(zip(("fuse_eval", "fuse_asm", "f32res", "update_grid"), (int(v) for v in out)))

    def solver_flops(self):
        """lba_solver_flops: (factorisation, substitutions) algorithmic FLOPs of one solve."""
        out = np.zeros(2, dtype=np.float64)
        self._check(lib().lba_solver_flops(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        return float(out[0]), float(out[1])

    SETUP_PHASES = ("order_pairs", "tiles", "slots_state", "upload", "solve_layout")

    def setup_phases(self):
        """lba_setup_phases: {phase: ms} of the last set-up."""
        out = np.zeros(8)
        k = lib().lba_setup_phases(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 8)
        self._check(min(k, 0))
        return dict(zip(self.SETUP_PHASES, out[:k].tolist()))

    def device_bytes(self):
        """lba_device_bytes: device memory held by the problem's buffers."""
        return int(lib().lba_device_bytes(self.h))

    def farm_exchange(self):
        self._check(lib().lba_farm_exchange(self.h))

    def trial_state(self):
        """lba_trial_state: the last solve_step's trial estimate (the device's x (+) dx), the current one unchanged."""
        kfs = np.zeros(self.n_kf, KF_DTYPE)
        lm = np.zeros((self.n_lm, 3))
        self._check(lib().lba_trial_state(self.h, ptr(kfs), _d(lm)))
        return kfs, lm

    def inject_fault(self, code):
        """lba_debug_inject_fault: set the device fault word as a timed-out in-launch wait does."""
        self._check(lib().lba_debug_inject_fault(self.h, int(code)))

    def set_state(self, kfs=None, lm=None):
        kfs = None if kfs is None else np.ascontiguousarray(kfs, dtype=KF_DTYPE)
        lm = None if lm is None else np.ascontiguousarray(lm, dtype=np.float64)
        self._check(lib().lba_set_state(self.h, ptr(kfs), _d(lm)))

    def eval(self):
        chi = ctypes.c_double()
        c2 = np.zeros(self.n_obs)
        ok = np.zeros(self.n_obs, np.uint8)
        self._check(lib().lba_eval(self.h, ctypes.byref(chi), _d(c2), ptr(ok)))
        return chi.value, c2, ok

    def trial_chi2(self):
        """Per-observation chi2 of the last computed errors (after optimize: its last trial state,
        g2o's e->chi2()), nothing re-evaluated (lba_trial_chi2)."""
        c2 = np.zeros(self.n_obs)
        self._check(lib().lba_trial_chi2(self.h, _d(c2)))
        return c2

    def linearize(self, dense=True):
        """(residuals, H_pp dense, b, H_ll); dense=False: no H_pp (None), for pose systems whose dense H_pp
        would not fit (config 4)."""
        np_ = self.pose_dim
        H = np.zeros((np_, np_)) if dense else None
        b = np.zeros(np_ + self.lm_dim)
        Hll = np.zeros((self.n_lm, 9))
        res = np.zeros((self.n_obs, 3))
        self._check(lib().lba_linearize(self.h, _d(res), _d(H), _d(b), _d(Hll)))
        return res, H, b, Hll

    def solve_step(self, lam):
        dx = np.zeros(self.pose_dim + self.lm_dim)
        rc = lib().lba_solve_step(self.h, lam, _d(dx))
        if rc == -2:
            return False, dx
        self._check(rc)
        return True, dx
