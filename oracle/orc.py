"""ctypes binding of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker / reported CPU baseline.  The product (amc-slam_amd) never loads it.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORC_LIB: another build of the oracle (bench.py's OpenMP CPU baseline loads _build/liblba_oracle_omp.so)
LIB = os.environ.get("ORC_LIB") or os.path.join(HERE, "_build", "liblba_oracle.so")
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "amc-slam_amd"))

from amc_lba.abi import LbaStats, make_config, ptr  # noqa: E402

_dp = ctypes.POINTER(ctypes.c_double)


def build(force=False):
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(
            os.path.getmtime(os.path.join(HERE, f)) for f in ("lba_oracle.c", "lba_oracle.h")):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB


_lib = None
_lib_omp = None
LIB_OMP = os.path.join(HERE, "_build", "liblba_oracle_omp.so")


def lib(omp=False):
    """The oracle library; omp=True: its OpenMP build (bitwise the serial build's results, the per-edge passes
    on OMP_NUM_THREADS threads), loaded beside it for the full-size checks."""
    global _lib, _lib_omp
    if omp:
        if _lib_omp is None:
            build()
            _lib_omp = _bind(ctypes.CDLL(LIB_OMP))
        return _lib_omp
    if _lib is None:
        build()
        _lib = _bind(ctypes.CDLL(LIB))
    return _lib


def _bind(L):
    L.orc_create.restype = ctypes.c_void_p
    L.orc_create.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p, ctypes.c_int] * 6
    L.orc_destroy.argtypes = [ctypes.c_void_p]
    L.orc_pose_dim.argtypes = [ctypes.c_void_p]
    L.orc_lm_dim.argtypes = [ctypes.c_void_p]
    L.orc_compute_errors.restype = ctypes.c_double
    L.orc_compute_errors.argtypes = [ctypes.c_void_p, _dp, _dp]
    L.orc_build_system.argtypes = [ctypes.c_void_p, _dp, _dp, _dp]
    L.orc_solve.argtypes = [ctypes.c_void_p, ctypes.c_double, _dp]
    L.orc_normal_residual.argtypes = [ctypes.c_void_p, ctypes.c_double, _dp, _dp]
    L.orc_normal_residual.restype = None
    L.orc_normal_residual_abs.argtypes = [ctypes.c_void_p, ctypes.c_double, _dp, _dp]
    L.orc_normal_residual_abs.restype = None
    L.orc_optimize.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(LbaStats)]
    L.orc_get_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _dp]
    L.orc_set_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _dp]
    L.orc_set_state.restype = None
    L.orc_apply_step.argtypes = [ctypes.c_void_p, _dp]
    L.orc_apply_step.restype = None
    L.orc_get_cams.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.orc_depth_ok.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.orc_last_obs_chi2.argtypes = [ctypes.c_void_p, _dp]
    L.orc_last_obs_chi2.restype = None
    L.orc_obs_linearize.argtypes = [ctypes.c_void_p, ctypes.c_int, _dp, _dp]
    L.orc_prior_linearize.argtypes = [ctypes.c_void_p, ctypes.c_int, _dp, _dp, _dp]
    for n in ("orc_se3_exp", "orc_se3_log", "orc_so3_exp", "orc_so3_log", "orc_right_jac_pose3",
              "orc_right_jac_pose3_inv", "orc_left_jac_pose3_q", "orc_gp_query_pose"):
        getattr(L, n).restype = None
    L.orc_ldlt_solve.argtypes = [ctypes.c_int, _dp, _dp, _dp]
    return L


def _d(a):
    return a.ctypes.data_as(_dp)


class Oracle:
    """g2o-semantics CPU restatement of LocalGPBA's optimisation on one window."""

    def __init__(self, win, cfg=None, omp=False, **cfg_over):
        self._omp = omp
        L = self._L = lib(omp)
        if cfg is None:
            kw = dict(win.cfg)
            kw.update(cfg_over)
            cfg = make_config(**kw)
        self.cfg = cfg
        self.win = win
        self.n_obs = len(win.obs)
        self.n_lm = len(win.lm)
        self.n_kf = len(win.kfs)
        self._keep = (win.kfs, win.lm, win.obs, win.priors, win.vel_kfs, win.cams)
        self.h = L.orc_create(ctypes.byref(cfg), ptr(win.kfs), len(win.kfs), ptr(win.lm), len(win.lm),
                              ptr(win.obs), len(win.obs), ptr(win.priors), len(win.priors),
                              ptr(win.vel_kfs), len(win.vel_kfs), ptr(win.cams), len(win.cams))

    def __del__(self):
        if getattr(self, "h", None):
            self._L.orc_destroy(self.h)
            self.h = None

    @property
    def pose_dim(self):
        return self._L.orc_pose_dim(self.h)

    @property
    def lm_dim(self):
        return self._L.orc_lm_dim(self.h)

    def errors(self):
        res = np.zeros((self.n_obs, 3))
        c2 = np.zeros(self.n_obs)
        chi = self._L.orc_compute_errors(self.h, _d(res), _d(c2))
        return chi, res, c2

    def build_system(self, dense=True):
        """(H_pp dense, b, H_ll); dense=False: H_pp only as the oracle's blocks (None returned), for systems
        whose dense H_pp would not fit (config 4: 59988^2)."""
        np_ = self.pose_dim
        H = np.zeros((np_, np_)) if dense else None
        b = np.zeros(np_ + self.lm_dim)
        Hll = np.zeros((self.n_lm, 9))
        self._L.orc_build_system(self.h, _d(H) if dense else None, _d(b), _d(Hll))
        return H, b, Hll

    def solve(self, lam):
        dx = np.zeros(self.pose_dim + self.lm_dim)
        ok = self._L.orc_solve(self.h, lam, _d(dx))
        return bool(ok), dx

    def normal_residual(self, lam, dx):
        """(H + lam I) dx - b on the last build_system (size-independent step check)."""
        dx = np.ascontiguousarray(dx, float)
        r = np.zeros(self.pose_dim + self.lm_dim)
        self._L.orc_normal_residual(self.h, lam, _d(dx), _d(r))
        return r

    def backward_error(self, lam, dx):
        """Backward errors of a step on the last build_system, with r = (H + lam I) dx - b and A = H + lam I:
        normwise |r|_inf / (|A|_inf |dx|_inf + |b|_inf) (near n eps for a backward-stable solve at any conditioning)
        and componentwise max_i |r_i| / (|A| |dx| + |b|)_i (Oettli-Prager; the Schur-complement solve does not bound
        it).  Returns (normwise, componentwise, r)."""
        dx = np.ascontiguousarray(dx, float)
        n = self.pose_dim + self.lm_dim
        d = np.zeros(n)
        self._L.orc_normal_residual_abs(self.h, lam, _d(dx), _d(d))
        r = self.normal_residual(lam, dx)
        ones = np.ones(n)
        rows = np.zeros(n)
        self._L.orc_normal_residual_abs(self.h, lam, _d(ones), _d(rows))
        absb = np.abs(self.normal_residual(lam, np.zeros(n)))   # |b| (r at dx = 0 is -b)
        a_inf = float(np.max(rows - absb))                       # max row sum of |A|
        eta = float(np.abs(r).max() / (a_inf * np.abs(dx).max() + absb.max()))
        omega = float(np.max(np.abs(r) / np.maximum(d, 1e-300)))
        return eta, omega, r

    def optimize(self, iters):
        st = LbaStats()
        n = self._L.orc_optimize(self.h, iters, ctypes.byref(st))
        return n, st

    def cams(self):
        c = np.array(self.win.cams, copy=True)
        self._L.orc_get_cams(self.h, ptr(c))
        return c

    def state(self):
        from amc_lba.abi import KF_DTYPE
        kfs = np.zeros(self.n_kf, KF_DTYPE)
        lm = np.zeros((self.n_lm, 3))
        self._L.orc_get_state(self.h, ptr(kfs), _d(lm))
        return kfs, lm

    def set_state(self, kfs, lm):
        """Overwrite the estimates (keyframe q / t / velocity, landmarks); a caller-driven LM's linearisation point."""
        kfs = np.ascontiguousarray(kfs)
        lm = np.ascontiguousarray(lm, float)
        self._L.orc_set_state(self.h, ptr(kfs), _d(lm))

    def apply_step(self, dx):
        """x <- x (+) dx (SparseOptimizer::update's oplus) for a step [pose_dim + lm_dim]."""
        dx = np.ascontiguousarray(dx, float)
        assert dx.shape == (self.pose_dim + self.lm_dim,)
        self._L.orc_apply_step(self.h, _d(dx))

    def last_obs_chi2(self):
        """chi2 of the last computed errors (after optimize: the last trial state), nothing recomputed."""
        c2 = np.zeros(self.n_obs)
        self._L.orc_last_obs_chi2(self.h, _d(c2))
        return c2

    def depth_ok(self):
        ok = np.zeros(self.n_obs, np.uint8)
        self._L.orc_depth_ok(self.h, ptr(ok))
        return ok

    def obs_linearize(self, i):
        e = np.zeros(3)
        J = np.zeros((3, 27))
        d = self._L.orc_obs_linearize(self.h, i, _d(e), _d(J))
        return e[:d], J[:d]

    def prior_linearize(self, i):
        e = np.zeros(12)
        Ji = np.zeros((12, 12))
        Jj = np.zeros((12, 12))
        self._L.orc_prior_linearize(self.h, i, _d(e), _d(Ji), _d(Jj))
        return e, Ji, Jj


# ---------------------------------------------------------------- primitives
def se3_exp(xi):
    q, t = np.zeros(4), np.zeros(3)
    lib().orc_se3_exp(_d(np.ascontiguousarray(xi, float)), _d(q), _d(t))
    return q, t


def se3_log(q, t):
    xi = np.zeros(6)
    lib().orc_se3_log(_d(np.ascontiguousarray(q, float)), _d(np.ascontiguousarray(t, float)), _d(xi))
    return xi


def so3_exp(w):
    q = np.zeros(4)
    lib().orc_so3_exp(_d(np.ascontiguousarray(w, float)), _d(q))
    return q


def so3_log(q):
    w = np.zeros(3)
    lib().orc_so3_log(_d(np.ascontiguousarray(q, float)), _d(w))
    return w


def right_jac_pose3(xi):
    J = np.zeros(36)
    lib().orc_right_jac_pose3(_d(np.ascontiguousarray(xi, float)), _d(J))
    return J.reshape(6, 6)


def right_jac_pose3_inv(xi):
    J = np.zeros(36)
    lib().orc_right_jac_pose3_inv(_d(np.ascontiguousarray(xi, float)), _d(J))
    return J.reshape(6, 6)


def left_jac_pose3_q(xi):
    Q = np.zeros(9)
    lib().orc_left_jac_pose3_q(_d(np.ascontiguousarray(xi, float)), _d(Q))
    return Q.reshape(3, 3)


def gp_query_pose(qc, q1, t1, q2, t2, v1, v2, time1, time2, t):
    outs = [np.zeros(4), np.zeros(3), np.zeros(72), np.zeros(72), np.zeros(4), np.zeros(3), np.zeros(6)]
    ins = [np.ascontiguousarray(a, float) for a in (qc, q1, t1, q2, t2, v1, v2)]
    lib().orc_gp_query_pose(*[_d(a) for a in ins], ctypes.c_double(time1), ctypes.c_double(time2),
                            ctypes.c_double(t), *[_d(a) for a in outs])
    qo, to, At1, Pt1, dq, dt, xi12 = outs
    return qo, to, At1.reshape(6, 12), Pt1.reshape(6, 12), dq, dt, xi12


def ldlt_solve(A, b):
    A = np.ascontiguousarray(A, float)
    b = np.ascontiguousarray(b, float)
    x = np.zeros_like(b)
    ok = lib().orc_ldlt_solve(len(b), _d(A), _d(b), _d(x))
    return bool(ok), x


def track_pose(cfg, frame, obs, cams):
    """orc_track_pose on one frame (a 1-element TRACK_FRAME_DTYPE array) and its observations;
    both arrays are updated in place.  Returns n_good."""
    L = lib()
    L.orc_track_pose.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] + [ctypes.c_void_p, ctypes.c_int]
    return L.orc_track_pose(ctypes.byref(cfg), ptr(frame), ptr(obs), len(obs), ptr(cams), len(cams))

