"""Tracking-side pose optimisation (Optimizer::PoseGPOptimizationFromeLastFrame, src/Optimizer.cc:369-686)
through the C ABI (lba_tracker_*, lba_track): a batch of frames, one GPU workgroup each, one launch.

`make_track_frames` cuts synthetic tracking problems out of a local-BA window: frame k's
observations (the asynchronous cameras' GP edges between k-1 and k, the reference camera's mono /
stereo edges) against fixed map points, the previous frame fixed or free.
"""
import ctypes

import numpy as np

from . import LbaError, lib
from .abi import CAM_DTYPE, KF_DTYPE, MONO, MONO_GP, STEREO, LbaConfig, make_config, ptr

TRACK_OBS_DTYPE = np.dtype([
    ("kind", "<i4"), ("cam", "<i4"), ("outlier", "<i4"), ("close", "<i4"),
    ("t", "<f8"), ("z", "<f8", (3,)), ("w", "<f8"), ("Xw", "<f8", (3,)),
], align=True)
TRACK_FRAME_DTYPE = np.dtype([
    ("prev", KF_DTYPE), ("cur", KF_DTYPE), ("obs0", "<i4"), ("n_obs", "<i4"), ("n_good", "<i4"),
    ("iterations", "<i4"),
], align=True)
assert TRACK_OBS_DTYPE.itemsize == 80
assert TRACK_FRAME_DTYPE.itemsize == 272


def _bind():
    L = lib()
    if not getattr(L, "_track_bound", False):
        vp = ctypes.c_void_p
        L.lba_tracker_create.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(LbaConfig)]
        L.lba_tracker_destroy.argtypes = [vp]
        L.lba_tracker_destroy.restype = None
        L.lba_track.argtypes = [vp, vp, ctypes.c_int32, vp, ctypes.c_int32, vp, ctypes.c_int32]
        L._track_bound = True
    return L


def track_config(**over):
    """The reference's tracking optimiser: Huber deltas as LocalGPBA, no user lambda
    (computeLambdaInit, src/Optimizer.cc:379-381), g2o stop rules."""
    kw = dict(lambda_init=0.0)
    kw.update(over)
    return make_config(**kw)


class Tracker:
    def __init__(self, cfg=None, device=0, **over):
        L = _bind()
        self.cfg = cfg if cfg is not None else track_config(device=device, **over)
        self.h = ctypes.c_void_p()
        rc = L.lba_tracker_create(ctypes.byref(self.h), ctypes.byref(self.cfg))
        if rc != 0:
            raise LbaError(rc, "lba_tracker_create failed")

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            _bind().lba_tracker_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        self.close()

    def track(self, frames, obs, cams):
        """Optimises the frames in place (cur, n_good, iterations) and the observations' outlier flags."""
        frames = np.ascontiguousarray(frames, TRACK_FRAME_DTYPE)
        obs = np.ascontiguousarray(obs, TRACK_OBS_DTYPE)
        cams = np.ascontiguousarray(cams, CAM_DTYPE)
        rc = _bind().lba_track(self.h, ptr(frames), len(frames), ptr(obs), len(obs), ptr(cams), len(cams))
        if rc != 0:
            raise LbaError(rc, "lba_track failed")
        return frames, obs


def make_track_frames(win, ks, fix_prev=True, outlier_init=0.05, close_frac=0.2, seed=0, point_noise=0.02,
                      sigma_t=0.03, sigma_r=0.3, sigma_v=0.05):
    """One tracking problem per KF index k in `ks` of an unperturbed window `win`
    (make_window(..., perturb=False)), k >= 1: prev = KF k-1 at its true state, cur = KF k with its
    pose / velocity perturbed (the motion-model prediction the tracker starts from), the observations
    of KF k with their points fixed at the true positions plus `point_noise` (m), rounded to float like
    GetWorldPos()."""
    from .synth import _expso3, quat_to_rot, rot_to_quat
    rng = np.random.default_rng(seed)
    o = win.obs
    frames = np.zeros(len(ks), TRACK_FRAME_DTYPE)
    rows = []
    for f, k in enumerate(ks):
        sel = np.nonzero(o["kf_b"] == k)[0]
        frames[f]["prev"] = win.kfs[k - 1]
        frames[f]["prev"]["fixed"] = int(fix_prev)
        frames[f]["cur"] = win.kfs[k]
        frames[f]["cur"]["fixed"] = 0
        R = quat_to_rot(win.kfs[k]["q"]) @ _expso3(rng.normal(0, np.deg2rad(sigma_r), 3))
        frames[f]["cur"]["q"] = rot_to_quat(R).astype(np.float32)
        frames[f]["cur"]["t"] = (win.kfs[k]["t"] + rng.normal(0, sigma_t, 3)).astype(np.float32)
        frames[f]["cur"]["vel"] = (win.kfs[k]["vel"] + rng.normal(0, sigma_v, 6)).astype(np.float32)
        frames[f]["obs0"] = len(rows)
        frames[f]["n_obs"] = sel.size
        for i in sel:
            rows.append(i)
    rows = np.array(rows, np.int64)
    obs = np.zeros(rows.size, TRACK_OBS_DTYPE)
    src = o[rows]
    kind = src["kind"].copy()
    kind[kind == 1] = MONO_GP   # (no stereo GP edge in the tracking graph)
    obs["kind"] = kind
    obs["cam"] = src["cam"]
    obs["t"] = src["t"]
    obs["z"] = src["z"]
    obs["w"] = src["w"]
    X = win.truth_lm[src["lm"]] + rng.normal(0, point_noise, (rows.size, 3))
    obs["Xw"] = X.astype(np.float32).astype(np.float64)
    obs["outlier"] = rng.random(rows.size) < outlier_init
    obs["close"] = rng.random(rows.size) < close_frac
    return frames, obs
