"""Window snapshots (include/amc_lba_map.h) and the ctypes binding of the LocalGPBA host adapter.

A snapshot is the slice of an AMC-SLAM map that `Optimizer::LocalGPBA` (src/Optimizer.cc:713-1432)
reads and writes: keyframes with their keypoints, temporal links and covisibility order, map points
with their keyframe observations (MapPoint::mObservations) and non-keyframe GP observations
(MapPoint::mObservationsForGPBA), the cameras and the GP Qc.  `pack` / `unpack` convert between
numpy record arrays and the byte layout; `make_map` builds a deterministic synthetic map from the
local-BA generator (amc_lba/synth.py); `LocalGPBAMap` loads a snapshot into
libamc_lba_map.so and calls LocalGPBA on it (GPU) or only builds its window (no GPU).
"""
import ctypes
import os
from dataclasses import dataclass

import numpy as np

from .abi import CAM_DTYPE, KF_DTYPE, MONO, MONO_GP, OBS_DTYPE, PRIOR_DTYPE, STEREO, LbaConfig, ptr
from .synth import Window, _Trajectory, make_window, quat_to_rot

MAX_CAM = 8
MAX_LEVEL = 16
F32 = np.float32

HEADER_DTYPE = np.dtype([
    ("magic", "S8"), ("version", "<i4"), ("n_cam", "<i4"), ("n_kf", "<i4"), ("n_kp", "<i4"), ("n_covis", "<i4"),
    ("n_mp", "<i4"), ("n_mpobs", "<i4"), ("n_gpobs", "<i4"), ("n_levels", "<i4"), ("pad", "<i4"),
    ("qc", "<f8", (36,)), ("inv_level_sigma2", "<f4", (MAX_LEVEL,)), ("scale_factor", "<f4", (MAX_LEVEL,)),
], align=True)
MCAM_DTYPE = np.dtype([("q", "<f4", (4,)), ("t", "<f4", (3,)), ("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"),
                       ("cy", "<f4"), ("rbc_ini", "<f4", (4,)), ("pad", "<f4")], align=True)
MKF_DTYPE = np.dtype([
    ("id", "<i8"), ("prev_id", "<i8"), ("next_id", "<i8"), ("time", "<f8"), ("cam_time", "<f8", (MAX_CAM,)),
    ("q", "<f4", (4,)), ("t", "<f4", (3,)), ("vel", "<f4", (6,)), ("bf", "<f4"), ("bad", "<i4"), ("map_id", "<i4"),
    ("kp_off", "<i4"), ("n_kp", "<i4"), ("covis_off", "<i4"), ("n_covis", "<i4"), ("has_twc", "<i4"),
    ("twc_q", "<f4", (MAX_CAM, 4)), ("twc_t", "<f4", (MAX_CAM, 3)),
], align=True)
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("octave", "<i4"), ("cam", "<i4"), ("ur", "<f4"), ("pad", "<i4"),
                     ("mp_id", "<i8")], align=True)
MP_DTYPE = np.dtype([
    ("id", "<i8"), ("pos", "<f4", (3,)), ("bad", "<i4"), ("ref_kf", "<i8"), ("track_depth", "<f4", (MAX_CAM,)),
    ("normal", "<f4", (3,)), ("min_dist", "<f4"), ("max_dist", "<f4"), ("obs_off", "<i4"), ("n_obs", "<i4"),
    ("gp_off", "<i4"), ("n_gp", "<i4"), ("pad", "<i4"),
], align=True)
MPOBS_DTYPE = np.dtype([("kf_id", "<i8"), ("idx", "<i4", (MAX_CAM,))], align=True)
GPOBS_DTYPE = np.dtype([("kf_id", "<i8"), ("time", "<f8"), ("cam", "<i4"), ("x", "<f4"), ("y", "<f4"),
                        ("octave", "<i4"), ("ur", "<f4"), ("pad", "<i4")], align=True)

assert HEADER_DTYPE.itemsize == 464
assert MCAM_DTYPE.itemsize == 64
assert MKF_DTYPE.itemsize == 408
assert KP_DTYPE.itemsize == 32
assert MP_DTYPE.itemsize == 104
assert MPOBS_DTYPE.itemsize == 40
assert GPOBS_DTYPE.itemsize == 40

SECTIONS = [("cams", MCAM_DTYPE, "n_cam"), ("kfs", MKF_DTYPE, "n_kf"), ("kps", KP_DTYPE, "n_kp"),
            ("covis", np.dtype("<i8"), "n_covis"), ("mps", MP_DTYPE, "n_mp"), ("mpobs", MPOBS_DTYPE, "n_mpobs"),
            ("gpobs", GPOBS_DTYPE, "n_gpobs")]


@dataclass
class Snapshot:
    n_cam: int
    qc: np.ndarray
    inv_level_sigma2: np.ndarray
    scale_factor: np.ndarray
    cams: np.ndarray
    kfs: np.ndarray
    kps: np.ndarray
    covis: np.ndarray
    mps: np.ndarray
    mpobs: np.ndarray
    gpobs: np.ndarray

    def copy(self):
        return Snapshot(**{k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in self.__dict__.items()})


def _pad8(n):
    return (n + 7) & ~7


def pack(s):
    h = np.zeros(1, HEADER_DTYPE)
    h["magic"] = b"AMCSNAP"
    h["version"] = 2
    h["n_cam"] = s.n_cam
    for name, _, cnt in SECTIONS:
        if cnt != "n_cam":
            h[cnt] = len(getattr(s, name))
    h["n_levels"] = len(s.inv_level_sigma2)
    h["qc"] = np.asarray(s.qc, np.float64).reshape(36)
    h["inv_level_sigma2"][0, : len(s.inv_level_sigma2)] = s.inv_level_sigma2
    h["scale_factor"][0, : len(s.scale_factor)] = s.scale_factor
    parts = [h.tobytes()]
    for name, dt, _ in SECTIONS:
        b = np.ascontiguousarray(getattr(s, name), dtype=dt).tobytes()
        parts.append(b + b"\0" * (_pad8(len(b)) - len(b)))
    return b"".join(parts)


def unpack(buf):
    buf = bytes(buf)
    h = np.frombuffer(buf, HEADER_DTYPE, 1)[0]
    assert h["magic"] == b"AMCSNAP", "not a snapshot"
    off = _pad8(HEADER_DTYPE.itemsize)
    out = {}
    for name, dt, cnt in SECTIONS:
        n = int(h[cnt])
        out[name] = np.frombuffer(buf, dt, n, off).copy()
        off += _pad8(n * dt.itemsize)
    nl = int(h["n_levels"])
    return Snapshot(n_cam=int(h["n_cam"]), qc=h["qc"].reshape(6, 6).copy(),
                    inv_level_sigma2=h["inv_level_sigma2"][:nl].copy(), scale_factor=h["scale_factor"][:nl].copy(),
                    **out)


# ------------------------------------------------------------------ float SE3 (Sophus formulas)
def qnorm32(q):
    q = np.asarray(q, F32)
    n = np.sqrt(F32(F32(F32(q[0] * q[0]) + F32(q[1] * q[1])) + F32(q[2] * q[2])) + F32(q[3] * q[3]))
    return (q / n).astype(F32)


def _cross(a, b):
    return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]], a.dtype)


def qrotate(q, p):
    """so3.hpp:363-366: p + w uv + v x uv with uv = 2 (v x p), in the dtype of q."""
    v = q[:3]
    uv = _cross(v, p)
    uv = uv + uv
    return (p + q[3] * uv) + _cross(v, uv)


def se3_inverse(q, t):
    dt = np.asarray(q).dtype
    qi = np.array([-q[0], -q[1], -q[2], q[3]], dt)
    qi = qnorm32(qi) if dt == F32 else qi / np.sqrt(qi[0] * qi[0] + qi[1] * qi[1] + qi[2] * qi[2] + qi[3] * qi[3])
    return qi, qrotate(qi, -np.asarray(t, dt))


def twb_from_tbw(q, t):
    """PoseVelocity::Twb = GetPoseInverse().cast<double>() (src/G2oTypes.cc:26): float inverse,
    then widen and renormalise in double."""
    qi, ti = se3_inverse(np.asarray(q, F32), np.asarray(t, F32))
    qd = qi.astype(np.float64)
    qd = qd / np.sqrt(qd[0] * qd[0] + qd[1] * qd[1] + qd[2] * qd[2] + qd[3] * qd[3])
    return qd, ti.astype(np.float64)


# ------------------------------------------------------------------ synthetic map
def _octave_of(w):
    return np.rint(np.log(1.0 / np.asarray(w)) / (2 * np.log(1.2))).astype(np.int32)


def make_map(n_kf=30, n_lm=3000, obs_per_lm=6, n_cam=4, n_gp_frames=1, gp_obs_frac=0.3, seed=7, bad_mp_frac=0.01,
             close_mp_frac=0.2, other_map_kf=None, bad_kf=None):
    """A synthetic map of `n_kf` keyframes (ids 0..n_kf-1, linked by mPrevKF / mNextKF) from the
    local-BA generator, plus non-keyframe GP observations: for a fraction of the points, one
    frame between keyframe k and k+1 sees them again (MapPoint::AddGPObservation).  A few points
    are bad, some are tracked closer than 10 m, and one
    keyframe can be put in another map or flagged bad to exercise the window rules."""
    rng = np.random.default_rng(seed + 1)
    win = make_window(n_opt_kf=n_kf - 1, n_fixed=1, n_lm=n_lm, obs_per_lm=obs_per_lm, n_cam=n_cam, gp=True,
                      seed=seed, name="map")
    kf_t = win.kfs["time"]
    traj = _Trajectory(kf_t[0] - 0.1, kf_t[-1] + 0.1)
    o = win.obs

    # per (KF, camera) time stamps from the observations (mvTimeStamps)
    cam_time = np.repeat(kf_t[:, None], n_cam, axis=1).astype(np.float64)
    gp = o["kind"] == MONO_GP
    cam_time[o["kf_b"][gp], o["cam"][gp]] = o["t"][gp]

    # keyframes: T_bw = Twb^-1 in float (MultiKeyFrame stores mTbw)
    kfs = np.zeros(n_kf, MKF_DTYPE)
    kfs["id"] = np.arange(n_kf)
    kfs["prev_id"] = np.arange(n_kf) - 1
    kfs["next_id"] = np.where(np.arange(n_kf) + 1 < n_kf, np.arange(n_kf) + 1, -1)
    kfs["time"] = kf_t
    kfs["cam_time"][:, :n_cam] = cam_time
    for k in range(n_kf):
        qi, ti = se3_inverse(win.kfs[k]["q"].astype(F32), win.kfs[k]["t"].astype(F32))
        kfs[k]["q"] = qi
        kfs[k]["t"] = ti
        kfs[k]["vel"] = win.kfs[k]["vel"].astype(F32)
    kfs["bf"] = F32(win.kfs[0]["bf"])
    if other_map_kf is not None:
        kfs[other_map_kf]["map_id"] = 1
    if bad_kf is not None:
        kfs[bad_kf]["bad"] = 1

    # keypoints: one per (KF, camera) observation; the GP cameras' keypoints carry no u_right
    cam_of = np.where(o["kind"] >= MONO, n_cam - 1, o["cam"])
    order = np.lexsort((o["lm"], cam_of, o["kf_b"]))
    kps = np.zeros(len(o), KP_DTYPE)
    kps["x"] = o["z"][order, 0].astype(F32)
    kps["y"] = o["z"][order, 1].astype(F32)
    kps["octave"] = _octave_of(o["w"][order])
    kps["cam"] = cam_of[order]
    kps["ur"] = np.where(o["kind"][order] == STEREO, o["z"][order, 2], -1.0).astype(F32)
    kps["mp_id"] = o["lm"][order]
    kf_of_kp = o["kf_b"][order]
    starts = np.searchsorted(kf_of_kp, np.arange(n_kf))
    kfs["kp_off"] = starts
    kfs["n_kp"] = np.diff(np.append(starts, len(o)))
    kp_index = np.empty(len(o), np.int64)            # observation -> keypoint index within its KF
    kp_index[order] = np.arange(len(o)) - starts[kf_of_kp]

    # covisibility order: shared points, descending, ties by id (UpdateConnections weights)
    lm_kf = np.zeros((n_lm, n_kf), bool)
    lm_kf[o["lm"], o["kf_b"]] = True
    w = lm_kf.T.astype(np.int64) @ lm_kf.astype(np.int64)
    covis, off = [], []
    for k in range(n_kf):
        cand = [j for j in range(n_kf) if j != k and w[k, j] >= 15]
        cand.sort(key=lambda j: (-w[k, j], j))
        off.append(len(covis))
        covis.extend(cand)
    kfs["covis_off"] = off
    kfs["n_covis"] = [len([j for j in range(n_kf) if j != k and w[k, j] >= 15]) for k in range(n_kf)]

    # map points and their keyframe observations
    mps = np.zeros(n_lm, MP_DTYPE)
    mps["id"] = np.arange(n_lm)
    mps["pos"] = win.lm.astype(F32)
    mps["track_depth"][:, :n_cam] = rng.uniform(10.0, 40.0, (n_lm, n_cam)).astype(F32)
    mps["bad"] = rng.random(n_lm) < bad_mp_frac
    mo_rows = []
    lm_order = np.lexsort((o["kf_b"], o["lm"]))
    s_lm = o["lm"][lm_order]
    lm_start = np.searchsorted(s_lm, np.arange(n_lm + 1))
    for m in range(n_lm):
        rows = lm_order[lm_start[m]:lm_start[m + 1]]
        mps[m]["obs_off"] = len(mo_rows)
        kf_seen = {}
        for r in rows:
            kf_seen.setdefault(int(o["kf_b"][r]), []).append(r)
        for k in sorted(kf_seen):
            idx = np.full(MAX_CAM, -1, np.int32)
            for r in kf_seen[k]:
                idx[cam_of[r]] = kp_index[r]
            mo_rows.append((k, idx))
        mps[m]["n_obs"] = len(kf_seen)
        mps[m]["ref_kf"] = min(kf_seen) if kf_seen else -1
    mpobs = np.zeros(len(mo_rows), MPOBS_DTYPE)
    mpobs["kf_id"] = [k for k, _ in mo_rows]
    mpobs["idx"] = np.stack([i for _, i in mo_rows]) if mo_rows else np.zeros((0, MAX_CAM), np.int32)

    # bad points are unmatched in their keyframes (SetBadFlag -> EraseMapPointMatch)
    for m in np.nonzero(mps["bad"])[0]:
        kps["mp_id"][kps["mp_id"] == m] = -1

    # GP observations: a frame at t_k + 0.04..0.06 (k -> k+1) re-observes a fraction of the points
    cams = win.cams
    Rbc = quat_to_rot(cams["q"])
    gp_rows = []
    for m in range(n_lm):
        if mps[m]["bad"] or rng.random() >= gp_obs_frac:
            continue
        ks = sorted({int(k) for k in o["kf_b"][o["lm"] == m]})
        for _ in range(n_gp_frames):
            k = int(rng.choice(ks))
            if k + 1 >= n_kf:
                continue
            t = kf_t[k] + rng.uniform(0.04, 0.06)
            c = int(rng.integers(0, n_cam - 1))
            R, p = traj.pose(np.array(t))
            Rwc = R @ Rbc[c]
            pwc = p + R @ cams[c]["t"]
            Xc = Rwc.T @ (win.truth_lm[m] - pwc)
            if Xc[2] < 0.5:
                continue
            u = 500.0 * Xc[0] / Xc[2] + 480.0
            v = 500.0 * Xc[1] / Xc[2] + 300.0
            if not (0 <= u < 960 and 0 <= v < 600):
                continue
            octv = int(min(rng.geometric(0.5) - 1, 7))
            sig = 1.2 ** octv
            u, v = u + rng.normal() * sig, v + rng.normal() * sig
            if rng.random() < 0.05:
                u, v = rng.uniform(0, 960), rng.uniform(0, 600)
            ur = -1.0
            gp_rows.append((m, k, t, c, u, v, octv, ur))
    gp_rows.sort(key=lambda r: (r[0], r[1], r[2]))
    gpobs = np.zeros(len(gp_rows), GPOBS_DTYPE)
    if gp_rows:
        g = np.array([(r[1], r[2], r[3], r[4], r[5], r[6], r[7]) for r in gp_rows])
        gpobs["kf_id"] = g[:, 0].astype(np.int64)
        gpobs["time"] = g[:, 1]
        gpobs["cam"] = g[:, 2].astype(np.int32)
        gpobs["x"] = g[:, 3].astype(F32)
        gpobs["y"] = g[:, 4].astype(F32)
        gpobs["octave"] = g[:, 5].astype(np.int32)
        gpobs["ur"] = g[:, 6].astype(F32)
    gm = np.array([r[0] for r in gp_rows], np.int64)
    gstart = np.searchsorted(gm, np.arange(n_lm + 1))
    mps["gp_off"] = gstart[:-1]
    mps["n_gp"] = np.diff(gstart)

    # tracked closer than 10 m: the post-pass relaxes their threshold 1.5x (Optimizer.cc:1267-1271)
    close = rng.random(n_lm) < close_mp_frac
    mps["track_depth"][close, :n_cam] = F32(5.0)

    mcams = np.zeros(n_cam, MCAM_DTYPE)
    mcams["q"] = cams["q"].astype(F32)
    mcams["t"] = cams["t"].astype(F32)
    mcams["rbc_ini"] = cams["q"].astype(F32)      # mRbc_ini = the initial mTbc rotation (Frame.cc:181)
    for f in ("fx", "fy", "cx", "cy"):
        mcams[f] = cams[f].astype(F32)
    levels = 8
    sf = np.array([1.2 ** i for i in range(levels)], F32)
    inv_s2 = np.array([1.0 / float(F32(x * x)) for x in sf], F32)
    qc = np.diag([0.02, 0.02, 0.02, 0.002, 0.002, 0.002])
    return Snapshot(n_cam=n_cam, qc=qc, inv_level_sigma2=inv_s2, scale_factor=sf, cams=mcams, kfs=kfs, kps=kps,
                    covis=np.array(covis, np.int64), mps=mps, mpobs=mpobs, gpobs=gpobs)


# ------------------------------------------------------------------ ctypes binding
PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LBAMAP_ABI_VERSION = 2   # include/amc_lba_map.h: the structs below (LbamapResult with ms_phase)
# AMC_LBA_MAP_LIB: another build of the adapter (A/B of two builds: scripts/cmp_map_libs.py)
MAP_LIB_PATH = os.environ.get("AMC_LBA_MAP_LIB") or os.path.join(PKG_DIR, "lib", "libamc_lba_map.so")
_lib = None


class LbamapOptions(ctypes.Structure):
    _fields_ = [("large", ctypes.c_int32), ("extrinsic", ctypes.c_int32), ("device", ctypes.c_int32),
                ("flags", ctypes.c_int32)]


class LbamapResult(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "status", "n_opt_kf", "n_vis_kf", "n_fixed_kf", "n_mp", "n_edges_mono_gp", "n_edges_stereo_gp", "n_edges_mono",
        "n_edges_stereo", "n_edges_mono_gp_kf", "n_erased_gp", "n_erased", "n_set_bad", "iterations")] + [
        ("chi2_initial", ctypes.c_double), ("chi2_final", ctypes.c_double), ("ms_phase", ctypes.c_double * 4)]


class LbamapBAResult(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("status", "n_kf", "n_fixed_kf", "n_mp", "n_priors", "n_vel")] + [
        ("n_edges", ctypes.c_int32 * 5), ("iterations", ctypes.c_int32),
        ("chi2_initial", ctypes.c_double), ("chi2_final", ctypes.c_double)]


def map_lib():
    global _lib
    if _lib is None:
        if not os.path.exists(MAP_LIB_PATH):
            raise RuntimeError(f"{MAP_LIB_PATH} not built: run python -c 'import __graft_entry__ as g; g.build()'")
        from . import check_fresh
        if not os.environ.get("AMC_LBA_MAP_LIB"):
            check_fresh("map")
        L = ctypes.CDLL(MAP_LIB_PATH)
        if hasattr(L, "lbamap_abi_version") and L.lbamap_abi_version() != LBAMAP_ABI_VERSION:
            raise RuntimeError(f"{MAP_LIB_PATH}: adapter ABI {L.lbamap_abi_version()}, this binding {LBAMAP_ABI_VERSION}")
        vp = ctypes.c_void_p
        L.lbamap_load.argtypes = [ctypes.POINTER(vp), ctypes.c_char_p, ctypes.c_size_t]
        L.lbamap_free.argtypes = [vp]
        L.lbamap_free.restype = None
        L.lbamap_last_error.argtypes = [vp]
        L.lbamap_last_error.restype = ctypes.c_char_p
        L.lbamap_snapshot_size.argtypes = [vp]
        L.lbamap_snapshot_size.restype = ctypes.c_size_t
        L.lbamap_save.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t]
        L.lbamap_save.restype = ctypes.c_int64
        L.lbamap_local_gpba.argtypes = [vp, ctypes.c_int64, vp, ctypes.POINTER(LbamapOptions),
                                        ctypes.POINTER(LbamapResult)]
        L.lbamap_build_window.argtypes = [vp, ctypes.c_int64, ctypes.POINTER(LbamapOptions),
                                          ctypes.POINTER(ctypes.c_int32)] + [vp] * 9 + [ctypes.POINTER(LbaConfig)]
        L.lbamap_global_ba.argtypes = [vp, ctypes.c_int32, vp, ctypes.c_uint64, ctypes.POINTER(LbamapOptions),
                                       ctypes.POINTER(LbamapBAResult)]
        L.lbamap_kf_gba.argtypes = [vp, ctypes.c_int64, vp, vp, vp, ctypes.POINTER(ctypes.c_uint64)]
        L.lbamap_mp_gba.argtypes = [vp, ctypes.c_int64, vp, ctypes.POINTER(ctypes.c_uint64)]
        L.lbamap_global_ba_thread.argtypes = [vp, ctypes.c_int32, vp, ctypes.c_uint64]
        L.lbamap_build_ba_window.argtypes = [vp, ctypes.POINTER(ctypes.c_int32)] + [vp] * 9 + [ctypes.POINTER(LbaConfig)]
        _lib = L
    return _lib


def exported_symbols():
    return ["lbamap_abi_version", "lbamap_load", "lbamap_free", "lbamap_last_error", "lbamap_snapshot_size", "lbamap_save",
            "lbamap_local_gpba", "lbamap_build_window", "lbamap_global_ba", "lbamap_global_ba_thread", "lbamap_kf_gba", "lbamap_mp_gba",
            "lbamap_build_ba_window"]


class LocalGPBAMap:
    """A map loaded into the C++ adapter (lbamap_load)."""

    def __init__(self, snap):
        L = map_lib()
        self.h = ctypes.c_void_p()
        data = pack(snap) if isinstance(snap, Snapshot) else bytes(snap)
        rc = L.lbamap_load(ctypes.byref(self.h), data, len(data))
        if rc != 0:
            raise RuntimeError(f"lbamap_load failed ({rc})")

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            map_lib().lbamap_free(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        self.close()

    def error(self):
        return map_lib().lbamap_last_error(self.h).decode()

    def save(self):
        L = map_lib()
        n = L.lbamap_snapshot_size(self.h)
        buf = ctypes.create_string_buffer(n)
        w = L.lbamap_save(self.h, buf, n)
        if w < 0:
            raise RuntimeError("lbamap_save failed")
        return unpack(buf.raw[:w])

    def local_gpba(self, kf_id, large=False, extrinsic=False, device=0, flags=0):
        opt = LbamapOptions(int(large), int(extrinsic), device, flags)
        res = LbamapResult()
        rc = map_lib().lbamap_local_gpba(self.h, kf_id, None, ctypes.byref(opt), ctypes.byref(res))
        return rc, res

    def global_ba(self, iterations=10, loop_kf=0, device=0, flags=0, stop_flag=None):
        """GlobalBundleAdjustemnt(map, iterations, stop, loop_kf) on the GPU; returns (rc, LbamapBAResult)."""
        opt = LbamapOptions(0, 0, device, flags)
        res = LbamapBAResult()
        sf = None if stop_flag is None else ctypes.byref(stop_flag)
        rc = map_lib().lbamap_global_ba(self.h, iterations, sf, loop_kf, ctypes.byref(opt), ctypes.byref(res))
        return rc, res

    def global_ba_thread(self, iterations=10, loop_kf=0):
        """The reference signature GlobalBundleAdjustemnt(pMap, it, pbStopFlag, nLoopKF) on the calling
        thread, with the engine owned by (and freed with) that thread; returns rc."""
        return map_lib().lbamap_global_ba_thread(self.h, iterations, None, loop_kf)

    def kf_gba(self, kf_id):
        q, t, v = np.zeros(4, np.float32), np.zeros(3, np.float32), np.zeros(6, np.float32)
        lk = ctypes.c_uint64()
        rc = map_lib().lbamap_kf_gba(self.h, kf_id, ptr(q), ptr(t), ptr(v), ctypes.byref(lk))
        if rc != 0:
            raise RuntimeError("lbamap_kf_gba failed")
        return q, t, v, lk.value

    def mp_gba(self, mp_id):
        p = np.zeros(3, np.float32)
        lk = ctypes.c_uint64()
        rc = map_lib().lbamap_mp_gba(self.h, mp_id, ptr(p), ctypes.byref(lk))
        if rc != 0:
            raise RuntimeError("lbamap_mp_gba failed")
        return p, lk.value

    def build_ba_window(self):
        """The flat global-BA graph BundleAdjustment would optimise (no GPU needed).  Returns (Window,
        kf_ids, mp_ids, obs_tag)."""
        L = map_lib()
        cnt = (ctypes.c_int32 * 6)()
        rc = L.lbamap_build_ba_window(self.h, cnt, *([None] * 9), None)
        if rc != 0:
            raise RuntimeError(self.error())
        return self._flat(cnt, lambda *a: L.lbamap_build_ba_window(self.h, cnt, *a), "global_ba")

    def _flat(self, cnt, fill, name):
        n_kf, n_lm, n_obs, n_pri, n_vel, n_cam = list(cnt)
        kfs = np.zeros(n_kf, KF_DTYPE)
        lm = np.zeros((n_lm, 3))
        obs = np.zeros(n_obs, OBS_DTYPE)
        pri = np.zeros(n_pri, PRIOR_DTYPE)
        vel = np.zeros(n_vel, np.int32)
        cams = np.zeros(n_cam, CAM_DTYPE)
        kf_ids = np.zeros(n_kf, np.int64)
        mp_ids = np.zeros(n_lm, np.int64)
        tag = np.zeros(n_obs, np.int32)
        cfg = LbaConfig()
        rc = fill(ptr(kfs), ptr(lm), ptr(obs), ptr(pri), ptr(vel), ptr(cams), ptr(kf_ids), ptr(mp_ids), ptr(tag),
                  ctypes.byref(cfg))
        if rc != 0:
            raise RuntimeError(self.error())
        wcfg = {"huber_mono": cfg.huber_mono, "huber_stereo": cfg.huber_stereo, "huber_prior": cfg.huber_prior,
                "lambda_init": cfg.lambda_init, "qc_diag": np.array(cfg.qc[:]).reshape(6, 6)}
        win = Window(kfs=kfs, lm=lm, obs=obs, priors=pri, vel_kfs=vel, cams=cams, cfg=wcfg, name=name)
        return win, kf_ids, mp_ids, tag

    def build_window(self, kf_id, large=False):
        """The flat window LocalGPBA would optimise (no GPU needed).  Returns (Window, kf_ids,
        mp_ids, obs_tag)."""
        L = map_lib()
        opt = LbamapOptions(int(large), 0, 0, 0)
        cnt = (ctypes.c_int32 * 6)()
        rc = L.lbamap_build_window(self.h, kf_id, ctypes.byref(opt), cnt, *([None] * 9), None)
        if rc != 0:
            raise RuntimeError(self.error())
        n_kf, n_lm, n_obs, n_pri, n_vel, n_cam = list(cnt)
        kfs = np.zeros(n_kf, KF_DTYPE)
        lm = np.zeros((n_lm, 3))
        obs = np.zeros(n_obs, OBS_DTYPE)
        pri = np.zeros(n_pri, PRIOR_DTYPE)
        vel = np.zeros(n_vel, np.int32)
        cams = np.zeros(n_cam, CAM_DTYPE)
        kf_ids = np.zeros(n_kf, np.int64)
        mp_ids = np.zeros(n_lm, np.int64)
        tag = np.zeros(n_obs, np.int32)
        cfg = LbaConfig()
        rc = L.lbamap_build_window(self.h, kf_id, ctypes.byref(opt), cnt, ptr(kfs), ptr(lm), ptr(obs), ptr(pri),
                                   ptr(vel), ptr(cams), ptr(kf_ids), ptr(mp_ids), ptr(tag), ctypes.byref(cfg))
        if rc != 0:
            raise RuntimeError(self.error())
        wcfg = {"huber_mono": cfg.huber_mono, "huber_stereo": cfg.huber_stereo, "huber_prior": cfg.huber_prior,
                "lambda_init": cfg.lambda_init, "qc_diag": np.array(cfg.qc[:]).reshape(6, 6)}
        win = Window(kfs=kfs, lm=lm, obs=obs, priors=pri, vel_kfs=vel, cams=cams, cfg=wcfg, name=f"localgpba_{kf_id}")
        return win, kf_ids, mp_ids, tag
