"""Deterministic synthetic local-BA windows.

A vehicle drives forward at 4 m/s with a gentle yaw sinusoid; keyframes every 0.1 s
(`Camera.fps: 10`, Examples/MultiCamera/orb_multicam.yaml:8); pinhole fx=fy=500, cx=480,
cy=300, 960x600 (:11-12); cameras 0..n-2 are asynchronous (time stamps uniform in
[t_KF-0.08, t_KF-0.01]) and the last camera is the reference at t_KF (src/Frame.cc:132);
landmarks lie in a 5-60 m shell and are seen by ~6 (KF, camera) pairs; ORB octave weights
1/1.2^(2*octave) (src/ORBextractor.cc:415-429); N(0, 1.2^octave px) noise plus 5 % uniform
outliers; every stored value is rounded to float32 like the reference's float storage
(src/G2oTypes.cc:26-27, src/Optimizer.cc:1016).  The graph shape mirrors LocalGPBA
(src/Optimizer.cc:858-1208): one fixed previous KF, EdgeVelocity on every optimisable KF,
EdgeGaussianPrior between consecutive optimisable KFs, EdgeMonoGPExtrinsic for cameras
0..n-2 (vertices prev KF, KF) and EdgeMono/EdgeStereo for the reference camera.
"""
from dataclasses import dataclass, field, replace

import numpy as np

from .abi import CAM_DTYPE, KF_DTYPE, MONO, MONO_GP, OBS_DTYPE, PRIOR_DTYPE, STEREO, STEREO_GP

F32 = np.float32


def _f32(a):
    return np.asarray(a, dtype=np.float64).astype(F32).astype(np.float64)


def _rotz(a):
    c, s = np.cos(a), np.sin(a)
    R = np.zeros(np.shape(a) + (3, 3))
    R[..., 0, 0] = c
    R[..., 0, 1] = -s
    R[..., 1, 0] = s
    R[..., 1, 1] = c
    R[..., 2, 2] = 1.0
    return R


def _expso3(w):
    w = np.asarray(w, dtype=np.float64)
    th = np.linalg.norm(w, axis=-1, keepdims=True)
    k = np.where(th > 1e-12, w / np.maximum(th, 1e-300), 0.0)
    K = np.zeros(w.shape[:-1] + (3, 3))
    K[..., 0, 1], K[..., 0, 2] = -k[..., 2], k[..., 1]
    K[..., 1, 0], K[..., 1, 2] = k[..., 2], -k[..., 0]
    K[..., 2, 0], K[..., 2, 1] = -k[..., 1], k[..., 0]
    th = th[..., None]
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * (K @ K)


def rot_to_quat(R):
    """Rotation matrix -> unit quaternion (x, y, z, w), w >= 0."""
    R = np.asarray(R)
    q = np.zeros(R.shape[:-2] + (4,))
    tr = R[..., 0, 0] + R[..., 1, 1] + R[..., 2, 2]
    w = np.sqrt(np.maximum(0.0, 1.0 + tr)) / 2
    x = np.sqrt(np.maximum(0.0, 1.0 + R[..., 0, 0] - R[..., 1, 1] - R[..., 2, 2])) / 2
    y = np.sqrt(np.maximum(0.0, 1.0 - R[..., 0, 0] + R[..., 1, 1] - R[..., 2, 2])) / 2
    z = np.sqrt(np.maximum(0.0, 1.0 - R[..., 0, 0] - R[..., 1, 1] + R[..., 2, 2])) / 2
    x = np.copysign(x, R[..., 2, 1] - R[..., 1, 2])
    y = np.copysign(y, R[..., 0, 2] - R[..., 2, 0])
    z = np.copysign(z, R[..., 1, 0] - R[..., 0, 1])
    q[..., 0], q[..., 1], q[..., 2], q[..., 3] = x, y, z, w
    return q / np.linalg.norm(q, axis=-1, keepdims=True)


def quat_to_rot(q):
    x, y, z, w = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    R = np.empty(q.shape[:-1] + (3, 3))
    R[..., 0, 0] = 1 - 2 * (y * y + z * z)
    R[..., 0, 1] = 2 * (x * y - z * w)
    R[..., 0, 2] = 2 * (x * z + y * w)
    R[..., 1, 0] = 2 * (x * y + z * w)
    R[..., 1, 1] = 1 - 2 * (x * x + z * z)
    R[..., 1, 2] = 2 * (y * z - x * w)
    R[..., 2, 0] = 2 * (x * z - y * w)
    R[..., 2, 1] = 2 * (y * z + x * w)
    R[..., 2, 2] = 1 - 2 * (x * x + y * y)
    return R


class _Trajectory:
    """Planar vehicle: yaw rate A cos(2 pi t / P), speed 4 m/s, body x forward, z up."""

    def __init__(self, t0, t1, speed=4.0, A=0.15, P=8.0, height=1.5):
        self.speed, self.A, self.P, self.h = speed, A, P, height
        self.tg = np.arange(t0 - 0.2, t1 + 0.2, 1e-3)
        yaw = self.yaw(self.tg)
        dx = speed * np.cos(yaw)
        dy = speed * np.sin(yaw)
        dt = np.diff(self.tg)
        self.xg = np.concatenate([[0.0], np.cumsum(0.5 * (dx[1:] + dx[:-1]) * dt)])
        self.yg = np.concatenate([[0.0], np.cumsum(0.5 * (dy[1:] + dy[:-1]) * dt)])

    def yaw(self, t):
        return self.A * self.P / (2 * np.pi) * np.sin(2 * np.pi * np.asarray(t) / self.P)

    def yaw_rate(self, t):
        return self.A * np.cos(2 * np.pi * np.asarray(t) / self.P)

    def pose(self, t):
        t = np.asarray(t, dtype=np.float64)
        R = _rotz(self.yaw(t))
        p = np.stack([np.interp(t, self.tg, self.xg), np.interp(t, self.tg, self.yg),
                      np.full(t.shape, self.h)], axis=-1)
        return R, p

    def twist(self, t):
        """Body twist [v; w]: T(t+d) ~ T(t) exp(d * twist)."""
        t = np.asarray(t, dtype=np.float64)
        v = np.zeros(t.shape + (6,))
        v[..., 0] = self.speed
        v[..., 5] = self.yaw_rate(t)
        return v


class _CircleTrajectory(_Trajectory):
    """One lap of a circle in `period` seconds (constant yaw rate): the last keyframes come back to where
    the first ones were, so landmarks near the start are seen again at the end (a loop closure)."""

    def __init__(self, t_start, period, speed=4.0, height=1.5):
        self.t_start, self.period, self.speed, self.h = t_start, period, speed, height
        self.w = 2 * np.pi / period
        self.r = speed / self.w

    def yaw(self, t):
        return self.w * (np.asarray(t) - self.t_start)

    def yaw_rate(self, t):
        return np.full(np.shape(t), self.w)

    def pose(self, t):
        t = np.asarray(t, dtype=np.float64)
        a = self.yaw(t)
        R = _rotz(a)
        p = np.stack([self.r * np.sin(a), self.r * (1 - np.cos(a)), np.full(t.shape, self.h)], axis=-1)
        return R, p


@dataclass
class Window:
    kfs: np.ndarray
    lm: np.ndarray
    obs: np.ndarray
    priors: np.ndarray
    vel_kfs: np.ndarray
    cams: np.ndarray
    cfg: dict = field(default_factory=dict)
    truth_lm: np.ndarray = None
    name: str = ""
    lm_gid: np.ndarray = None     # global landmark ids (window farm)
    kf_gid: np.ndarray = None     # global keyframe ids (window farm)

    @property
    def n_pairs(self):
        """Unique (non-fixed KF, landmark) Hpl blocks (SURVEY.md §8(d) n_pairs)."""
        fixed = self.kfs["fixed"] != 0
        keys = []
        gp = (self.obs["kind"] == MONO_GP) | (self.obs["kind"] == STEREO_GP)
        for col, m in (("kf_b", np.ones(len(self.obs), bool)), ("kf_a", gp)):
            k = self.obs[col][m]
            lmi = self.obs["lm"][m]
            ok = ~fixed[k]
            keys.append(k[ok].astype(np.int64) * (len(self.lm) + 1) + lmi[ok])
        return int(np.unique(np.concatenate(keys)).size)

    def summary(self):
        kinds = np.bincount(self.obs["kind"], minlength=4)
        return {"n_kf": int(len(self.kfs)), "n_opt_kf": int((self.kfs["fixed"] == 0).sum()),
                "n_lm": int(len(self.lm)), "n_obs": int(len(self.obs)),
                "mono_gp": int(kinds[MONO_GP]), "stereo_gp": int(kinds[STEREO_GP]),
                "mono": int(kinds[MONO]), "stereo": int(kinds[STEREO]),
                "n_priors": int(len(self.priors)), "n_vel": int(len(self.vel_kfs))}


def make_window(n_opt_kf=50, n_fixed=1, n_lm=20000, obs_per_lm=6, n_cam=4, gp=True, stereo_frac=0.5,
                outlier_frac=0.05, seed=20250912, global_ba=False, perturb=True, t0=100.0, name="",
                track=None, max_track=40, band=25, loop=False, straight=False):
    """Build one window.  n_fixed KFs come first (oldest); global_ba=True gives the
    BundleAdjustment graph shape (priors from the first KF, Huber 21.026 on priors, lambda0
    1e-5, src/Optimizer.cc:61-321).  Landmarks are seen from a band of `band` KFs around their
    anchor; track=None draws obs_per_lm +- 2 observations per landmark, track="geometric" a
    long-tailed track length 2 + Geometric(1 / (obs_per_lm - 1)) capped at max_track (long tracks:
    landmarks seen from more keyframes than one tile of the device path holds).  loop=True drives one
    lap of a circle: the keyframe band around a landmark's anchor wraps around, so the last keyframes
    re-observe the first ones' landmarks (the long-range blocks of a loop-closure global BA); loop=k
    drives k laps, so every place is revisited k - 1 times and a landmark is seen from the keyframes
    near its place on every lap.  straight=True drives a straight line (no yaw) and perturbs no
    orientation or angular velocity: consecutive keyframes' relative rotations, the interpolated samples'
    and the velocities' omega are then zero (below every small-angle threshold of Sophus and Pose3utils)
    at the first linearisation."""
    rng = np.random.default_rng(seed)
    n_kf = n_fixed + n_opt_kf
    kf_t = t0 + 0.1 * np.arange(n_kf)
    laps = int(loop)
    traj = (_CircleTrajectory(kf_t[0], 0.1 * n_kf / laps) if loop else
            _Trajectory(kf_t[0] - 0.1, kf_t[-1] + 0.1, A=0.0 if straight else 0.15))

    # --- cameras: reference camera (last) looks forward; others yawed +90, 180, -90 deg
    Rbc0 = np.array([[0.0, 0.0, 1.0], [-1.0, 0.0, 0.0], [0.0, -1.0, 0.0]])
    yaws = [np.pi / 2, np.pi, -np.pi / 2, 0.0]
    cam_yaw = [yaws[c % 3] for c in range(n_cam - 1)] + [0.0]
    cams = np.zeros(n_cam, CAM_DTYPE)
    Rbc = np.zeros((n_cam, 3, 3))
    tbc = np.zeros((n_cam, 3))
    for c in range(n_cam):
        R = _rotz(cam_yaw[c]) @ Rbc0
        q = _f32(rot_to_quat(R))
        Rbc[c] = quat_to_rot(q)
        tbc[c] = _f32([0.5 * np.cos(cam_yaw[c]), 0.5 * np.sin(cam_yaw[c]), 0.2])
        cams[c]["q"] = q
        cams[c]["t"] = tbc[c]
        cams[c]["fx"], cams[c]["fy"], cams[c]["cx"], cams[c]["cy"] = 500.0, 500.0, 480.0, 300.0
        cams[c]["rbc_ini"] = q                                  # MultiFrame::mRbc_ini (Frame.cc:181)
        cams[c]["rbc_info"] = (0.2 * np.eye(3)).ravel()         # mRbc_ini_cov (Frame.cc:182)
    W, H = 960.0, 600.0
    bf = float(F32(0.12 * 500.0))

    # --- per (KF, camera) time stamps (MultiKeyFrame::mvTimeStamps)
    ts = np.repeat(kf_t[:, None], n_cam, axis=1)
    if gp and n_cam > 1:
        ts[:, : n_cam - 1] -= rng.uniform(0.01, 0.08, size=(n_kf, n_cam - 1))
    Rwb_t, pwb_t = traj.pose(ts)                      # [n_kf, n_cam, 3, 3], [n_kf, n_cam, 3]
    Rwc = Rwb_t @ Rbc[None]                           # camera orientation in world
    pwc = pwb_t + np.einsum("kcij,cj->kci", Rwb_t, tbc)

    # --- landmarks: anchor (KF, cam), pixel, depth 5-60 m
    nl_gen = int(n_lm * 1.6) + 64
    k0 = rng.integers(0, n_kf, nl_gen)
    c0 = rng.integers(0, n_cam, nl_gen)
    u0 = rng.uniform(0, W, nl_gen)
    v0 = rng.uniform(0, H, nl_gen)
    d0 = rng.uniform(5.0, 60.0, nl_gen)
    Xc0 = np.stack([(u0 - 480.0) / 500.0 * d0, (v0 - 300.0) / 500.0 * d0, d0], axis=-1)
    Xw = np.einsum("nij,nj->ni", Rwc[k0, c0], Xc0) + pwc[k0, c0]

    # --- visibility over a KF band around the anchor (chunked over landmarks to bound memory)
    band = min(n_kf, band)
    koff = np.arange(band) - band // 2
    if loop:   # the band wraps around the lap (and is repeated on every lap: the places revisited)
        if laps > 1:
            koff = (koff[None, :] + np.round(np.arange(laps) * n_kf / laps).astype(int)[:, None]).ravel()
        kk = (k0[:, None] + koff[None, :]) % n_kf
        kk_valid = np.ones(kk.shape, bool)
    else:
        kk = np.clip(k0[:, None] + koff[None, :], 0, n_kf - 1)                 # [nl, band]
        kk_valid = (k0[:, None] + koff[None, :] >= 0) & (k0[:, None] + koff[None, :] < n_kf)
    band = kk.shape[1]
    u = np.empty((nl_gen, band, n_cam))
    v = np.empty((nl_gen, band, n_cam))
    z = np.empty((nl_gen, band, n_cam))
    vis = np.empty((nl_gen, band, n_cam), bool)
    CH = 16384
    for c0_ in range(0, nl_gen, CH):
        sl = slice(c0_, min(nl_gen, c0_ + CH))
        dXw = Xw[sl, None, None, :] - pwc[kk[sl]]                            # [ch, band, ncam, 3]
        Xc = np.einsum("nbcji,nbcj->nbci", Rwc[kk[sl]], dXw)
        zc = Xc[..., 2]
        with np.errstate(divide="ignore", invalid="ignore"):
            uc = 500.0 * Xc[..., 0] / zc + 480.0
            vc = 500.0 * Xc[..., 1] / zc + 300.0
        u[sl], v[sl], z[sl] = uc, vc, zc
        vis[sl] = (zc > 0.5) & (uc >= 0) & (uc < W) & (vc >= 0) & (vc < H) & (np.linalg.norm(Xc, axis=-1) < 70.0)
    vis &= kk_valid[:, :, None]
    if gp and n_cam > 1:
        # GP edges need the previous KF inside the window (src/Optimizer.cc:1112-1116)
        vis[:, :, : n_cam - 1] &= (kk > 0)[:, :, None]
    dk = np.abs(kk - k0[:, None])
    if loop:   # distance along the lap
        per = n_kf / laps
        dk = np.mod(dk, per) if laps > 1 else dk
        dk = np.minimum(dk, (per if laps > 1 else n_kf) - dk)
    score = dk[:, :, None] * n_cam + rng.random(vis.shape)
    score = np.where(vis, score, np.inf).reshape(nl_gen, -1)
    order = np.argsort(score, axis=1, kind="stable")
    nvalid = np.isfinite(score).sum(axis=1)
    if track == "geometric":
        target = np.minimum(max_track, 2 + rng.geometric(1.0 / max(obs_per_lm - 1, 1), nl_gen))
    else:
        target = rng.integers(obs_per_lm - 2, obs_per_lm + 3, nl_gen)
    take = np.minimum(target, nvalid)
    keep = np.nonzero(take >= 2)[0][:n_lm]
    if keep.size < n_lm:
        raise RuntimeError("synthetic generator could not place enough landmarks")

    tk = take[keep]
    rows_j = np.repeat(np.arange(keep.size), tk)
    pos = np.arange(rows_j.size) - np.repeat(np.cumsum(tk) - tk, tk)
    sel = order[keep[rows_j], pos]
    b_i, c_i = np.divmod(sel, n_cam)
    k_i = kk[keep[rows_j], b_i]
    o = np.lexsort((c_i, k_i, rows_j))      # per landmark, per KF: GP cams first, reference cam last
    lm_i, k_i, c_i, b_i = rows_j[o], k_i[o], c_i[o], b_i[o]
    src_j = keep[lm_i]
    n_obs = lm_i.size

    uu = u[src_j, b_i, c_i]
    vv = v[src_j, b_i, c_i]
    zz = z[src_j, b_i, c_i]
    octave = np.minimum(rng.geometric(0.5, n_obs) - 1, 7)
    sigma = 1.2 ** octave
    uu_n = uu + rng.normal(0, 1, n_obs) * sigma
    vv_n = vv + rng.normal(0, 1, n_obs) * sigma
    outl = rng.random(n_obs) < outlier_frac
    uu_n[outl] = rng.uniform(0, W, outl.sum())
    vv_n[outl] = rng.uniform(0, H, outl.sum())
    ur = uu - bf / zz + rng.normal(0, 1, n_obs) * sigma

    is_ref = c_i == n_cam - 1
    if gp and n_cam > 1:
        kind = np.where(is_ref, MONO, MONO_GP)
    else:
        kind = np.full(n_obs, MONO)
    stereo_sel = is_ref & (zz < 20.0) & (rng.random(n_obs) < stereo_frac)
    kind = np.where(stereo_sel, STEREO, kind)

    obs = np.zeros(n_obs, OBS_DTYPE)
    obs["kind"] = kind
    obs["kf_b"] = k_i
    obs["kf_a"] = np.where((kind == MONO_GP) | (kind == STEREO_GP), k_i - 1, -1)
    obs["lm"] = lm_i
    obs["cam"] = np.where(kind >= MONO, n_cam - 1, c_i)
    obs["t"] = ts[k_i, c_i]
    obs["z"][:, 0] = _f32(uu_n)
    obs["z"][:, 1] = _f32(vv_n)
    obs["z"][:, 2] = np.where(kind == STEREO, _f32(ur), 0.0)
    obs["w"] = _f32(1.0 / (1.2 ** (2 * octave)))

    # --- keyframe states (truth at KF time, perturbed for the optimisable ones)
    Rk, pk = traj.pose(kf_t)
    vk = traj.twist(kf_t)
    kfs = np.zeros(n_kf, KF_DTYPE)
    for i in range(n_kf):
        R, p, vel = Rk[i], pk[i].copy(), vk[i].copy()
        fixed = i < n_fixed
        if perturb and not fixed:
            dR = rng.normal(0, np.deg2rad(0.5), 3)
            p = p + rng.normal(0, 0.05, 3)
            dv = rng.normal(0, 0.1, 6)
            if straight:
                dv[3:] = 0.0
            else:
                R = R @ _expso3(dR)
            vel = vel + dv
        kfs[i]["q"] = _f32(rot_to_quat(R))
        kfs[i]["t"] = _f32(p)
        kfs[i]["vel"] = _f32(vel)
        kfs[i]["time"] = kf_t[i]
        kfs[i]["bf"] = bf
        kfs[i]["fixed"] = int(fixed)

    truth_lm = Xw[keep]
    lm = truth_lm + (rng.normal(0, 0.1, truth_lm.shape) if perturb else 0.0)
    lm = _f32(lm)

    # --- motion-prior and velocity edges
    if gp:
        first = 0 if global_ba else n_fixed
        pri = [(k, k + 1) for k in range(first, n_kf - 1)]
        vel_kfs = np.arange(0 if global_ba else n_fixed, n_kf, dtype=np.int32)
    else:
        pri, vel_kfs = [], np.zeros(0, np.int32)
    priors = np.zeros(len(pri), PRIOR_DTYPE)
    if pri:
        priors["kf_a"] = [a for a, _ in pri]
        priors["kf_b"] = [b for _, b in pri]

    cfg = {"huber_prior": 21.026 if global_ba else 0.0, "lambda_init": 1e-5 if global_ba else 1.0}
    return Window(kfs=kfs, lm=np.ascontiguousarray(lm), obs=obs, priors=priors,
                  vel_kfs=np.ascontiguousarray(vel_kfs, dtype=np.int32), cams=cams, cfg=cfg,
                  truth_lm=truth_lm, name=name)


def with_free_extrinsics(win, cams=None, rot_deg=0.3, trans=0.01, seed=7):
    """The window of an extrinsic-calibration pass (LocalGPBA bExtrinsic, src/Optimizer.cc:1228-1240):
    the asynchronous cameras' (all but the reference camera) VertexExtrinsic free, their Tbc estimates
    perturbed by rot_deg / trans (float-rounded like MultiKeyFrame::mTbc) while the extrinsic prior keeps
    the generating rotation as mRbc_ini."""
    rng = np.random.default_rng(seed)
    cam = win.cams.copy()
    sel = range(len(cam) - 1) if cams is None else cams
    for c in sel:
        R = quat_to_rot(cam[c]["q"]) @ _expso3(rng.normal(0, np.deg2rad(rot_deg), 3))
        cam[c]["q"] = _f32(rot_to_quat(R))
        cam[c]["t"] = _f32(cam[c]["t"] + rng.normal(0, trans, 3))
        cam[c]["ext_free"] = 1
    return replace(win, cams=cam, name=(win.name or "window") + "_ext")


# BASELINE.json configs (SURVEY.md §8(d) per-config instances)
CONFIGS = {
    "cfg0_cpu_plumbing": dict(n_opt_kf=9, n_fixed=1, n_lm=2000, obs_per_lm=5, n_cam=1, gp=False, stereo_frac=0.0),
    "cfg1_local_50kf": dict(n_opt_kf=50, n_fixed=1, n_lm=20000, obs_per_lm=6, n_cam=4, gp=True),
    "cfg2_global_500kf": dict(n_opt_kf=499, n_fixed=1, n_lm=200000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True),
    # config 4: AMV-Bench-shaped full-trajectory global BA, partitioned over the GPUs (amc_lba/gba.py)
    "cfg4_global_5k": dict(n_opt_kf=4999, n_fixed=1, n_lm=1000000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True),
}


def make_config_window(name, seed=20250912, **over):
    kw = dict(CONFIGS[name])
    kw.update(over)
    return make_window(seed=seed, name=name, **kw)


def cut_window(g, k0, n_opt, name=""):
    """LocalGPBA-shaped sub-window of a long map: KF k0 fixed (the oldest KF's mPrevKF), KFs
    k0+1..k0+n_opt optimisable; GP edges whose previous KF falls outside are dropped exactly like
    src/Optimizer.cc:1112-1116; landmarks are the ones the kept observations see."""
    ks = np.arange(k0, k0 + 1 + n_opt)
    kmap = -np.ones(len(g.kfs), np.int64)
    kmap[ks] = np.arange(ks.size)
    o = g.obs
    gp = (o["kind"] == MONO_GP) | (o["kind"] == STEREO_GP)
    keep = (kmap[o["kf_b"]] >= 0) & (~gp | (kmap[np.maximum(o["kf_a"], 0)] >= 0))
    obs = o[keep].copy()
    gpk = gp[keep]
    obs["kf_b"] = kmap[obs["kf_b"]]
    obs["kf_a"] = np.where(gpk, kmap[np.maximum(obs["kf_a"], 0)], -1)
    lm_g = np.unique(obs["lm"])
    lmap = -np.ones(len(g.lm), np.int64)
    lmap[lm_g] = np.arange(lm_g.size)
    obs["lm"] = lmap[obs["lm"]]
    order = np.argsort(obs["lm"], kind="stable")
    obs = obs[order]
    kfs = g.kfs[ks].copy()
    kfs["fixed"] = 0
    kfs[0]["fixed"] = 1
    pri = np.zeros(max(n_opt - 1, 0), PRIOR_DTYPE)
    pri["kf_a"] = np.arange(1, n_opt)
    pri["kf_b"] = np.arange(2, n_opt + 1)
    return Window(kfs=kfs, lm=np.ascontiguousarray(g.lm[lm_g]), obs=obs, priors=pri,
                  vel_kfs=np.arange(1, n_opt + 1, dtype=np.int32), cams=g.cams.copy(), cfg=dict(g.cfg),
                  truth_lm=g.truth_lm[lm_g], name=name, lm_gid=lm_g, kf_gid=ks)
