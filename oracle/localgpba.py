"""CPU restatement of Optimizer::LocalGPBA's host logic — TEST INFRASTRUCTURE ONLY.

Restates src/Optimizer.cc:713-1432 (window selection, graph shape, outlier post-pass, write-back)
and the map methods it calls (src/MapPoint.cc:196-337,356-386,611-686; src/KeyFrame.cc:116-145,
364-392) on a window snapshot (amc_lba.mapsnap.Snapshot), with the LM engine replaced by the C
oracle (oracle/lba_oracle.c via orc.Oracle).  tests/ compare the C++ adapter
(amc-slam_amd/host/, libamc_lba_map.so) against it: the flat window bit for bit, and after
LocalGPBA the erased observations, bad flags and written-back poses / points.

It is written independently of the product's adapter: plain dicts and lists, numpy float32 for the
reference's float arithmetic, the oracle's 12x12 GP query for the camera centres.
"""
import math

import numpy as np

import orc
from amc_lba.abi import CAM_DTYPE, KF_DTYPE, OBS_DTYPE, PRIOR_DTYPE, make_config
from amc_lba.synth import Window

F32 = np.float32
MONO_GP, STEREO_GP, MONO, STEREO = 0, 1, 2, 3
TAG_MONO_GP, TAG_STEREO_GP, TAG_MONO, TAG_STEREO, TAG_MONO_GP_KF = 0, 1, 2, 3, 4


# ------------------------------------------------------------------ Sophus float / double helpers
def _qn32(q):
    q = [F32(x) for x in q]
    n = np.sqrt(F32(F32(F32(q[0] * q[0]) + F32(q[1] * q[1])) + F32(q[2] * q[2])) + F32(q[3] * q[3]))
    return [F32(x / n) for x in q]


def _qn64(q):
    q = [float(x) for x in q]
    n = math.sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3])
    return [x / n for x in q]


def _rot(q, p):
    """so3.hpp:363-366 in the scalar type of q (p + w uv + v x uv, uv = 2 v x p)."""
    x, y, z, w = q
    uv = [y * p[2] - z * p[1], z * p[0] - x * p[2], x * p[1] - y * p[0]]
    uv = [a + a for a in uv]
    c = [y * uv[2] - z * uv[1], z * uv[0] - x * uv[2], x * uv[1] - y * uv[0]]
    return [(p[i] + w * uv[i]) + c[i] for i in range(3)]


def _inv(q, t, n):
    qi = n([-q[0], -q[1], -q[2], q[3]])
    return qi, _rot(qi, [-a for a in t])


def _mul(qa, ta, qb, tb, n):
    a, b = qa, qb
    w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2]
    x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1]
    y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2]
    z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0]
    r = _rot(qa, tb)
    return n([x, y, z, w]), [ta[i] + r[i] for i in range(3)]


def f2d(q, t):
    """Sophus SE3f::cast<double>()"""
    return _qn64(q), [float(a) for a in t]


def d2f(q, t):
    """Sophus SE3d::cast<float>()"""
    return _qn32(q), [F32(a) for a in t]


# ------------------------------------------------------------------ map model
class KF:
    def __init__(self, r, kps, n_cam, snap):
        self.id = int(r["id"])
        self.prev_id, self.next_id = int(r["prev_id"]), int(r["next_id"])
        self.time = float(r["time"])
        self.cam_time = [float(x) for x in r["cam_time"][:n_cam]]
        self.Tbw = ([F32(x) for x in r["q"]], [F32(x) for x in r["t"]])
        self.vel = [F32(x) for x in r["vel"]]
        self.bf = F32(r["bf"])
        self.bad = bool(r["bad"])
        self.map_id = int(r["map_id"])
        k = kps[int(r["kp_off"]): int(r["kp_off"]) + int(r["n_kp"])]
        self.kp_x, self.kp_y = list(k["x"]), list(k["y"])
        self.kp_oct, self.kp_cam, self.kp_ur = [int(x) for x in k["octave"]], [int(x) for x in k["cam"]], list(k["ur"])
        self.matches = [int(x) for x in k["mp_id"]]
        self.covis = [int(x) for x in snap.covis[int(r["covis_off"]): int(r["covis_off"]) + int(r["n_covis"])]]
        self.ba_local = 0
        self.ba_fixed = 0
        self.Twc = None
        if int(r["has_twc"]):   # the snapshot's cached camera poses (mTwc[c])
            self.Twc = [([F32(x) for x in r["twc_q"][c]], [F32(x) for x in r["twc_t"][c]]) for c in range(n_cam)]

    def Twb(self):   # GetPoseInverse (float)
        return _inv(*self.Tbw, _qn32)


class MP:
    def __init__(self, r, snap, n_cam, kfs):
        self.id = int(r["id"])
        self.pos = [F32(x) for x in r["pos"]]
        self.bad = bool(r["bad"])
        self.ref_kf = int(r["ref_kf"])
        self.track_depth = [F32(x) for x in r["track_depth"][:n_cam]]
        self.normal = [F32(x) for x in r["normal"]]
        self.min_dist, self.max_dist = F32(r["min_dist"]), F32(r["max_dist"])
        self.obs = {}
        self.nobs = 0
        for o in snap.mpobs[int(r["obs_off"]): int(r["obs_off"]) + int(r["n_obs"])]:
            k = int(o["kf_id"])
            idx = [int(x) for x in o["idx"][:n_cam]]
            self.obs[k] = idx
            for c, i in enumerate(idx):   # AddObservation nObs counting (src/MapPoint.cc:224-228)
                if i >= 0:
                    self.nobs += 2 if (c == n_cam - 1 and kfs[k].kp_ur[i] >= 0) else 1
        self.gp = [(int(g["kf_id"]), g.copy()) for g in snap.gpobs[int(r["gp_off"]): int(r["gp_off"]) + int(r["n_gp"])]]
        self.ba_local = 0


class PyMap:
    def __init__(self, snap):
        self.snap = snap
        self.n_cam = snap.n_cam
        self.kfs = {}
        for r in snap.kfs:
            k = KF(r, snap.kps, snap.n_cam, snap)
            self.kfs[k.id] = k
        self.mps = {}
        for r in snap.mps:
            m = MP(r, snap, snap.n_cam, self.kfs)
            self.mps[m.id] = m
        self.cams = [(list(c["q"]), list(c["t"]), c) for c in snap.cams]
        self.max_kf_id = max(self.kfs)
        self.qc = np.asarray(snap.qc, float)
        for kid in sorted(self.kfs):
            if self.kfs[kid].Twc is None:
                self.set_pose(self.kfs[kid], self.kfs[kid].Tbw)

    def kfs_in_map(self, map_id):
        return sum(1 for k in self.kfs.values() if not k.bad and k.map_id == map_id)

    # MultiKeyFrame::SetPose (src/KeyFrame.cc:116-145)
    def set_pose(self, K, Tbw):
        K.Tbw = Tbw
        Twb = _inv(*Tbw, _qn32)
        n = self.n_cam
        K.Twc = [([F32(0), F32(0), F32(0), F32(1)], [F32(0), F32(0), F32(0)])] * n   # identity until derived
        qbc, tbc = self.cams[n - 1][0], self.cams[n - 1][1]
        qcb, tcb = _inv([F32(x) for x in qbc], [F32(x) for x in tbc], _qn32)
        K.Twc[n - 1] = _inv(*_mul(qcb, tcb, *Tbw, _qn32), _qn32)
        if K.id == 0 or K.prev_id < 0:
            return
        P = self.kfs[K.prev_id]
        pq, pt = f2d(*_inv(*P.Tbw, _qn32))
        cq, ct = f2d(*Twb)
        for c in range(n - 1):
            qo, to, *_ = orc.gp_query_pose(self.qc, pq, pt, cq, ct, np.array(P.vel, float), np.array(K.vel, float),
                                           P.time, K.time, K.cam_time[c])
            fq, ft = d2f(qo, to)
            K.Twc[c] = _mul(fq, ft, [F32(x) for x in self.cams[c][0]], [F32(x) for x in self.cams[c][1]], _qn32)

    # MapPoint::EraseObservation(pKF, c) (src/MapPoint.cc:275-315) + MultiKeyFrame::EraseMapPointMatch
    def erase_obs(self, M, K, c):
        idx = M.obs.get(K.id)
        if idx is not None and idx[c] != -1:   # EraseMapPointMatch(pMP, c) (src/KeyFrame.cc:386-392)
            K.matches[idx[c]] = -1
        bad = False
        if idx is not None:
            idx = list(idx)
            if idx[c] != -1:
                M.nobs -= 1
                if c == self.n_cam - 1 and K.kp_ur[idx[c]] >= 0:
                    M.nobs -= 1
                idx[c] = -1
            if all(i == -1 for i in idx):
                del M.obs[K.id]
                if M.ref_kf == K.id:
                    M.ref_kf = min(M.obs) if M.obs else -1
            else:
                M.obs[K.id] = idx
            bad = M.nobs <= 2
        if bad:   # SetBadFlag (src/MapPoint.cc:356-386)
            M.bad = True
            for k, ii in M.obs.items():
                for i in ii:
                    if i != -1:
                        self.kfs[k].matches[i] = -1
            M.obs = {}

    def erase_gp_obs(self, M, kf_id, g):   # src/MapPoint.cc:323-337 (first equal entry)
        for j, (k, r) in enumerate(M.gp):
            if k == kf_id and r["time"] == g["time"] and r["cam"] == g["cam"] and r["x"] == g["x"] and \
                    r["y"] == g["y"] and r["ur"] == g["ur"]:
                del M.gp[j]
                return

    # MapPoint::UpdateNormalAndDepth (src/MapPoint.cc:611-686)
    def update_normal_and_depth(self, M):
        if M.bad or not M.obs:
            return
        normal = [F32(0), F32(0), F32(0)]
        n = 0
        for k in sorted(M.obs):
            for c in range(self.n_cam):
                if M.obs[k][c] != -1:
                    O = self.kfs[k].Twc[c][1]
                    d = [F32(M.pos[i] - O[i]) for i in range(3)]
                    nr = np.sqrt(F32(F32(d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]))
                    normal = [F32(normal[i] + F32(d[i] / nr)) for i in range(3)]
                    n += 1
        mx, mn = np.finfo(F32).tiny, np.finfo(F32).max
        if M.ref_kf in M.obs:
            R = self.kfs[M.ref_kf]
            sf = self.snap.scale_factor
            for c in range(self.n_cam):
                i = M.obs[M.ref_kf][c]
                if i != -1:
                    O = R.Twc[c][1]
                    d = [F32(M.pos[j] - O[j]) for j in range(3)]
                    dist = np.sqrt(F32(F32(d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]))
                    lsf = sf[R.kp_oct[i]]
                    mx = max(mx, F32(dist * lsf))
                    mn = min(mn, F32(F32(dist * lsf) / sf[len(sf) - 1]))
        M.max_dist, M.min_dist = F32(mx), F32(mn)
        M.normal = [F32(normal[i] / F32(n)) for i in range(3)]

    def to_snapshot(self):
        s = self.snap.copy()
        for r in s.kfs:
            K = self.kfs[int(r["id"])]
            r["q"], r["t"] = K.Tbw[0], K.Tbw[1]
            r["has_twc"] = 1
            for c in range(self.n_cam):
                r["twc_q"][c], r["twc_t"][c] = K.Twc[c][0], K.Twc[c][1]
            s.kps["mp_id"][int(r["kp_off"]): int(r["kp_off"]) + int(r["n_kp"])] = K.matches
        mo, go = [], []
        for r in s.mps:
            M = self.mps[int(r["id"])]
            r["pos"], r["bad"], r["ref_kf"] = M.pos, int(M.bad), M.ref_kf
            r["normal"], r["min_dist"], r["max_dist"] = M.normal, M.min_dist, M.max_dist
            r["obs_off"], r["n_obs"] = len(mo), len(M.obs)
            for k in sorted(M.obs):
                mo.append((k, M.obs[k]))
            r["gp_off"], r["n_gp"] = len(go), len(M.gp)
            go.extend(g for _, g in sorted(M.gp, key=lambda kg: kg[0]))   # multimap order: by KF, stable
        s.mpobs = np.zeros(len(mo), s.mpobs.dtype)
        if mo:
            s.mpobs["kf_id"] = [k for k, _ in mo]
            idx = np.full((len(mo), s.mpobs["idx"].shape[1]), -1, np.int32)
            for i, (_, ii) in enumerate(mo):
                idx[i, : len(ii)] = ii
            s.mpobs["idx"] = idx
        s.gpobs = np.array(go, dtype=s.gpobs.dtype) if go else np.zeros(0, s.gpobs.dtype)
        return s


# ------------------------------------------------------------------ LocalGPBA
class WindowBuild:
    pass


def build_window(pm, kf_id, large=False):
    """src/Optimizer.cc:713-1208 on PyMap pm (mutates the BA flags like the reference)."""
    W = WindowBuild()
    pKF = pm.kfs[kf_id]
    mid = pKF.id
    max_opt = 25 if large else 10
    Nd = min(pm.kfs_in_map(pKF.map_id) - 2, max_opt)
    opt = [pKF]
    pKF.ba_local = mid
    for _ in range(1, Nd):
        b = opt[-1]
        if b.prev_id >= 0:
            opt.append(pm.kfs[b.prev_id])
            opt[-1].ba_local = mid
        else:
            break
    local_mps = []

    def collect(K):
        for m in K.matches:
            if m < 0:
                continue
            M = pm.mps[m]
            if not M.bad and M.ba_local != mid:
                local_mps.append(M)
                M.ba_local = mid

    for K in opt:
        collect(K)
    fixed = []
    if opt[-1].prev_id >= 0:
        P = pm.kfs[opt[-1].prev_id]
        fixed.append(P)
        P.ba_fixed = mid
    else:
        opt[-1].ba_local = 0
        opt[-1].ba_fixed = mid
        fixed.append(opt.pop())
    vis = []
    for c in pKF.covis:
        if len(vis) > 0:
            break
        K = pm.kfs[c]
        if K.ba_local == mid or K.ba_fixed == mid:
            continue
        K.ba_local = mid
        if not K.bad and K.map_id == pKF.map_id:
            vis.append(K)
            collect(K)
    for M in local_mps:
        for k in sorted(M.obs):
            K = pm.kfs[k]
            if K.ba_local != mid and K.ba_fixed != mid:
                K.ba_fixed = mid
                if not K.bad:
                    fixed.append(K)
                    break
        if len(fixed) >= 50:
            break

    verts = sorted([(K, False) for K in opt] + [(K, False) for K in vis] + [(K, True) for K in fixed],
                   key=lambda e: e[0].id)
    kidx, kfs, kf_ids = {}, [], []
    for K, fx in verts:
        if K.id in kidx:
            continue
        kidx[K.id] = len(kfs)
        q, t = f2d(*K.Twb())
        r = np.zeros(1, KF_DTYPE)[0]
        r["q"], r["t"], r["vel"] = q, t, [float(v) for v in K.vel]
        r["time"], r["bf"], r["fixed"] = K.time, float(K.bf), int(fx)
        kfs.append(r)
        kf_ids.append(K.id)
    vel = [kidx[K.id] for K in opt]
    pri = [(kidx[opt[i].id], kidx[opt[i - 1].id]) for i in range(len(opt) - 1, 0, -1)]
    cams = np.zeros(pm.n_cam, CAM_DTYPE)
    for c, (q, t, rec) in enumerate(pm.cams):
        cams[c]["q"], cams[c]["t"] = f2d([F32(x) for x in q], [F32(x) for x in t])
        for f in ("fx", "fy", "cx", "cy"):
            cams[c][f] = float(rec[f])
        # EdgeExtrinsicPrior(mRbc_ini[c].cast<double>()), information mRbc_ini_cov = 0.2 I (Frame.cc:181-182)
        cams[c]["rbc_ini"] = [float(x) for x in rec["rbc_ini"]]
        cams[c]["rbc_info"] = (0.2 * np.eye(3)).ravel()

    mp_sorted = sorted(local_mps, key=lambda M: M.id)
    lidx = {M.id: i for i, M in enumerate(mp_sorted)}
    lm = np.array([[float(x) for x in M.pos] for M in mp_sorted]).reshape(-1, 3)
    inv_s2 = pm.snap.inv_level_sigma2
    rows, obs, tags = [], [], []
    cam_obs = [0] * pm.n_cam

    def add(tag, kind, ka, kb, l, cam, t, u, v, ur, w, K, M, g):
        obs.append((kind, ka, kb, l, cam, t, float(u), float(v), float(ur), float(w)))
        tags.append(tag)
        rows.append((K, M, g, cam))

    n = pm.n_cam
    for M in local_mps:
        l = lidx[M.id]
        for i in range(len(opt) - 1, 0, -1):
            K = opt[i]
            if K.next_id < 0 or K.next_id not in kidx:
                continue
            for k, g in M.gp:
                if k != K.id:
                    continue
                w = F32(inv_s2[int(g["octave"])] / F32(1.0))
                if g["ur"] >= 0:
                    add(TAG_STEREO_GP, STEREO_GP, kidx[K.id], kidx[K.next_id], l, int(g["cam"]), float(g["time"]),
                        g["x"], g["y"], g["ur"], w, K, M, g)
                else:
                    add(TAG_MONO_GP, MONO_GP, kidx[K.id], kidx[K.next_id], l, int(g["cam"]), float(g["time"]),
                        g["x"], g["y"], 0.0, w, K, M, g)
        for k in sorted(M.obs):
            K = pm.kfs[k]
            if K.ba_local != mid and K.ba_fixed != mid:
                continue
            if K.id not in kidx:
                continue
            idxs = M.obs[k]
            for c in range(n - 1):
                i = idxs[c]
                if i < 0 or K.prev_id < 0:
                    continue
                P = pm.kfs[K.prev_id]
                if P.ba_local != mid and P.ba_fixed != mid:
                    continue
                if P.id not in kidx:
                    continue
                cam_obs[c] += 1
                w = F32(inv_s2[K.kp_oct[i]] / F32(1.0))
                add(TAG_MONO_GP_KF, MONO_GP, kidx[P.id], kidx[K.id], l, c, K.cam_time[c], K.kp_x[i], K.kp_y[i], 0.0, w,
                    K, M, None)
            i = idxs[n - 1]
            if i < 0:
                continue
            w = F32(inv_s2[K.kp_oct[i]] / F32(1.0))
            if K.kp_ur[i] < 0:
                add(TAG_MONO, MONO, -1, kidx[K.id], l, n - 1, K.time, K.kp_x[i], K.kp_y[i], 0.0, w, K, M, None)
            else:
                add(TAG_STEREO, STEREO, -1, kidx[K.id], l, n - 1, K.time, K.kp_x[i], K.kp_y[i], K.kp_ur[i], w, K, M,
                    None)

    o = np.zeros(len(obs), OBS_DTYPE)
    for j, (kind, ka, kb, l, cam, t, u, v, ur, w) in enumerate(obs):
        o[j]["kind"], o[j]["kf_a"], o[j]["kf_b"], o[j]["lm"], o[j]["cam"] = kind, ka, kb, l, cam
        o[j]["t"], o[j]["z"], o[j]["w"] = t, (u, v, ur), w
    priors = np.zeros(len(pri), PRIOR_DTYPE)
    if pri:
        priors["kf_a"] = [a for a, _ in pri]
        priors["kf_b"] = [b for _, b in pri]
    cfg = {"qc_diag": pm.qc, "huber_prior": 0.0, "lambda_init": 1e-2 if large else 1.0}
    W.win = Window(kfs=np.array(kfs, KF_DTYPE), lm=np.ascontiguousarray(lm), obs=o, priors=priors,
                   vel_kfs=np.array(vel, np.int32), cams=cams, cfg=cfg, name=f"oracle_localgpba_{kf_id}")
    W.kf_ids, W.mp_ids, W.tags = np.array(kf_ids, np.int64), np.array([M.id for M in mp_sorted], np.int64), \
        np.array(tags, np.int32)
    W.opt, W.vis, W.fixed, W.local_mps, W.rows, W.cam_obs = opt, vis, fixed, local_mps, rows, cam_obs
    return W


def local_gpba(snap, kf_id, large=False, iters=10, extrinsic=False):
    """Full LocalGPBA on a copy of `snap` with the C oracle as the engine.  Returns
    (status, new_snapshot, info)."""
    pm = PyMap(snap.copy())
    W = build_window(pm, kf_id, large)
    o = orc.Oracle(W.win, cfg=make_config(**W.win.cfg))
    n_it, st = o.optimize(iters)
    err = F32(st.chi2_initial)
    chi2_initial = st.chi2_initial
    if extrinsic:
        # bExtrinsic (:1228-1240): cameras with >= 50 keyframe observations get a free VertexExtrinsic;
        # initializeOptimization / computeActiveErrors / optimize(opt_it2) from the current estimate
        kfs, lm = o.state()
        cams = W.win.cams.copy()
        for c in range(pm.n_cam - 1):
            if W.cam_obs[c] >= 50:
                cams[c]["ext_free"] = 1
        W.win = Window(kfs=kfs, lm=lm, obs=W.win.obs, priors=W.win.priors, vel_kfs=W.win.vel_kfs, cams=cams,
                       cfg=W.win.cfg, name=W.win.name + "_ext")
        o = orc.Oracle(W.win, cfg=make_config(**W.win.cfg))
        n2, st = o.optimize(4 if large else 10)
        n_it += n2
    chi2 = o.last_obs_chi2()   # g2o's e->chi2(): the last computeActiveErrors (last trial state)
    depth = o.depth_ok()
    err_end = F32(st.chi2_final)
    n = pm.n_cam
    chi2_mono, chi2_stereo = F32(5.991), F32(7.815)

    def mono_out(i, c):
        close = W.rows[i][1].track_depth[c] < F32(10.0)
        return (chi2[i] > float(chi2_mono) and not close) or (chi2[i] > float(F32(1.5) * chi2_mono) and close) or \
            not depth[i]

    erase_nkf, erase = [], []
    for tag in range(5):
        for i, t in enumerate(W.tags):
            if t != tag:
                continue
            K, M, g, cam = W.rows[i]
            if M.bad:
                continue
            if tag == TAG_MONO_GP and mono_out(i, int(g["cam"])):
                erase_nkf.append((K, M, g))
            elif tag == TAG_STEREO_GP and chi2[i] > float(chi2_stereo):
                erase_nkf.append((K, M, g))
            elif tag == TAG_MONO and mono_out(i, n - 1):
                erase.append((K, M, n - 1))
            elif tag == TAG_STEREO and chi2[i] > float(chi2_stereo):
                erase.append((K, M, n - 1))
            elif tag == TAG_MONO_GP_KF and mono_out(i, cam):
                W.cam_obs[cam] -= 1
                erase.append((K, M, cam))
    info = {"window": W, "iterations": n_it, "chi2_initial": chi2_initial, "chi2_final": st.chi2_final,
            "chi2": chi2, "depth_ok": depth, "n_erased_gp": len(erase_nkf), "n_erased": len(erase)}
    if (F32(2) * err < err_end or np.isnan(err) or np.isnan(err_end)) and not large:
        return -3, snap.copy(), info
    for K, M, g in erase_nkf:
        pm.erase_gp_obs(M, K.id, g)
    n_bad = 0
    for K, M, c in erase:
        was = M.bad
        pm.erase_obs(M, K, c)
        n_bad += int(M.bad and not was)
    info["n_set_bad"] = n_bad
    kfs, lm = o.state()
    row = {k: i for i, k in enumerate(W.kf_ids)}

    def set_pose(K):
        v = kfs[row[K.id]]
        q, t = _inv(list(v["q"]), list(v["t"]), _qn64)
        pm.set_pose(K, d2f(q, t))

    for K in reversed(W.opt):
        set_pose(K)
    for K in W.vis:
        set_pose(K)
    for r, mid in enumerate(W.mp_ids):
        pm.mps[int(mid)].pos = [F32(x) for x in lm[r]]
    for M in W.local_mps:
        pm.update_normal_and_depth(M)
    snap_out = pm.to_snapshot()
    est = o.cams()
    for c in range(n - 1):   # extrinsics with >= 50 observations: mTbc = v->estimate().cast<float>() (:1419-1428)
        if W.cam_obs[c] >= 50:
            q, t = d2f(list(est[c]["q"]), list(est[c]["t"]))
            snap_out.cams[c]["q"], snap_out.cams[c]["t"] = q, t
    return 0, snap_out, info
