"""CPU restatement of Optimizer::BundleAdjustment / GlobalBundleAdjustemnt — TEST INFRASTRUCTURE ONLY.

Restates src/Optimizer.cc:53-367 (the global BA graph over every keyframe and map point of a map, the
write-back, the loop-closure variant that holds the results back in mTbwGBA / mVwbGBA / mPosGBA) on a
window snapshot, with the C oracle (oracle/lba_oracle.c via orc.Oracle) as the engine, over the map
model of oracle/localgpba.py.  tests/ compare the C++ adapter (amc-slam_amd/host/bundle_adjustment.cpp,
lbamap_global_ba) against it: the flat graph bit for bit, and after the optimisation the written-back
poses, velocities and points.  Written independently of the adapter: dicts and lists, numpy float32 for
the reference's float arithmetic.
"""
import numpy as np

import orc
from amc_lba.abi import CAM_DTYPE, KF_DTYPE, OBS_DTYPE, PRIOR_DTYPE, make_config
from amc_lba.synth import Window
from localgpba import (F32, MONO, MONO_GP, STEREO, STEREO_GP, TAG_MONO, TAG_MONO_GP, TAG_MONO_GP_KF, TAG_STEREO,
                       TAG_STEREO_GP, PyMap, _inv, _qn64, d2f, f2d)


class BAGraph:
    pass


def all_keyframes(pm, map_id=0):
    """Map::GetAllKeyFrames: the map's (non-erased) keyframes."""
    return [pm.kfs[k] for k in sorted(pm.kfs) if not pm.kfs[k].bad and pm.kfs[k].map_id == map_id]


def all_map_points(pm):
    return [pm.mps[m] for m in sorted(pm.mps) if not pm.mps[m].bad]


def init_kf_id(pm, map_id=0):
    return min(k.id for k in pm.kfs.values() if k.map_id == map_id)


def build_ba_graph(pm, vpKFs, vpMP):
    """src/Optimizer.cc:61-292 on PyMap pm."""
    G = BAGraph()
    init = init_kf_id(pm)
    verts = sorted([K for K in vpKFs if not K.bad], key=lambda K: K.id)
    max_id = max((K.id for K in verts), default=0)
    kidx, kfs, kf_ids = {}, [], []
    for K in verts:                                   # VertexPoseVel, fixed = the map's initial KF (:84-97)
        if K.id in kidx:
            continue
        kidx[K.id] = len(kfs)
        q, t = f2d(*K.Twb())
        r = np.zeros(1, KF_DTYPE)[0]
        r["q"], r["t"], r["vel"] = q, t, [float(v) for v in K.vel]
        r["time"], r["bf"], r["fixed"] = K.time, float(K.bf), int(K.id == init)
        kfs.append(r)
        kf_ids.append(K.id)
    vel, pri = [], []
    for K in vpKFs:                                   # EdgeVelocity, EdgeGaussianPrior (:100-135)
        if K.id not in kidx or K.bad:
            continue
        vel.append(kidx[K.id])
        if K.prev_id < 0:
            continue
        if K.id <= max_id:
            P = pm.kfs[K.prev_id]
            if K.bad or P.id > max_id or P.id not in kidx or P.bad:
                continue
            pri.append((kidx[P.id], kidx[K.id]))
    cams = np.zeros(pm.n_cam, CAM_DTYPE)
    for c, (q, t, rec) in enumerate(pm.cams):
        cams[c]["q"], cams[c]["t"] = f2d([F32(x) for x in q], [F32(x) for x in t])
        for f in ("fx", "fy", "cx", "cy"):
            cams[c][f] = float(rec[f])
        cams[c]["rbc_ini"] = [float(x) for x in rec["rbc_ini"]]
        cams[c]["rbc_info"] = (0.2 * np.eye(3)).ravel()

    inv_s2 = pm.snap.inv_level_sigma2
    n = pm.n_cam
    kept = []                                         # (point, its edges)
    for M in vpMP:                                    # points and their edges (:143-292)
        E = []
        n_edges = 0
        for k in sorted(M.obs):
            K = pm.kfs[k]
            if K.bad or K.id > max_id or K.id not in kidx:
                continue
            n_edges += 1
            idxs = M.obs[k]
            if K.prev_id >= 0 and K.prev_id <= max_id:
                for c in range(len(idxs) - 1):
                    i = idxs[c]
                    if i < 0 or K.prev_id not in kidx:
                        continue
                    w = F32(inv_s2[K.kp_oct[i]])
                    E.append((TAG_MONO_GP_KF, MONO_GP, kidx[K.prev_id], kidx[K.id], c, K.cam_time[c], K.kp_x[i],
                              K.kp_y[i], 0.0, w))
            i = idxs[len(idxs) - 1]
            if i >= 0:
                w = F32(inv_s2[K.kp_oct[i]])
                if K.kp_ur[i] < 0:
                    E.append((TAG_MONO, MONO, -1, kidx[K.id], n - 1, K.time, K.kp_x[i], K.kp_y[i], 0.0, w))
                else:
                    E.append((TAG_STEREO, STEREO, -1, kidx[K.id], n - 1, K.time, K.kp_x[i], K.kp_y[i], K.kp_ur[i], w))
        for K in vpKFs:
            if K.bad or K.next_id < 0 or K.id > max_id or K.next_id > max_id:
                continue
            if K.id not in kidx or K.next_id not in kidx:
                continue
            for k, g in M.gp:
                if k != K.id:
                    continue
                w = F32(inv_s2[int(g["octave"])])
                if g["ur"] >= 0:
                    E.append((TAG_STEREO_GP, STEREO_GP, kidx[K.id], kidx[K.next_id], int(g["cam"]), float(g["time"]),
                              g["x"], g["y"], g["ur"], w))
                else:
                    E.append((TAG_MONO_GP, MONO_GP, kidx[K.id], kidx[K.next_id], int(g["cam"]), float(g["time"]),
                              g["x"], g["y"], 0.0, w))
        if n_edges > 0:
            kept.append((M, E))
    kept.sort(key=lambda me: me[0].id)
    rows, tags = [], []
    for l, (M, E) in enumerate(kept):
        for tag, kind, ka, kb, cam, t, u, v, ur, w in E:
            rows.append((kind, ka, kb, l, cam, t, float(u), float(v), float(ur), float(w)))
            tags.append(tag)
    o = np.zeros(len(rows), OBS_DTYPE)
    for j, (kind, ka, kb, l, cam, t, u, v, ur, w) in enumerate(rows):
        o[j]["kind"], o[j]["kf_a"], o[j]["kf_b"], o[j]["lm"], o[j]["cam"] = kind, ka, kb, l, cam
        o[j]["t"], o[j]["z"], o[j]["w"] = t, (u, v, ur), w
    priors = np.zeros(len(pri), PRIOR_DTYPE)
    if pri:
        priors["kf_a"] = [a for a, _ in pri]
        priors["kf_b"] = [b for _, b in pri]
    lm = np.array([[float(x) for x in M.pos] for M, _ in kept]).reshape(-1, 3)
    cfg = {"qc_diag": pm.qc, "huber_prior": 21.026, "lambda_init": 1e-5,
           "huber_mono": float(F32(np.sqrt(5.991))), "huber_stereo": float(F32(np.sqrt(7.815)))}
    G.win = Window(kfs=np.array(kfs, KF_DTYPE), lm=np.ascontiguousarray(lm), obs=o, priors=priors,
                   vel_kfs=np.array(vel, np.int32), cams=cams, cfg=cfg, name="oracle_global_ba")
    G.kf_ids = np.array(kf_ids, np.int64)
    G.mp_ids = np.array([M.id for M, _ in kept], np.int64)
    G.tags = np.array(tags, np.int32)
    G.included = {M.id for M, _ in kept}
    return G


def global_ba(snap, iters=10, loop_kf=0):
    """GlobalBundleAdjustemnt on a copy of `snap` with the C oracle as the engine.  Returns
    (status, new_snapshot, info); info["gba"] holds the loop-closure results when loop_kf != 0."""
    pm = PyMap(snap.copy())
    vpKFs, vpMP = all_keyframes(pm), all_map_points(pm)
    G = build_ba_graph(pm, vpKFs, vpMP)
    o = orc.Oracle(G.win, cfg=make_config(**G.win.cfg))
    n_it, st = o.optimize(iters)
    kfs, lm = o.state()
    row = {k: i for i, k in enumerate(G.kf_ids)}
    info = {"graph": G, "iterations": n_it, "chi2_initial": st.chi2_initial, "chi2_final": st.chi2_final,
            "gba_kf": {}, "gba_mp": {}}
    for K in vpKFs:                                   # (:300-326)
        if K.bad or K.id not in row:
            continue
        v = kfs[row[K.id]]
        Tbw = d2f(*_inv(list(v["q"]), list(v["t"]), _qn64))
        vel = [F32(x) for x in v["vel"]]
        if loop_kf == 0:
            pm.set_pose(K, Tbw)
            K.vel = vel
        else:
            info["gba_kf"][K.id] = (Tbw, vel)
    prow = {m: i for i, m in enumerate(G.mp_ids)}
    for M in vpMP:                                    # (:328-345)
        if M.id not in G.included:
            continue
        pos = [F32(x) for x in lm[prow[M.id]]]
        if loop_kf == 0:
            M.pos = pos
            pm.update_normal_and_depth(M)
        else:
            info["gba_mp"][M.id] = pos
    out = pm.to_snapshot()
    for r in out.kfs:   # SetVelocity (the LocalGPBA restatement never writes velocities)
        r["vel"] = pm.kfs[int(r["id"])].vel
    return 0, out, info
