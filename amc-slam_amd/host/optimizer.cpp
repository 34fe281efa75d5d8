// optimizer.cpp — Optimizer::LocalGPBA (src/Optimizer.cc:713-1432) on the GPU engine.
//
// Control flow, selection rules, thresholds and the float/double conversions follow the
// reference line by line (citations inline).  What changes is the engine: instead of
// g2o::SparseOptimizer the window becomes the flat arrays of include/amc_lba.h and runs through
// lba_set_problem / lba_optimize / lba_eval / lba_get_state on the GPU.
//
// Deliberate deviations (all are reference states that would dereference a null vertex):
//  * an observation whose keyframe is marked for this BA but was never added as a vertex (a bad
//    covisible KF, or a bad KF marked while collecting fixed KFs) is skipped;
//  * a GP observation whose mNextKF is not a vertex is skipped.
// Post-pass: chi2 values are those of the last computed errors (lba_trial_chi2: the last trial state,
// also when the run ended on rejected trials, like g2o's e->chi2()), the depth test runs on the final
// estimate (isDepthPositive reads the vertices, lba_eval).
#include "optimizer.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <unordered_map>
#include <unordered_set>

namespace amc_slam {

namespace {

lba_kf make_kf(MultiKeyFrame* K, bool fixed) {   // PoseVelocity(MultiKeyFrame*) (src/G2oTypes.cc:25-31)
    lba_kf v{};
    const SE3d Twb = SE3d::from_float(K->GetPoseInverse());
    std::memcpy(v.q, Twb.q, sizeof(v.q));
    std::memcpy(v.t, Twb.t, sizeof(v.t));
    for (int i = 0; i < 6; ++i) v.vel[i] = (double)K->GetVelocity()[i];
    v.time = K->mTimeStamp;
    v.bf = (double)K->mbf;
    v.fixed = fixed ? 1 : 0;
    return v;
}

}  // namespace

void Optimizer::BuildLocalGPBAWindow(MultiKeyFrame* pKF, bool bLarge, LocalGPBAWindow* W) {
    Map* pCurrentMap = pKF->GetMap();
    const int currentMapId = pKF->mMapId;
    const unsigned long id = pKF->mnId;

    // ---- temporal window (Optimizer.cc:717-748)
    const int maxOpt = bLarge ? 25 : 10;
    const int Nd = std::min((int)pCurrentMap->KeyFramesInMap() - 2, maxOpt);
    std::vector<MultiKeyFrame*>& vpOptimizableKFs = W->vpOptimizableKFs;
    const std::vector<MultiKeyFrame*> vpNeighsKFs = pKF->GetVectorCovisibleKeyFrames();
    vpOptimizableKFs.reserve(std::max(Nd, 1));
    vpOptimizableKFs.push_back(pKF);
    pKF->mnBALocalForKF = id;
    for (int i = 1; i < Nd; i++) {
        if (vpOptimizableKFs.back()->mPrevKF) {
            vpOptimizableKFs.push_back(vpOptimizableKFs.back()->mPrevKF);
            vpOptimizableKFs.back()->mnBALocalForKF = id;
        } else {
            break;
        }
    }
    int N = (int)vpOptimizableKFs.size();

    // ---- points seen by the temporal window (:750-767)
    std::vector<MapPoint*>& lLocalMapPoints = W->lLocalMapPoints;
    lLocalMapPoints.reserve(4096);
    auto collect = [&](MultiKeyFrame* K) {
        const std::vector<MapPoint*>& vpMPs = K->mvpMapPoints;   // GetMapPointMatches(), read in place
        for (MapPoint* pMP : vpMPs)
            if (pMP && !pMP->isBad() && pMP->mnBALocalForKF != id) {
                lLocalMapPoints.push_back(pMP);
                pMP->mnBALocalForKF = id;
            }
    };
    for (int i = 0; i < N; ++i) collect(vpOptimizableKFs[i]);

    // ---- fixed keyframe: the previous KF of the window (:769-782)
    std::vector<MultiKeyFrame*>& lFixedKeyFrames = W->lFixedKeyFrames;
    if (vpOptimizableKFs.back()->mPrevKF) {
        lFixedKeyFrames.push_back(vpOptimizableKFs.back()->mPrevKF);
        vpOptimizableKFs.back()->mPrevKF->mnBAFixedForKF = id;
    } else {
        vpOptimizableKFs.back()->mnBALocalForKF = 0;
        vpOptimizableKFs.back()->mnBAFixedForKF = id;
        lFixedKeyFrames.push_back(vpOptimizableKFs.back());
        vpOptimizableKFs.pop_back();
    }

    // ---- optimisable covisible KFs, maxCovKF = 0 admits one (:784-812)
    const size_t maxCovKF = 0;
    for (size_t i = 0, iend = vpNeighsKFs.size(); i < iend; ++i) {
        if (W->lpOptVisKFs.size() > maxCovKF) break;
        MultiKeyFrame* pKFi = vpNeighsKFs[i];
        if (pKFi->mnBALocalForKF == id || pKFi->mnBAFixedForKF == id) continue;
        pKFi->mnBALocalForKF = id;
        if (!pKFi->isBad() && pKFi->mMapId == currentMapId) {
            W->lpOptVisKFs.push_back(pKFi);
            collect(pKFi);
        }
    }

    // ---- fixed KFs observing the local points, at most 50 (:814-835)
    const size_t maxFixKF = 50;
    for (MapPoint* pMP : lLocalMapPoints) {
        const auto& observations = pMP->ObservationsRef();
        for (const auto& kv : observations) {
            MultiKeyFrame* pKFi = kv.first;
            if (pKFi->mnBALocalForKF != id && pKFi->mnBAFixedForKF != id) {
                pKFi->mnBAFixedForKF = id;
                if (!pKFi->isBad()) {
                    lFixedKeyFrames.push_back(pKFi);
                    break;
                }
            }
        }
        if (lFixedKeyFrames.size() >= maxFixKF) break;
    }

    // ---- vertices (:858-891).  g2o orders the Hessian by vertex id with non-marginalised
    //      vertices first (sparse_optimizer.cpp:166-190): keyframes by mnId, then points by mnId.
    N = (int)vpOptimizableKFs.size();
    std::vector<std::pair<MultiKeyFrame*, bool>> kv;   // (KF, fixed)
    for (MultiKeyFrame* K : vpOptimizableKFs) kv.push_back({K, false});
    for (MultiKeyFrame* K : W->lpOptVisKFs) kv.push_back({K, false});
    for (MultiKeyFrame* K : lFixedKeyFrames) kv.push_back({K, true});
    std::stable_sort(kv.begin(), kv.end(), [](const auto& a, const auto& b) { return a.first->mnId < b.first->mnId; });
    // a keyframe's vertex index is stamped on it with this build's number (no hash lookup per observation)
    static std::atomic<unsigned long> builds{0};
    const unsigned long stamp = ++builds;
    for (const auto& e : kv) {
        if (e.first->mnBAVertexStamp == stamp) continue;   // g2o addVertex refuses a duplicate id; the first one stays
        e.first->mnBAVertexStamp = stamp;
        e.first->mnBAVertex = (int)W->kfs.size();
        W->kfs.push_back(make_kf(e.first, e.second));
        W->kf_ids.push_back((int64_t)e.first->mnId);
    }
    auto vtx = [stamp](const MultiKeyFrame* K) { return K->mnBAVertexStamp == stamp ? K->mnBAVertex : -1; };

    // EdgeVelocity on every temporal KF (:866-871), EdgeGaussianPrior between neighbours (:894-906)
    for (int i = 0; i < N; ++i) W->vel_kfs.push_back(vtx(vpOptimizableKFs[i]));
    for (int i = N - 1; i > 0; --i) W->priors.push_back(lba_prior{vtx(vpOptimizableKFs[i]), vtx(vpOptimizableKFs[i - 1])});

    // cameras: MultiKeyFrame::mTbc[c].cast<double>() + Pinhole parameters (VertexExtrinsic, fixed, :982-995)
    // and the EdgeExtrinsicPrior of each: mRbc_ini[c].cast<double>(), information mRbc_ini_cov = 0.2 I
    // (src/Frame.cc:181-182); it only acts once the extrinsic is freed (bExtrinsic, :1228-1240)
    const std::vector<CameraParams>& cams = *pKF->mvpCamera;
    const int nCam = pKF->nCamera;
    for (int c = 0; c < nCam; ++c) {
        lba_cam lc{};
        const SE3d T = SE3d::from_float(cams[c].Tbc);
        std::memcpy(lc.q, T.q, sizeof(lc.q));
        std::memcpy(lc.t, T.t, sizeof(lc.t));
        lc.fx = cams[c].fx; lc.fy = cams[c].fy; lc.cx = cams[c].cx; lc.cy = cams[c].cy;
        for (int i = 0; i < 4; ++i) lc.rbc_ini[i] = (double)cams[c].Rbc_ini[i];
        for (int i = 0; i < 3; ++i) lc.rbc_info[4 * i] = 0.2;
        W->cams.push_back(lc);
    }

    // ---- point vertices and reprojection edges (:1012-1208)
    const std::vector<MapPoint*>& mps = lLocalMapPoints;
    std::vector<int> mp_order(mps.size());
    for (size_t i = 0; i < mps.size(); ++i) mp_order[i] = (int)i;
    std::stable_sort(mp_order.begin(), mp_order.end(), [&](int a, int b) { return mps[a]->mnId < mps[b]->mnId; });
    std::vector<int> lidx(mps.size());
    for (size_t r = 0; r < mp_order.size(); ++r) {
        MapPoint* P = mps[mp_order[r]];
        lidx[mp_order[r]] = (int)r;
        const Vec3f X = P->GetWorldPos();
        W->lm.push_back((double)X.x); W->lm.push_back((double)X.y); W->lm.push_back((double)X.z);
        W->mp_ids.push_back((int64_t)P->mnId);
        W->mp_vtx.push_back(P);
    }
    W->cam_obs.assign(nCam, 0);
    W->obs.reserve(8 * mps.size());
    W->obs_tag.reserve(8 * mps.size());
    W->rows.reserve(8 * mps.size());
    const float thHuberMono = std::sqrt(5.991);     // :975-978
    const float thHuberStereo = std::sqrt(7.815);
    auto add = [&](int tag, int kind, int ka, int kb, int lm, int cam, double t, double u, double v, double ur, float w,
                   MultiKeyFrame* K, MapPoint* P, const GPObs& g) {
        lba_obs o{};
        o.kind = kind; o.kf_a = ka; o.kf_b = kb; o.lm = lm; o.cam = cam; o.t = t;
        o.z[0] = u; o.z[1] = v; o.z[2] = ur;
        o.w = (double)w;
        W->obs.push_back(o);
        W->obs_tag.push_back(tag);
        W->rows.push_back(LocalGPBAWindow::Row{K, P, g, cam});
        W->n_edges[tag]++;
    };
    // the GP segments of the loop below, in its order (i = N-1 .. 1): keyframe, its vertex, its next keyframe's
    struct GPSeg { MultiKeyFrame* K; int a, b; };
    std::vector<GPSeg> segs;
    for (int i = (int)vpOptimizableKFs.size() - 1; i > 0; --i) {
        MultiKeyFrame* pKFi = vpOptimizableKFs[i];
        if (!pKFi->mNextKF) continue;
        const int a = vtx(pKFi), b = vtx(pKFi->mNextKF);
        if (b < 0) continue;
        segs.push_back({pKFi, a, b});
    }
    std::vector<std::pair<int, const GPObs*>> gp_hits;
    for (size_t m = 0; m < mps.size(); ++m) {
        MapPoint* pMP = mps[m];
        const int l = lidx[m];
        const auto& observations = pMP->ObservationsRef();
        const auto& observationsGP = pMP->GPObservationsRef();

        // GP observations of non-keyframes between pKFi and pKFi->mNextKF (:1027-1101).  The reference takes
        // equal_range(pKFi) for every segment i = N-1 .. 1; one pass over the point's entries, stably ordered by
        // segment, adds the same edges in the same order (a multimap keeps equal keys in insertion order)
        gp_hits.clear();
        for (const auto& e : observationsGP)
            for (size_t s = 0; s < segs.size(); ++s)
                if (segs[s].K == e.first) {
                    gp_hits.push_back({(int)s, &e.second});
                    break;
                }
        std::stable_sort(gp_hits.begin(), gp_hits.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
        for (const auto& h : gp_hits) {
            const GPSeg& sg = segs[h.first];
            MultiKeyFrame* pKFi = sg.K;
            const GPObs& g = *h.second;
            const float unc2 = cams[g.cam].uncertainty2();
            const float invSigma2 = (*pKFi->mvInvLevelSigma2)[g.obs.octave] / unc2;
            if (g.ur >= 0)
                add(1, LBA_STEREO_GP, sg.a, sg.b, l, g.cam, g.time, g.obs.x, g.obs.y, g.ur, invSigma2, pKFi, pMP, g);
            else
                add(0, LBA_MONO_GP, sg.a, sg.b, l, g.cam, g.time, g.obs.x, g.obs.y, 0.0, invSigma2, pKFi, pMP, g);
        }

        // keyframe observations (:1104-1206)
        for (const auto& kvo : observations) {
            MultiKeyFrame* pKFi = kvo.first;
            if (pKFi->mnBALocalForKF != id && pKFi->mnBAFixedForKF != id) continue;
            const int kb = vtx(pKFi);
            if (kb < 0) continue;   // marked but not a vertex (see header)
            const std::vector<int>& idxs = kvo.second;
            const int ncam = (int)idxs.size();
            for (int c = 0; c < ncam - 1; ++c) {
                const int idx = idxs[c];
                if (idx < 0) continue;
                MultiKeyFrame* pKFprev = pKFi->mPrevKF;
                if (!pKFprev) continue;
                if (pKFprev->mnBALocalForKF != id && pKFprev->mnBAFixedForKF != id) continue;
                const int ka = vtx(pKFprev);
                if (ka < 0) continue;
                const KeyPoint& kpUn = pKFi->mvKeysUn[idx];
                W->cam_obs[c]++;
                const float unc2 = cams[c].uncertainty2();
                const float invSigma2 = (*pKFi->mvInvLevelSigma2)[kpUn.octave] / unc2;
                add(4, LBA_MONO_GP, ka, kb, l, c, pKFi->mvTimeStamps[c], kpUn.x, kpUn.y, 0.0, invSigma2, pKFi, pMP, GPObs{});
            }
            const int c = ncam - 1;
            const int idx = idxs[c];
            if (idx < 0) continue;
            const KeyPoint kpUn = pKFi->mvKeysUn[idx];
            const float kp_ur = pKFi->mvuRight[idx];
            const float unc2 = cams[c].uncertainty2();
            const float invSigma2 = (*pKFi->mvInvLevelSigma2)[kpUn.octave] / unc2;
            if (kp_ur < 0)
                add(2, LBA_MONO, -1, kb, l, c, pKFi->mTimeStamp, kpUn.x, kpUn.y, 0.0, invSigma2, pKFi, pMP, GPObs{});
            else
                add(3, LBA_STEREO, -1, kb, l, c, pKFi->mTimeStamp, kpUn.x, kpUn.y, kp_ur, invSigma2, pKFi, pMP, GPObs{});
        }
    }

    // ---- optimiser settings (:838-856, 975-978)
    lba_config& cfg = W->cfg;
    std::memcpy(cfg.qc, pCurrentMap->mQc, sizeof(cfg.qc));
    cfg.huber_mono = (double)thHuberMono;
    cfg.huber_stereo = (double)thHuberStereo;
    cfg.huber_prior = 0.0;                     // no robust kernel on EdgeGaussianPrior (:902-904)
    cfg.lambda_init = bLarge ? 1e-2 : 1e0;
    cfg.tau = 1e-5;
    cfg.max_trials = 10;
    cfg.early_stop = 1;
}

int Optimizer::LocalGPBA(MultiKeyFrame* pKF, Map* pMap, const lbamap_options& opt, lba_problem* problem,
                         lbamap_result* out) {
    lbamap_result res{};
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](int k) {   // res.ms_phase[k] += the wall time since the previous lap
        const auto t = std::chrono::steady_clock::now();
        res.ms_phase[k] += std::chrono::duration<double, std::milli>(t - t_last).count();
        t_last = t;
    };
    const bool bLarge = opt.large != 0;
    const unsigned long id = pKF->mnId;
    LocalGPBAWindow W;
    BuildLocalGPBAWindow(pKF, bLarge, &W);
    lap(0);
    res.n_opt_kf = (int)W.vpOptimizableKFs.size();
    res.n_vis_kf = (int)W.lpOptVisKFs.size();
    res.n_fixed_kf = (int)W.lFixedKeyFrames.size();
    res.n_mp = (int)W.lLocalMapPoints.size();
    res.n_edges_mono_gp = W.n_edges[0];
    res.n_edges_stereo_gp = W.n_edges[1];
    res.n_edges_mono = W.n_edges[2];
    res.n_edges_stereo = W.n_edges[3];
    res.n_edges_mono_gp_kf = W.n_edges[4];

    // ---- optimise (:1221-1224): initializeOptimization, computeActiveErrors, activeRobustChi2, optimize(10)
    W.cfg.device = opt.device;
    W.cfg.flags = opt.flags;
    int rc = lba_set_config(problem, &W.cfg);
    if (rc >= 0)
        rc = lba_set_problem(problem, W.kfs.data(), (int)W.kfs.size(), W.lm.data(), (int)W.mp_ids.size(), W.obs.data(),
                             (int)W.obs.size(), W.priors.data(), (int)W.priors.size(), W.vel_kfs.data(),
                             (int)W.vel_kfs.size(), W.cams.data(), (int)W.cams.size());
    lap(1);
    lba_stats st{};
    if (rc >= 0) rc = lba_optimize(problem, 10, nullptr, &st);   // opt_it1 = 10 (:1218)
    lap(2);
    if (rc < 0) {
        res.status = rc;
        if (out) *out = res;
        return rc;
    }
    const float err = (float)st.chi2_initial;
    res.iterations = st.iterations;
    res.chi2_initial = st.chi2_initial;
    if (opt.extrinsic) {
        // :1228-1240: free the extrinsics of the cameras with >= extrin_thresh keyframe observations, then
        // initializeOptimization + computeActiveErrors + optimize(opt_it2) from the current estimate
        const int opt_it2 = bLarge ? 4 : 10;
        for (int c = 0; c < pKF->nCamera - 1; ++c)
            if (W.cam_obs[c] >= 50) W.cams[c].ext_free = 1;
        std::vector<lba_kf> kf_now(W.kfs.size());
        std::vector<double> lm_now(W.lm.size());
        rc = lba_get_state(problem, kf_now.data(), lm_now.data());
        if (rc >= 0)
            rc = lba_set_problem(problem, kf_now.data(), (int)kf_now.size(), lm_now.data(), (int)W.mp_ids.size(),
                                 W.obs.data(), (int)W.obs.size(), W.priors.data(), (int)W.priors.size(),
                                 W.vel_kfs.data(), (int)W.vel_kfs.size(), W.cams.data(), (int)W.cams.size());
        lap(1);
        if (rc >= 0) rc = lba_optimize(problem, opt_it2, nullptr, &st);
        lap(2);
        if (rc < 0) {
            res.status = rc;
            if (out) *out = res;
            return rc;
        }
        res.iterations += st.iterations;
    }
    res.chi2_final = st.chi2_final;
    const float err_end = (float)st.chi2_final;

    std::vector<double> chi2(W.obs.size());
    std::vector<uint8_t> depth_ok(W.obs.size());
    if (!W.obs.empty()) {
        rc = lba_trial_chi2(problem, chi2.data());
        if (rc >= 0) rc = lba_eval(problem, nullptr, nullptr, depth_ok.data());
        if (rc < 0) {
            res.status = rc;
            if (out) *out = res;
            return rc;
        }
    }

    // ---- outlier post-pass (:1257-1345), lists in the reference's order
    const float chi2Mono2 = 5.991f, chi2Stereo2 = 7.815f;
    struct EraseNKF { MultiKeyFrame* kf; MapPoint* mp; GPObs g; };
    struct Erase { MultiKeyFrame* kf; MapPoint* mp; int c; };
    std::vector<EraseNKF> vToEraseNKF;
    std::vector<Erase> vToErase;
    auto mono_out = [&](size_t i, int c) {
        const bool bClose = W.rows[i].mp->mvTrackDepth[c] < 10.f;
        return (chi2[i] > chi2Mono2 && !bClose) || (chi2[i] > 1.5f * chi2Mono2 && bClose) || !depth_ok[i];
    };
    for (int tag : {0, 1, 2, 3, 4}) {
        for (size_t i = 0; i < W.obs.size(); ++i) {
            if (W.obs_tag[i] != tag) continue;
            const LocalGPBAWindow::Row& r = W.rows[i];
            if (r.mp->isBad()) continue;
            switch (tag) {
                case 0: if (mono_out(i, r.gp.cam)) vToEraseNKF.push_back({r.kf, r.mp, r.gp}); break;
                case 1: if (chi2[i] > chi2Stereo2) vToEraseNKF.push_back({r.kf, r.mp, r.gp}); break;
                case 2: if (mono_out(i, pKF->nCamera - 1)) vToErase.push_back({r.kf, r.mp, pKF->nCamera - 1}); break;
                case 3: if (chi2[i] > chi2Stereo2) vToErase.push_back({r.kf, r.mp, pKF->nCamera - 1}); break;
                case 4:
                    if (mono_out(i, r.cam)) {
                        --W.cam_obs[r.cam];
                        vToErase.push_back({r.kf, r.mp, r.cam});
                    }
                    break;
            }
        }
    }
    res.n_erased_gp = (int)vToEraseNKF.size();
    res.n_erased = (int)vToErase.size();

    std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);
    // divergence guard (:1354-1358): nothing is written back
    if ((2 * err < err_end || std::isnan(err) || std::isnan(err_end)) && !bLarge) {
        res.status = LBA_E_DIVERGED;
        if (out) *out = res;
        return LBA_E_DIVERGED;
    }
    for (const EraseNKF& e : vToEraseNKF) e.mp->EraseGPObservation(e.kf, e.g);
    for (const Erase& e : vToErase) {
        const bool was_bad = e.mp->isBad();
        e.kf->EraseMapPointMatch(e.mp, e.c);
        e.mp->EraseObservation(e.kf, e.c);
        if (!was_bad && e.mp->isBad()) res.n_set_bad++;
    }
    for (MultiKeyFrame* K : W.lFixedKeyFrames) K->mnBAFixedForKF = 0;

    // ---- recover the estimates (:1384-1431)
    std::vector<lba_kf> kf_out(W.kfs.size());
    std::vector<double> lm_out(W.lm.size());
    rc = lba_get_state(problem, kf_out.data(), lm_out.data());
    if (rc < 0) {
        res.status = rc;
        if (out) *out = res;
        return rc;
    }
    std::unordered_map<unsigned long, int> row_of;
    for (size_t i = 0; i < W.kf_ids.size(); ++i) row_of[(unsigned long)W.kf_ids[i]] = (int)i;
    auto set_pose = [&](MultiKeyFrame* K) {   // SetPose(Twb.inverse().cast<float>())
        const lba_kf& v = kf_out[row_of[K->mnId]];
        SE3d Twb;
        std::memcpy(Twb.q, v.q, sizeof(Twb.q));
        std::memcpy(Twb.t, v.t, sizeof(Twb.t));
        K->SetPose(Twb.inverse().cast_float());
        K->mnBALocalForKF = 0;
    };
    for (int i = (int)W.vpOptimizableKFs.size() - 1; i >= 0; --i) set_pose(W.vpOptimizableKFs[i]);
    for (MultiKeyFrame* K : W.lpOptVisKFs) set_pose(K);
    for (size_t r = 0; r < W.mp_vtx.size(); ++r) {
        MapPoint* P = W.mp_vtx[r];
        P->SetWorldPos(Vec3f{(float)lm_out[3 * r], (float)lm_out[3 * r + 1], (float)lm_out[3 * r + 2]});
    }
    for (MapPoint* P : W.lLocalMapPoints) P->UpdateNormalAndDepth();   // in lLocalMapPoints order (:1412-1416)
    // extrinsics of the cameras that kept >= 50 observations: mTbc[c] = v->estimate().cast<float>()
    // (:1419-1428; a camera that was not freed round-trips its mTbc through double)
    std::vector<lba_cam> cam_out(W.cams.size());
    rc = lba_get_cams(problem, cam_out.data());
    if (rc < 0) {
        res.status = rc;
        if (out) *out = res;
        return rc;
    }
    for (int c = 0; c < pKF->nCamera - 1; ++c) {
        if (W.cam_obs[c] < 50) continue;
        SE3d T;
        std::memcpy(T.q, cam_out[c].q, sizeof(T.q));
        std::memcpy(T.t, cam_out[c].t, sizeof(T.t));
        pMap->mCameras[c].Tbc = T.cast_float();
    }
    pMap->IncreaseChangeIndex();
    (void)id;
    lap(3);
    res.status = LBA_OK;
    if (out) *out = res;
    return LBA_OK;
}

void Optimizer::LocalGPBA(MultiKeyFrame* pKF, bool* pbStopFlag, Map* pMap, int& num_fixedKF, int& num_OptKF, int& num_MPs,
                          int& num_edges, bool bLarge, bool bExtrinsic, bool bRecInit) {
    (void)pbStopFlag; (void)num_fixedKF; (void)num_OptKF; (void)num_MPs; (void)num_edges; (void)bRecInit;
    // one engine per mapping thread, reused across calls
    thread_local lba_problem* p = nullptr;
    if (!p) {
        lba_config cfg{};
        if (lba_create(&p, &cfg) != LBA_OK) { p = nullptr; return; }
    }
    lbamap_options opt{bLarge ? 1 : 0, bExtrinsic ? 1 : 0, 0, 0};
    const int rc = LocalGPBA(pKF, pMap, opt, p, nullptr);
    if (rc < 0)   // (the reference's void LocalGPBA has no status to return; the map stays untouched)
        std::fprintf(stderr, "LocalGPBA: local BA skipped (%d): %s\n", rc, lba_last_error(p));
}

}  // namespace amc_slam
