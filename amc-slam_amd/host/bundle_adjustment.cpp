// bundle_adjustment.cpp — Optimizer::BundleAdjustment / GlobalBundleAdjustemnt (src/Optimizer.cc:53-367)
// on the GPU engine.
//
// The graph follows the reference line by line (citations inline): keyframe vertices (the map's initial
// keyframe fixed), EdgeVelocity on every keyframe, EdgeGaussianPrior between consecutive keyframes with
// a Huber kernel of 21.026, and per map point its keyframe observations (EdgeMonoGP from the previous
// keyframe for the asynchronous cameras, EdgeMono / EdgeStereo for the reference camera) and its GP
// observations of non-keyframes (EdgeMonoGP / EdgeStereoGP); a point with no keyframe observation is
// removed again.  g2o's SparseOptimizer + BlockSolverX + LinearSolverEigen + Levenberg (lambda0 1e-5,
// :66-76) becomes one lba_problem: the reduced camera system is solved by k_chol_flow's band path above
// 64 panels.
//
// Deliberate deviations (reference states that depend on pointer order or would touch a null vertex):
//  * keyframe and observation maps iterate by keyframe id (the reference's std::set / std::map of
//    pointers iterate by address), which only changes the order of the edges;
//  * an edge whose vertex is missing (a bad previous / next keyframe) is not added: g2o's addEdge
//    refuses an edge with a null vertex, so the reference ends the same way;
//  * a point listed twice in vpMP is added once (g2o's addVertex refuses the duplicate id).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "optimizer.hpp"

namespace amc_slam {

namespace {

lba_kf kf_vertex(MultiKeyFrame* K, bool fixed) {   // VertexPoseVel(pKF): PoseVelocity (src/G2oTypes.cc:25-31)
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

void Optimizer::BuildBundleAdjustmentWindow(const std::vector<MultiKeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                                            BundleAdjustmentWindow* W) {
    if (vpKFs.empty()) return;
    Map* pMap = vpKFs[0]->GetMap();   // (:64)
    const unsigned long initKF = pMap->GetInitKFid();

    // ---- keyframe vertices (:84-97), in g2o's Hessian order (by id)
    unsigned long maxKFid = 0;
    std::vector<MultiKeyFrame*> kv;
    for (MultiKeyFrame* K : vpKFs) {
        if (K->isBad()) continue;
        kv.push_back(K);
        maxKFid = std::max(maxKFid, K->mnId);
    }
    std::stable_sort(kv.begin(), kv.end(), [](const MultiKeyFrame* a, const MultiKeyFrame* b) { return a->mnId < b->mnId; });
    std::unordered_map<const MultiKeyFrame*, int> kidx;
    std::unordered_set<unsigned long> ids;
    for (MultiKeyFrame* K : kv) {
        if (!ids.insert(K->mnId).second) continue;   // a duplicate id: g2o keeps the first vertex
        kidx[K] = (int)W->kfs.size();
        const bool fixed = K->mnId == initKF;
        W->n_fixed += fixed;
        W->kfs.push_back(kf_vertex(K, fixed));
        W->kf_ids.push_back((int64_t)K->mnId);
        W->kf_vtx.push_back(K);
    }
    auto vtx = [&](const MultiKeyFrame* K) {
        if (!K) return -1;
        auto it = kidx.find(K);
        return it == kidx.end() ? -1 : it->second;
    };

    // ---- EdgeVelocity on every keyframe, EdgeGaussianPrior (prev, KF) with Huber 21.026 (:100-135)
    for (MultiKeyFrame* K : vpKFs) {
        const int v = vtx(K);
        if (v < 0) continue;   // (a bad keyframe has no vertex: the edge is refused)
        W->vel_kfs.push_back(v);
        if (!K->mPrevKF) continue;
        if (K->mnId <= maxKFid) {
            if (K->isBad() || K->mPrevKF->mnId > maxKFid) continue;
            const int a = vtx(K->mPrevKF);
            if (a < 0) continue;
            W->priors.push_back(lba_prior{a, v});
        }
    }

    // cameras: MultiKeyFrame::mTbc (EdgeMonoGP reads the static extrinsics) + Pinhole parameters
    const std::vector<CameraParams>& cams = *vpKFs[0]->mvpCamera;
    const int nCam = vpKFs[0]->nCamera;
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

    // ---- point vertices and their edges (:137-282)
    const float thHuberMono = std::sqrt(5.991);    // :137-138
    const float thHuberStereo = std::sqrt(7.815);
    struct Pending {
        lba_obs o;
        int tag;
    };
    std::vector<std::vector<Pending>> per_point;
    std::vector<MapPoint*> pts;
    std::vector<int> pt_of(vpMP.size(), -1);
    std::unordered_map<const MapPoint*, int> seen;
    std::unordered_multimap<const MultiKeyFrame*, int> kf_pos;   // keyframe -> its positions in vpKFs
    for (size_t k = 0; k < vpKFs.size(); ++k) kf_pos.emplace(vpKFs[k], (int)k);
    for (size_t i = 0; i < vpMP.size(); ++i) {
        MapPoint* pMP = vpMP[i];
        if (!pMP || seen.count(pMP)) continue;
        seen[pMP] = (int)i;
        std::vector<Pending> E;
        auto add = [&](int tag, int kind, int ka, int kb, int cam, double t, double u, double v, double ur, float w) {
            lba_obs o{};
            o.kind = kind; o.kf_a = ka; o.kf_b = kb; o.lm = -1; o.cam = cam; o.t = t;
            o.z[0] = u; o.z[1] = v; o.z[2] = ur;
            o.w = (double)w;
            E.push_back(Pending{o, tag});
        };
        int nEdges = 0;
        const auto& observations = pMP->ObservationsRef();
        const auto& observationsGP = pMP->GPObservationsRef();
        for (const auto& kvo : observations) {   // keyframe observations (:157-232)
            MultiKeyFrame* pKFi = kvo.first;
            if (pKFi->isBad() || pKFi->mnId > maxKFid) continue;
            const int kb = vtx(pKFi);
            if (kb < 0) continue;
            nEdges++;
            const std::vector<int>& idxs = kvo.second;
            const int ncam = (int)idxs.size();
            if (pKFi->mPrevKF != nullptr && pKFi->mPrevKF->mnId <= maxKFid) {
                const int ka = vtx(pKFi->mPrevKF);
                for (int c = 0; c < ncam - 1; ++c) {
                    const int index = idxs[c];
                    if (index < 0 || ka < 0) continue;
                    const KeyPoint& kp = pKFi->mvKeysUn[index];
                    const float invSigma2 = (*pKFi->mvInvLevelSigma2)[kp.octave];
                    add(4, LBA_MONO_GP, ka, kb, c, pKFi->mvTimeStamps[c], kp.x, kp.y, 0.0, invSigma2);
                }
            }
            const int c = ncam - 1;
            const int index = idxs[c];
            if (index >= 0) {
                const float kp_ur = pKFi->mvuRight[index];
                const KeyPoint kpUn = pKFi->mvKeysUn[index];
                const float invSigma2 = (*pKFi->mvInvLevelSigma2)[kpUn.octave];
                if (kp_ur < 0)
                    add(2, LBA_MONO, -1, kb, c, pKFi->mTimeStamp, kpUn.x, kpUn.y, 0.0, invSigma2);
                else
                    add(3, LBA_STEREO, -1, kb, c, pKFi->mTimeStamp, kpUn.x, kpUn.y, kp_ur, invSigma2);
            }
        }
        // GP observations of non-keyframes (:234-282).  The reference walks vpKFs and takes each keyframe's
        // equal_range of the point's multimap: O(points x keyframes).  Here the point's own GP observations
        // are visited and ordered by (position of their keyframe in vpKFs, multimap order), which is the
        // same edge order at O(observations log observations).
        if (!observationsGP.empty()) {
            struct GPEdge {
                int pos, seq;
                MultiKeyFrame* K;
                const GPObs* g;
            };
            std::vector<GPEdge> ge;
            int seq = 0;
            for (auto it = observationsGP.begin(); it != observationsGP.end(); ++it, ++seq) {
                auto pr = kf_pos.equal_range(it->first);
                for (auto q = pr.first; q != pr.second; ++q) ge.push_back(GPEdge{q->second, seq, it->first, &it->second});
            }
            std::sort(ge.begin(), ge.end(), [](const GPEdge& x, const GPEdge& y) {
                return x.pos != y.pos ? x.pos < y.pos : x.seq < y.seq;
            });
            for (const GPEdge& e : ge) {
                MultiKeyFrame* pKFi = e.K;
                if (pKFi->isBad() || !pKFi->mNextKF) continue;
                if (pKFi->mnId > maxKFid || pKFi->mNextKF->mnId > maxKFid) continue;
                const int a = vtx(pKFi), b = vtx(pKFi->mNextKF);
                if (a < 0 || b < 0) continue;
                const GPObs& g = *e.g;
                const float invSigma2 = (*pKFi->mvInvLevelSigma2)[g.obs.octave];
                if (g.ur >= 0)
                    add(1, LBA_STEREO_GP, a, b, g.cam, g.time, g.obs.x, g.obs.y, g.ur, invSigma2);
                else
                    add(0, LBA_MONO_GP, a, b, g.cam, g.time, g.obs.x, g.obs.y, 0.0, invSigma2);
            }
        }
        if (nEdges == 0) continue;   // optimizer.removeVertex(vP): the point and its GP edges go (:284-292)
        pt_of[i] = (int)pts.size();
        pts.push_back(pMP);
        per_point.push_back(std::move(E));
    }
    // point vertices in g2o's order (by id), edges per point in that order
    std::vector<int> order(pts.size());
    for (size_t r = 0; r < order.size(); ++r) order[r] = (int)r;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return pts[a]->mnId < pts[b]->mnId; });
    for (size_t r = 0; r < order.size(); ++r) {
        MapPoint* P = pts[order[r]];
        const Vec3f X = P->GetWorldPos();
        W->lm.push_back((double)X.x); W->lm.push_back((double)X.y); W->lm.push_back((double)X.z);
        W->mp_ids.push_back((int64_t)P->mnId);
        W->mp_vtx.push_back(P);
        for (Pending& e : per_point[order[r]]) {
            e.o.lm = (int)r;
            W->obs.push_back(e.o);
            W->obs_tag.push_back(e.tag);
            W->n_edges[e.tag]++;
        }
    }
    W->included.assign(vpMP.size(), 0);
    for (size_t i = 0; i < vpMP.size(); ++i)   // (a repeated entry shares its first occurrence's vertex)
        W->included[i] = vpMP[i] && pt_of[seen.at(vpMP[i])] >= 0;

    // ---- optimiser settings (:66-76, :137-138)
    lba_config& cfg = W->cfg;
    std::memcpy(cfg.qc, pMap->mQc, sizeof(cfg.qc));
    cfg.huber_mono = (double)thHuberMono;
    cfg.huber_stereo = (double)thHuberStereo;
    cfg.huber_prior = 21.026;      // rk->setDelta(21.026) on EdgeGaussianPrior (:128-130)
    cfg.lambda_init = 1e-5;        // solver->setUserLambdaInit(1e-5) (:75)
    cfg.tau = 1e-5;
    cfg.max_trials = 10;
    cfg.early_stop = 1;
}

int Optimizer::BundleAdjustment(const std::vector<MultiKeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                                int nIterations, volatile const int32_t* stop, unsigned long nLoopKF,
                                const lbamap_options& opt, lba_problem* problem, lbamap_ba_result* out) {
    lbamap_ba_result res{};
    auto finish = [&](int rc) {
        res.status = rc;
        if (out) *out = res;
        return rc;
    };
    if (vpKFs.empty()) return finish(LBA_E_ARG);
    BundleAdjustmentWindow W;
    BuildBundleAdjustmentWindow(vpKFs, vpMP, &W);
    res.n_kf = (int)W.kfs.size();
    res.n_fixed_kf = W.n_fixed;
    res.n_mp = (int)W.mp_ids.size();
    res.n_priors = (int)W.priors.size();
    res.n_vel = (int)W.vel_kfs.size();
    for (int t = 0; t < 5; ++t) res.n_edges[t] = W.n_edges[t];

    // ---- initializeOptimization + optimize(nIterations) (:294-297)
    W.cfg.device = opt.device;
    W.cfg.flags = opt.flags;
    int rc = lba_set_config(problem, &W.cfg);
    if (rc >= 0)
        rc = lba_set_problem(problem, W.kfs.data(), (int)W.kfs.size(), W.lm.data(), (int)W.mp_ids.size(), W.obs.data(),
                             (int)W.obs.size(), W.priors.data(), (int)W.priors.size(), W.vel_kfs.data(),
                             (int)W.vel_kfs.size(), W.cams.data(), (int)W.cams.size());
    lba_stats st{};
    if (rc >= 0) rc = lba_optimize(problem, nIterations, stop, &st);
    if (rc < 0) return finish(rc);
    res.iterations = st.iterations;
    res.chi2_initial = st.chi2_initial;
    res.chi2_final = st.chi2_final;

    // ---- recover the estimates (:300-365)
    std::vector<lba_kf> kf_out(W.kfs.size());
    std::vector<double> lm_out(W.lm.size());
    rc = lba_get_state(problem, kf_out.data(), lm_out.data());
    if (rc < 0) return finish(rc);
    std::unordered_map<const MultiKeyFrame*, int> row;
    for (size_t i = 0; i < W.kf_vtx.size(); ++i) row[W.kf_vtx[i]] = (int)i;
    for (MultiKeyFrame* pKF : vpKFs) {
        if (pKF->isBad()) continue;
        auto it = row.find(pKF);
        if (it == row.end()) continue;
        const lba_kf& v = kf_out[it->second];
        SE3d Twb;
        std::memcpy(Twb.q, v.q, sizeof(Twb.q));
        std::memcpy(Twb.t, v.t, sizeof(Twb.t));
        const SE3f Tbw = Twb.inverse().cast_float();   // Sophus::SE3f(v->estimate().Twb.inverse().cast<float>())
        float vel[6];
        for (int i = 0; i < 6; ++i) vel[i] = (float)v.vel[i];
        if (nLoopKF == 0) {
            pKF->SetPose(Tbw);
            pKF->SetVelocity(vel);
        } else {
            pKF->mTbwGBA = Tbw;
            std::memcpy(pKF->mVwbGBA, vel, sizeof(vel));
            pKF->mnBAGlobalForKF = nLoopKF;
        }
    }
    std::unordered_map<const MapPoint*, int> prow;
    for (size_t r = 0; r < W.mp_vtx.size(); ++r) prow[W.mp_vtx[r]] = (int)r;
    for (size_t i = 0; i < vpMP.size(); ++i) {
        if (!W.included[i]) continue;   // vbNotIncludedMP[i]
        MapPoint* pMP = vpMP[i];
        const int r = prow.at(pMP);
        const Vec3f X{(float)lm_out[3 * r], (float)lm_out[3 * r + 1], (float)lm_out[3 * r + 2]};
        if (nLoopKF == 0) {
            pMP->SetWorldPos(X);
            pMP->UpdateNormalAndDepth();
        } else {
            pMP->mPosGBA = X;
            pMP->mnBAGlobalForKF = nLoopKF;
        }
    }
    return finish(LBA_OK);
}

void Optimizer::BundleAdjustment(const std::vector<MultiKeyFrame*>& vpKFs, const std::vector<MapPoint*>& vpMP,
                                 int nIterations, bool* pbStopFlag, const unsigned long nLoopKF, const bool bRobust) {
    (void)bRobust;   // unused by the reference too
    // One engine per calling thread, freed when the thread exits: LoopClosing starts a new thread for
    // every global BA (src/LoopClosing.cc:1044), and the reference's optimiser dies with the call.
    struct ThreadEngine {
        lba_problem* p = nullptr;
        ~ThreadEngine() {
            if (p) lba_destroy(p);
        }
    };
    thread_local ThreadEngine engine;
    if (!engine.p) {
        lba_config cfg{};
        if (lba_create(&engine.p, &cfg) != LBA_OK) { engine.p = nullptr; return; }
    }
    lba_problem* p = engine.p;
    // g2o's setForceStopFlag(pbStopFlag): the engine polls an int32 between iterations and trials, which a
    // watcher keeps equal to *pbStopFlag while the optimisation runs
    volatile int32_t flag = 0;
    std::atomic<bool> done{false};
    std::thread watcher;
    if (pbStopFlag)
        watcher = std::thread([&] {
            while (!done.load(std::memory_order_relaxed)) {
                flag = *static_cast<volatile bool*>(pbStopFlag) ? 1 : 0;
                std::this_thread::sleep_for(std::chrono::microseconds(100));
            }
        });
    if (pbStopFlag) flag = *pbStopFlag ? 1 : 0;
    lbamap_options opt{0, 0, 0, 0};
    const int rc = BundleAdjustment(vpKFs, vpMP, nIterations, pbStopFlag ? &flag : nullptr, nLoopKF, opt, p, nullptr);
    done = true;
    if (watcher.joinable()) watcher.join();
    if (rc < 0) std::fprintf(stderr, "BundleAdjustment: not run (%d): %s\n", rc, lba_last_error(p));
}

void Optimizer::GlobalBundleAdjustemnt(Map* pMap, int nIterations, bool* pbStopFlag, const unsigned long nLoopKF,
                                       const bool bRobust) {
    // (:53-58)
    std::vector<MultiKeyFrame*> vpKFs = pMap->GetAllKeyFrames();
    std::vector<MapPoint*> vpMP = pMap->GetAllMapPoints();
    BundleAdjustment(vpKFs, vpMP, nIterations, pbStopFlag, nLoopKF, bRobust);
}

}  // namespace amc_slam
