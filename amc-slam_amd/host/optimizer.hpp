// optimizer.hpp — Optimizer::LocalGPBA with the reference's signature, running on the GPU engine.
//
// Reference: include/Optimizer.h:58, src/Optimizer.cc:713-1432.  The window selection, graph
// shape, outlier post-pass and write-back are restated on the map classes of lba_map.hpp; the
// g2o SparseOptimizer + BlockSolverX + LinearSolverDense + OptimizationAlgorithmLevenberg
// (src/Optimizer.cc:838-856) is replaced by one lba_problem (include/amc_lba.h).
#pragma once

#include <list>
#include <vector>

#include "../../include/amc_lba.h"
#include "../../include/amc_lba_map.h"
#include "lba_map.hpp"

namespace amc_slam {

// The window LocalGPBA builds, as the flat arrays of the C ABI plus, per observation row, what
// the post-pass needs (the reference's vpEdgeKF* / vpMapPointEdge* / vpGPObs* vectors).
struct LocalGPBAWindow {
    std::vector<MultiKeyFrame*> vpOptimizableKFs;
    // (the reference's std::lists, as vectors: the same appends and iteration order, no allocation per element)
    std::vector<MultiKeyFrame*> lpOptVisKFs, lFixedKeyFrames;
    std::vector<MapPoint*> lLocalMapPoints;

    std::vector<lba_kf> kfs;
    std::vector<int64_t> kf_ids;
    std::vector<double> lm;
    std::vector<int64_t> mp_ids;
    std::vector<MapPoint*> mp_vtx;          // the point of each landmark vertex (mp_ids' order)
    std::vector<lba_obs> obs;
    std::vector<int32_t> obs_tag;           // 0 MonoGP, 1 StereoGP, 2 Mono, 3 Stereo, 4 MonoGP at KF time
    std::vector<lba_prior> priors;
    std::vector<int32_t> vel_kfs;
    std::vector<lba_cam> cams;
    lba_config cfg{};

    struct Row {                            // one post-pass entry per observation row
        MultiKeyFrame* kf;                  // vpEdgeKF*  (the KF the observation is erased from)
        MapPoint* mp;
        GPObs gp;                           // tags 0/1
        int cam;
    };
    std::vector<Row> rows;
    std::vector<int> cam_obs;               // cam_obs[c] (Optimizer.cc:1010, 1145)
    int n_edges[5] = {0, 0, 0, 0, 0};
};

// The global BA graph (Optimizer::BundleAdjustment, src/Optimizer.cc:61-282) as the C ABI's flat arrays.
struct BundleAdjustmentWindow {
    std::vector<MultiKeyFrame*> kf_vtx;     // vertex order (by mnId)
    std::vector<lba_kf> kfs;
    std::vector<int64_t> kf_ids;
    std::vector<MapPoint*> mp_vtx;          // the included points (nEdges > 0), by mnId
    std::vector<double> lm;
    std::vector<int64_t> mp_ids;
    std::vector<char> included;             // per vpMP entry: !vbNotIncludedMP[i]
    std::vector<lba_obs> obs;
    std::vector<int32_t> obs_tag;           // 0 MonoGP, 1 StereoGP, 2 Mono, 3 Stereo, 4 MonoGP at KF time
    std::vector<lba_prior> priors;
    std::vector<int32_t> vel_kfs;
    std::vector<lba_cam> cams;
    lba_config cfg{};
    int n_edges[5] = {0, 0, 0, 0, 0};
    int n_fixed = 0;
};

class Optimizer {
public:
    // The reference entry points (include/Optimizer.h:50-53).  bRobust is unused, as in the reference
    // (every reprojection and prior edge carries its Huber kernel).  pbStopFlag is polled between LM
    // iterations and trials, like g2o's setForceStopFlag.
    static void BundleAdjustment(const std::vector<MultiKeyFrame*>& vpKF, const std::vector<MapPoint*>& vpMP,
                                 int nIterations = 5, bool* pbStopFlag = nullptr, const unsigned long nLoopKF = 0,
                                 const bool bRobust = true);
    static void GlobalBundleAdjustemnt(Map* pMap, int nIterations = 5, bool* pbStopFlag = nullptr,
                                       const unsigned long nLoopKF = 0, const bool bRobust = true);
    // The same with the device / flags, an int32 stop flag and a report.
    static int BundleAdjustment(const std::vector<MultiKeyFrame*>& vpKF, const std::vector<MapPoint*>& vpMP,
                                int nIterations, volatile const int32_t* stop, unsigned long nLoopKF,
                                const lbamap_options& opt, lba_problem* problem, lbamap_ba_result* out);
    // Graph build (src/Optimizer.cc:61-282) without optimising.
    static void BuildBundleAdjustmentWindow(const std::vector<MultiKeyFrame*>& vpKF, const std::vector<MapPoint*>& vpMP,
                                            BundleAdjustmentWindow* W);

    // The reference entry point.  pbStopFlag is handed to the optimiser only after optimize()
    // returns, exactly as src/Optimizer.cc:1254-1255 does, so it never interrupts the LM loop.
    // The num_* out-parameters are left untouched, as in the reference.
    static void LocalGPBA(MultiKeyFrame* pKF, bool* pbStopFlag, Map* pMap, int& num_fixedKF, int& num_OptKF,
                          int& num_MPs, int& num_edges, bool bLarge = false, bool bExtrinsic = false,
                          bool bRecInit = false);

    // The same call with the GPU device / flags and a report of what happened.
    static int LocalGPBA(MultiKeyFrame* pKF, Map* pMap, const lbamap_options& opt, lba_problem* problem,
                         lbamap_result* out);

    // Window selection + graph build (src/Optimizer.cc:713-1208) without optimising.  Marks the BA
    // flags on keyframes and map points exactly as the reference does.
    static void BuildLocalGPBAWindow(MultiKeyFrame* pKF, bool bLarge, LocalGPBAWindow* W);
};

}  // namespace amc_slam
