/*
 * amc_lba_map.h — C ABI of the LocalGPBA host adapter.
 *
 * The reference's local BA entry point is
 *     void Optimizer::LocalGPBA(MultiKeyFrame* pKF, bool* pbStopFlag, Map* pMap, int& num_fixedKF,
 *                               int& num_OptKF, int& num_MPs, int& num_edges, bool bLarge,
 *                               bool bExtrinsic, bool bRecInit)          (include/Optimizer.h:58)
 * defined at src/Optimizer.cc:713-1432.  It selects a window from the covisibility / temporal
 * graph, builds a g2o graph, optimises 10 LM iterations, drops outlier observations and writes
 * the estimates back into the map.  The C++ adapter in amc-slam_amd/host/ restates all of that
 * on a minimal map (amc_slam::MultiKeyFrame / MapPoint / Map, host/lba_map.hpp) and runs the
 * optimisation through the GPU engine of include/amc_lba.h.  This header is the C view of it:
 * a map is loaded from a *window snapshot* (the flat record layout below, the bytes a real
 * AMC-SLAM process would serialise from its Atlas), LocalGPBA runs on it, and the updated map
 * is saved back into the same layout.
 *
 * Snapshot layout (little endian, every section 8-byte aligned, records in this order):
 *     lbamap_header
 *     lbamap_cam     [n_cam]          MultiKeyFrame::mTbc[c] + Pinhole parameters
 *     lbamap_kf      [n_kf]           keyframes
 *     lbamap_kp      [n_kp]           keypoints of all keyframes (kf.kp_off .. + kf.n_kp)
 *     int64_t        [n_covis]        ordered covisible keyframe ids (kf.covis_off .. + kf.n_covis)
 *     lbamap_mp      [n_mp]           map points
 *     lbamap_mpobs   [n_mpobs]        MapPoint::mObservations entries (mp.obs_off .. + mp.n_obs)
 *     lbamap_gpobs   [n_gpobs]        MapPoint::mObservationsForGPBA entries (mp.gp_off .. + mp.n_gp)
 *
 * Ordering: std::map<MultiKeyFrame*, ...> iterates by pointer in the reference; here it iterates
 * by keyframe id (KFs are allocated in id order, so this is the reference's order in practice
 * and is deterministic).  The order of GP observations of one (point, KF) pair is the snapshot's.
 */
#ifndef AMC_LBA_MAP_H
#define AMC_LBA_MAP_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#include "amc_lba.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LBAMAP_VERSION   2      /* the snapshot format */
#define LBAMAP_ABI_VERSION 2    /* the adapter's structs: 2: lbamap_result gained ms_phase[4] */
#define LBAMAP_MAX_CAM   8
#define LBAMAP_MAX_LEVEL 16

typedef struct lbamap_header {
    char    magic[8];           /* "AMCSNAP" + NUL */
    int32_t version;            /* LBAMAP_VERSION */
    int32_t n_cam;              /* MultiKeyFrame::nCamera; camera n_cam-1 is the reference (stereo) camera */
    int32_t n_kf, n_kp, n_covis, n_mp, n_mpobs, n_gpobs;
    int32_t n_levels;           /* ORB pyramid levels (mnScaleLevels) */
    int32_t pad;
    double  qc[36];             /* GaussianProcess::mQc (6x6 row-major) */
    float   inv_level_sigma2[LBAMAP_MAX_LEVEL];   /* mvInvLevelSigma2 */
    float   scale_factor[LBAMAP_MAX_LEVEL];       /* mvScaleFactors */
} lbamap_header;

typedef struct lbamap_cam {     /* Sophus::SE3f MultiKeyFrame::mTbc[c] and Pinhole::mvParameters */
    float q[4];                 /* (x, y, z, w) */
    float t[3];
    float fx, fy, cx, cy;
    float rbc_ini[4];           /* MultiFrame::mRbc_ini[c] (x, y, z, w): the extrinsic prior's rotation (Frame.cc:181) */
    float pad;
} lbamap_cam;

typedef struct lbamap_kf {
    int64_t id;                 /* mnId */
    int64_t prev_id, next_id;   /* mPrevKF / mNextKF ids, -1 = none */
    double  time;               /* mTimeStamp */
    double  cam_time[LBAMAP_MAX_CAM];  /* mvTimeStamps[c] */
    float   q[4];               /* mTcw (body pose T_bw, float Sophus::SE3f as the reference stores it) */
    float   t[3];
    float   vel[6];             /* GetVelocity() */
    float   bf;                 /* mbf */
    int32_t bad;                /* isBad() */
    int32_t map_id;             /* GetMap(): keyframes of another map are never optimised */
    int32_t kp_off, n_kp;       /* keypoints */
    int32_t covis_off, n_covis; /* GetVectorCovisibleKeyFrames() */
    int32_t has_twc;            /* 1: twc_* hold the cached camera poses mTwc[c]; 0: derive them with
                                   SetPose (src/KeyFrame.cc:116-145) when the snapshot is loaded */
    float   twc_q[LBAMAP_MAX_CAM][4];   /* mTwc[c]: cached at the last SetPose, used by
                                           MapPoint::UpdateNormalAndDepth through GetCameraCenter */
    float   twc_t[LBAMAP_MAX_CAM][3];
} lbamap_kf;

typedef struct lbamap_kp {      /* mvKeysUn[idx], mmpKeyToCam[idx], mvuRight[mmpGlobalToLocalID[idx]], mvpMapPoints[idx] */
    float   x, y;
    int32_t octave;
    int32_t cam;
    float   ur;                 /* right-image u, < 0 if none */
    int32_t pad;
    int64_t mp_id;              /* matched map point id, -1 = none */
} lbamap_kp;

typedef struct lbamap_mp {
    int64_t id;                 /* mnId */
    float   pos[3];             /* mWorldPos */
    int32_t bad;                /* mbBad */
    int64_t ref_kf;             /* mpRefKF id */
    float   track_depth[LBAMAP_MAX_CAM];  /* mvTrackDepth[c] */
    float   normal[3];          /* mNormalVector */
    float   min_dist, max_dist; /* mfMinDistance, mfMaxDistance */
    int32_t obs_off, n_obs;     /* observations */
    int32_t gp_off, n_gp;       /* GP observations */
    int32_t pad;
} lbamap_mp;

typedef struct lbamap_mpobs {   /* one entry of MapPoint::mObservations */
    int64_t kf_id;
    int32_t idx[LBAMAP_MAX_CAM];    /* keypoint index per camera, -1 = not observed */
} lbamap_mpobs;

typedef struct lbamap_gpobs {   /* GPObs (include/MapPoint.h:46-62) keyed by the KF before the frame */
    int64_t kf_id;
    double  time;
    int32_t cam;
    float   x, y;
    int32_t octave;
    float   ur;
    int32_t pad;
} lbamap_gpobs;

/* Options of one LocalGPBA call (the reference's arguments plus the GPU device). */
typedef struct lbamap_options {
    int32_t large;              /* bLarge: window of 25 KFs, lambda0 1e-2, no divergence guard */
    int32_t extrinsic;          /* bExtrinsic: second pass with the extrinsics of well-observed cameras free (:1228-1240) */
    int32_t device;             /* HIP device */
    int32_t flags;              /* lba_config.flags */
} lbamap_options;

/* What LocalGPBA did (the reference's num_* out-parameters are never written; these are). */
typedef struct lbamap_result {
    int32_t status;             /* LBA_OK, LBA_E_DIVERGED ("FAIL LOCAL-GP BA", nothing written back), ... */
    int32_t n_opt_kf, n_vis_kf, n_fixed_kf, n_mp;
    int32_t n_edges_mono_gp, n_edges_stereo_gp, n_edges_mono, n_edges_stereo, n_edges_mono_gp_kf;
    int32_t n_erased_gp, n_erased;      /* outlier observations removed */
    int32_t n_set_bad;                  /* map points that became bad while erasing */
    int32_t iterations;
    double  chi2_initial, chi2_final;   /* err, err_end (Optimizer.cc:1221-1253) */
    double  ms_phase[4];                /* wall ms of the call's parts: window build (graph construction, :717-1208),
                                           lba_set_problem, lba_optimize (both passes with bExtrinsic), outlier
                                           post-pass + write-back (:1257-1431); the reference's LocalMapping keeps
                                           such timers (vtime, src/LocalMapping.cc:129-135) */
} lbamap_result;

/* What BundleAdjustment / GlobalBundleAdjustemnt did (src/Optimizer.cc:53-367). */
typedef struct lbamap_ba_result {
    int32_t status;             /* LBA_OK or an LBA_E_* code (nothing written back) */
    int32_t n_kf, n_fixed_kf;   /* keyframe vertices; fixed: the map's initial keyframe */
    int32_t n_mp;               /* point vertices kept (at least one keyframe observation) */
    int32_t n_priors, n_vel;    /* EdgeGaussianPrior / EdgeVelocity */
    int32_t n_edges[5];         /* MonoGP, StereoGP (non-keyframes), Mono, Stereo, MonoGP at keyframe times */
    int32_t iterations;
    double  chi2_initial, chi2_final;
} lbamap_ba_result;

typedef struct lbamap lbamap;   /* opaque: the loaded map + a reusable lba_problem */

/* Load a snapshot (bytes as laid out above).  Returns LBA_OK or LBA_E_ARG. */
/* LBAMAP_ABI_VERSION of the library: a caller built against another header must not pass its structs. */
int    lbamap_abi_version(void);
int    lbamap_load(lbamap** out, const void* bytes, size_t n_bytes);
void   lbamap_free(lbamap* m);
const char* lbamap_last_error(const lbamap* m);
/* Size of the snapshot lbamap_save would write, and the write itself (returns bytes written or <0). */
size_t lbamap_snapshot_size(const lbamap* m);
int64_t lbamap_save(const lbamap* m, void* bytes, size_t cap);

/* Optimizer::LocalGPBA(pKF = keyframe kf_id, ...) on the loaded map: window selection, GPU LM,
 * outlier post-pass and write-back, exactly as src/Optimizer.cc:713-1432. */
int lbamap_local_gpba(lbamap* m, int64_t kf_id, volatile const int32_t* stop_flag, const lbamap_options* opt,
                      lbamap_result* out);

/* Optimizer::GlobalBundleAdjustemnt(pMap, n_iterations, stop, loop_kf) on the whole map (every keyframe
 * and map point of it, GetAllKeyFrames / GetAllMapPoints), GPU engine on opt->device (opt->large and
 * opt->extrinsic are ignored).  loop_kf == 0 writes poses, velocities and points back (SetPose /
 * SetVelocity / SetWorldPos + UpdateNormalAndDepth); loop_kf != 0 stores them as the GBA results
 * (mTbwGBA, mVwbGBA, mPosGBA, mnBAGlobalForKF), read back with lbamap_kf_gba / lbamap_mp_gba. */
int lbamap_global_ba(lbamap* m, int32_t n_iterations, volatile const int32_t* stop_flag, uint64_t loop_kf,
                     const lbamap_options* opt, lbamap_ba_result* out);
int lbamap_kf_gba(const lbamap* m, int64_t kf_id, float q[4], float t[3], float vel[6], uint64_t* loop_kf);
int lbamap_mp_gba(const lbamap* m, int64_t mp_id, float pos[3], uint64_t* loop_kf);
/* The reference's own entry, void Optimizer::GlobalBundleAdjustemnt(pMap, n_iterations, pbStopFlag,
 * nLoopKF, bRobust) (src/Optimizer.cc:53-58), on the calling thread and GPU 0: its engine belongs to the
 * calling thread and is destroyed when that thread exits (LoopClosing starts one thread per global BA,
 * src/LoopClosing.cc:1044).  stop may be NULL.  Returns LBA_OK (the reference returns nothing). */
int lbamap_global_ba_thread(lbamap* m, int32_t n_iterations, bool* stop, uint64_t loop_kf);
/* The global BA graph as flat arrays, without optimising (parity tests), same outputs as
 * lbamap_build_window. */
int lbamap_build_ba_window(lbamap* m, int32_t counts[6], lba_kf* kfs, double* lm_xyz, lba_obs* obs,
                           lba_prior* priors, int32_t* vel_kfs, lba_cam* cams, int64_t* kf_ids, int64_t* mp_ids,
                           int32_t* obs_tag, lba_config* cfg);

/* The window LocalGPBA would build for kf_id, as the flat arrays of include/amc_lba.h, without
 * optimising and without touching the map (the BA flags are restored).  Two calls: first with
 * NULL arrays to get the counts in *counts = {n_kf, n_lm, n_obs, n_priors, n_vel, n_cam}, then
 * with arrays of those sizes.  kf_ids / mp_ids / obs_tag (may be NULL) give the map ids of each
 * keyframe / landmark row and, per observation, the post-pass list it belongs to
 * (0 MonoGP, 1 StereoGP, 2 Mono, 3 Stereo, 4 MonoGP at KF time). */
int lbamap_build_window(lbamap* m, int64_t kf_id, const lbamap_options* opt, int32_t counts[6],
                        lba_kf* kfs, double* lm_xyz, lba_obs* obs, lba_prior* priors, int32_t* vel_kfs,
                        lba_cam* cams, int64_t* kf_ids, int64_t* mp_ids, int32_t* obs_tag, lba_config* cfg);

#ifdef __cplusplus
}
#endif
#endif /* AMC_LBA_MAP_H */
