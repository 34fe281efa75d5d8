/*
 * amc_lba.h — C ABI of the MI355X-native continuous-time (GP) local bundle adjustment.
 *
 * This is the drop-in boundary for AMC-SLAM's local BA hot path.  The reference builds a
 * g2o::SparseOptimizer inside Optimizer::LocalGPBA (src/Optimizer.cc:713-1432, declared at
 * include/Optimizer.h:58) and calls SparseOptimizer::optimize (Thirdparty/g2o/g2o/core/
 * sparse_optimizer.cpp:354-419).  A caller using this library keeps LocalGPBA's window
 * selection and post-pass, fills the flat arrays below instead of g2o vertices/edges, and
 * calls lba_optimize().  Plain C types only; every array is caller-owned and copied.
 *
 * Conventions (mirroring g2o):
 *   - Tangent order is Sophus [translation; rotation]; pose update T <- T*exp(d)
 *     (src/G2oTypes.cc:41-46), velocity and landmark updates are additive.
 *   - Quaternions are stored (x, y, z, w) like Eigen::Quaternion::coeffs().
 *   - Hessian vertex order: non-fixed keyframes in array order, then landmarks in array
 *     order (g2o sorts active vertices by id and puts non-marginalized first,
 *     sparse_optimizer.cpp:166-190).  Callers that want g2o's exact ordering pass
 *     keyframes sorted by mnId.
 *   - b = -sum J^T rho' Omega e, H dx = b (base_multi_edge.hpp:35-48, 170-222).
 *   - Status codes: >= 0 success (lba_optimize: iterations run), LBA_E_* < 0 on error.
 */
#ifndef AMC_LBA_H
#define AMC_LBA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LBA_ABI_VERSION 5   /* 5: lba_solver_info writes out[8] (was out[5]) */

/* status codes */
#define LBA_OK              0
#define LBA_E_EMPTY        -1   /* empty graph: no edges or no free vertices (sparse_optimizer.cpp:358-361) */
#define LBA_E_SOLVE        -2   /* reduced-camera factorisation not positive (linear_solver_dense.h:108-112) */
#define LBA_E_DIVERGED     -3   /* LocalGPBA divergence guard (src/Optimizer.cc:1354-1358), set by host adapter */
#define LBA_E_ARG          -4   /* invalid argument / malformed problem */
#define LBA_E_HIP          -5   /* HIP runtime error */
#define LBA_E_LIMIT        -6   /* problem exceeds a compiled limit (see lba_last_error) */
#define LBA_E_TIMEOUT      -7   /* a bounded device hand-off wait gave up (never expected: e.g. a GPU shared with
                                   another launch that keeps workgroups from being scheduled); the results are not
                                   used and the problem's state is undefined until the next lba_set_problem */

/* observation kinds (the reprojection edges of include/G2oTypes.h) */
#define LBA_MONO_GP    0   /* EdgeMonoGPExtrinsic / EdgeMonoGP: 2-d, vertices (kf_a=prev KF, kf_b=KF, lm, the camera extrinsic: optimised when lba_cam.ext_free)
                              (include/G2oTypes.h:292-402, src/G2oTypes.cc:225-367) */
#define LBA_STEREO_GP  1   /* EdgeStereoGP: 3-d [u, v, u_r] (include/G2oTypes.h:404-421, src/G2oTypes.cc:369-443) */
#define LBA_MONO       2   /* EdgeMono: 2-d, vertices (kf_b, lm) at KF time (include/G2oTypes.h:423-446, src/G2oTypes.cc:445-468) */
#define LBA_STEREO     3   /* EdgeStereo: 3-d (include/G2oTypes.h:448-468, src/G2oTypes.cc:470-495) */

/* lba_config.flags.  Timing inserts HIP events into the stream (each costs a few us of
 * device idle time), so both are off by default. */
#define LBA_FLAG_TIME_SWEEP   1   /* time every launch of the residual/Jacobian sweep kernel
                                     (lba_stats.ms_k_linearize) */
#define LBA_FLAG_TIME_PHASES  2   /* also time every phase (ms_linearize .. ms_update_eval); runs the
                                     host-driven loop */
#define LBA_FLAG_HOST_LOOP    4   /* take every LM decision on the host, one trial at a time (default:
                                     the trials are queued and decided on the device; same results) */
#define LBA_FLAG_BAND_SOLVE   8   /* solve the reduced camera system by forward / back substitution after
                                     the factorisation instead of through the tiles of L^-1 (default:
                                     chosen by size; large pose systems always take this path) */
#define LBA_FLAG_DENSE_SOLVE 16   /* force the L^-1-tile solve (pose systems up to 6144 only) */
#define LBA_FLAG_TIME_SAMPLED 32  /* with LBA_FLAG_TIME_SWEEP in the queued loop: events on one trial in
                                     ten (the 6th of each ten of a batch), so their idle time costs ~1/10 */
#define LBA_FLAG_SUBTREE_SOLVE 64 /* partitioned problems: distributed factorisation of the reduced camera
                                     system (each rank factors its subtree of the nested dissection, the ranks
                                     sum their contributions to the top separators, every rank factors the
                                     top); the window must be split by lba_partition_assign */
#define LBA_FLAG_F32_RESIDUAL 128 /* the fp32-residual option of BASELINE configs[4] ("fp32 residuals + fp64
                                     accumulate"): each observation's projection, residual and Jacobian rows in
                                     fp32 (the world offset Xw - twb in fp64), the robust weights and every sum of
                                     H / b, the Schur complement and the solve in fp64; results within fp32
                                     rounding of the fp64 path, not bitwise */

/* LM termination codes in lba_stats.result (OptimizationAlgorithm::SolverResult) */
#define LBA_RESULT_OK         0
#define LBA_RESULT_TERMINATE  1
#define LBA_RESULT_STOPPED    2   /* stop flag raised (SparseOptimizer::terminate) */

typedef struct lba_config {
    double qc[36];          /* GaussianProcess::mQc, 6x6 row-major (Tracking.cc:753-758 builds diag(Gaussian.Qc)) */
    double huber_mono;      /* Huber delta for 2-d edges; LocalGPBA: (double)(float)sqrt(5.991)  (Optimizer.cc:975) */
    double huber_stereo;    /* Huber delta for 3-d edges; (double)(float)sqrt(7.815)           (Optimizer.cc:977) */
    double huber_prior;     /* Huber delta on EdgeGaussianPrior; <= 0: none (LocalGPBA), 21.026 in BundleAdjustment (:99-136) */
    double lambda_init;     /* OptimizationAlgorithmLevenberg userLambdaInit; <= 0 -> tau * max diag (levenberg.cpp:171-185) */
    double tau;             /* 1e-5 (levenberg.cpp:47) */
    int    max_trials;      /* _maxTrialsAfterFailure, 10 (levenberg.cpp:51) */
    int    early_stop;      /* 1: g2o stop rules active (3 iterations of <1e-3 gain, levenberg.cpp:157-166); 0: fixed count */
    int    device;          /* HIP device ordinal */
    int    flags;           /* LBA_FLAG_* bits, 0 for production use */
} lba_config;

typedef struct lba_kf {     /* VertexPoseVel / PoseVelocity (include/G2oTypes.h:59-80,104-126) */
    double q[4];            /* Twb rotation (x,y,z,w) */
    double t[3];            /* Twb translation */
    double vel[6];          /* PoseVelocity::Vel, world-frame twist [v; w] */
    double time;            /* PoseVelocity::time (KF time stamp) */
    double bf;              /* PoseVelocity::bf (stereo baseline * fx) */
    int32_t fixed;          /* vertex fixed (no Hessian rows) */
    int32_t pad;
} lba_kf;

typedef struct lba_obs {
    int32_t kind;           /* LBA_MONO_GP .. LBA_STEREO */
    int32_t kf_a;           /* GP kinds: previous KF (vertex 0); non-GP: ignored (-1) */
    int32_t kf_b;           /* GP kinds: KF (vertex 1); non-GP: the KF (vertex 0) */
    int32_t lm;             /* landmark index */
    int32_t cam;            /* camera index (EdgeMono/EdgeStereo use the reference camera = n_cam-1) */
    int32_t pad;
    double  t;              /* observation time (GP kinds: pKFi->mvTimeStamps[c]) */
    double  z[3];           /* u, v, (u_right for stereo) */
    double  w;              /* information weight invSigma2 / unc2 (Omega = w * I) */
} lba_obs;

typedef struct lba_prior {  /* EdgeGaussianPrior(v0 = kf_a older, v1 = kf_b newer), info QiInv(t_b - t_a) */
    int32_t kf_a;
    int32_t kf_b;
} lba_prior;

typedef struct lba_cam {    /* GeometricCamera (Pinhole) + MultiKeyFrame::mTbc[c] */
    double q[4];            /* Tbc rotation (x,y,z,w) */
    double t[3];            /* Tbc translation */
    double fx, fy, cx, cy;  /* Pinhole::mvParameters (float values widened) */
    /* extrinsic calibration (LocalGPBA bExtrinsic, src/Optimizer.cc:982-995,1228-1240): ext_free = 1
     * makes this camera's VertexExtrinsic (include/G2oTypes.h:83-102, T <- T exp(d)) optimisable.  Its
     * 6 dofs follow the keyframes' in the pose system (g2o id order: iniMPid + c + 1 > every KF id);
     * the LBA_MONO_GP observations of the camera (EdgeMonoGPExtrinsic, src/G2oTypes.cc:241-314) link it,
     * and an EdgeExtrinsicPrior (include/G2oTypes.h:470-494) e = log(Rbc_ini^-1 Rbc), information
     * rbc_info, is attached to it.  0: fixed, as in every call without bExtrinsic (the prior is then
     * inactive: all its vertices are fixed).  Not with a partitioned problem (LBA_E_LIMIT), and an
     * LBA_STEREO_GP observation of such a camera is rejected (EdgeStereoGP projects through the static
     * MultiKeyFrame::mTbc, not the vertex). */
    int32_t ext_free;
    int32_t pad;
    double  rbc_ini[4];     /* MultiFrame::mRbc_ini[c] (x,y,z,w), float values widened (Frame.cc:181) */
    double  rbc_info[9];    /* MultiFrame::mRbc_ini_cov[c] used as the information, row-major (0.2 I, Frame.cc:182) */
} lba_cam;

typedef struct lba_stats {
    int32_t iterations;     /* LM iterations run (SparseOptimizer::optimize return) */
    int32_t trials;         /* total LM trials (sum of qmax) */
    int32_t result;         /* LBA_RESULT_* of the last iteration */
    int32_t solve_failures; /* trials whose factorisation was not positive */
    double  chi2_initial;   /* activeRobustChi2 before the first iteration */
    double  chi2_final;     /* activeRobustChi2 of the last computed errors (g2o semantics) */
    double  lambda_final;
    double  ms_linearize;   /* device time per phase, summed (HIP events; LBA_FLAG_TIME_PHASES):
                               ms_linearize the fused linearisation + landmark elimination of every
                               trial, ms_schur the pose-sample expansion + assembly of S */
    double  ms_schur;
    double  ms_solve;
    double  ms_update_eval;
    double  ms_total;       /* host wall time of lba_optimize */
    double  ms_k_linearize; /* device time of the fused sweep kernel (residual / Jacobian / J^T W J and the
                               landmark elimination, k_lin_schur), summed over its dispatches
                               (LBA_FLAG_TIME_SWEEP or LBA_FLAG_TIME_PHASES) */
    int32_t n_k_linearize;  /* launches of that kernel */
    int32_t n_k_solve;      /* launches of the factorisation + solve kernel (k_chol_flow) */
    double  ms_k_solve;     /* its device time, summed (same flags) */
} lba_stats;

typedef struct lba_problem lba_problem;   /* opaque: owns device buffers + stream */

/* lifecycle */
int         lba_create(lba_problem** out, const lba_config* cfg);
void        lba_destroy(lba_problem* p);
const char* lba_last_error(const lba_problem* p);
int         lba_abi_version(void);
/* Engines created by lba_create and not yet destroyed, process-wide (leak checks: the reference
 * builds and frees its g2o optimiser on every call, src/Optimizer.cc:61-367, so a caller that runs one
 * engine per call or per thread must see this return to its previous value). */
int         lba_live_problems(void);

/* Replace the configuration (Huber deltas, lambda0, Qc, flags) of an existing problem, e.g. between
 * LocalGPBA calls with and without bLarge (OptimizationAlgorithmLevenberg::setUserLambdaInit,
 * RobustKernelHuber::setDelta).  Takes effect at the next lba_set_problem; the device cannot change. */
int lba_set_config(lba_problem* p, const lba_config* cfg);

/* Copy a window to the device (replaces SparseOptimizer::addVertex/addEdge +
 * initializeOptimization, sparse_optimizer.cpp:197-267).  vel_kfs lists the KFs carrying an
 * EdgeVelocity (info QcInv(2,2), Optimizer.cc:858-870). */
int lba_set_problem(lba_problem* p,
                    const lba_kf* kfs, int32_t n_kf,
                    const double* lm_xyz, int32_t n_lm,
                    const lba_obs* obs, int32_t n_obs,
                    const lba_prior* priors, int32_t n_priors,
                    const int32_t* vel_kfs, int32_t n_vel,
                    const lba_cam* cams, int32_t n_cam);

/* ---- partitioned global BA (BASELINE config 4): one problem per GPU (rank), every
 * rank holding ALL keyframes (same array, same fixed flags), a disjoint subset of the landmarks with
 * all of their observations, and rank 0 alone the motion-prior / velocity edges.  Per LM trial the
 * ranks sum their reduced camera systems (the envelope of S, the reduced rhs and b_p: one
 * all-reduce) and their trial sums (chi2 before / after, computeScale: a 4-double all-reduce); every
 * rank then solves the same system, so the keyframe states and the LM decisions stay identical and
 * each rank back-substitutes its own landmarks.  The all-reduce is the caller's (sum, in place, on
 * device memory, enqueued on the given HIP stream, bitwise identical on every rank): RCCL over
 * xGMI (lba_set_partition_rccl), an in-process group of problems on one device (lba_group, for
 * tests), or any function.  Call before lba_set_problem; set_problem is then collective (the ranks
 * agree on the union envelope of S), as are lba_optimize calls, which need lambda_init > 0 and the
 * same iteration count and stop flag on every rank.  A set_problem that fails on one rank fails on
 * every rank: the ranks exchange their set-up status in one all-reduce before the first collective
 * (the others return LBA_E_ARG, "another rank of the partition failed its set-up").  An lba_group
 * rank waits at most 120 s for its peers, then the group is poisoned (every call returns an error). */
typedef int (*lba_allreduce_fn)(double* dev_buf, int64_t count, void* hip_stream, void* user);
int lba_set_partition(lba_problem* p, int32_t rank, int32_t nranks, lba_allreduce_fn fn, void* user);
int lba_rccl_unique_id(void* id_out);   /* NCCL_UNIQUE_ID_BYTES (128) bytes, on one rank, shared by the caller */
int lba_set_partition_rccl(lba_problem* p, const void* id, int32_t rank, int32_t nranks);
typedef struct lba_group lba_group;     /* in-process all-reduce across problems on one device */
int  lba_group_create(lba_group** out, int32_t nranks);
void lba_group_destroy(lba_group* g);
int  lba_set_partition_group(lba_problem* p, lba_group* g, int32_t rank);
/* The landmark / edge split of a window for LBA_FLAG_SUBTREE_SOLVE (host only, no device): the reduced camera
 * system's nested dissection (the plan lba_set_problem makes) is cut into nranks subtrees and the top; each
 * landmark goes to the rank whose subtree holds its keyframes (a landmark that only sees top keyframes, or
 * fixed ones: rank = index mod nranks), each motion prior / velocity edge likewise.  Every rank then holds all
 * keyframes, its landmarks with all their observations, and its edges (the replacement of the l mod N split of
 * lba_set_partition, BlockSolver's Schur complement per partition, block_solver.hpp:381-445).  Outputs
 * lm_rank[n_lm], prior_rank[n_priors], vel_rank[n_vel]; panels_out (may be NULL) [3]: panels of the system,
 * panels in the top, columns of the largest subtree; kf_rank (may be NULL) [n_kf]: the rank whose subtree holds
 * the keyframe (-1: the top, or fixed).  Cameras are not an input: a partitioned lba_set_problem rejects free
 * extrinsics (lba_cam.ext_free, LBA_E_LIMIT) before it plans, so the pattern planned here (keyframe blocks only)
 * is the one every partitioned set-up factors. */
int lba_partition_assign(const lba_config* cfg, const lba_kf* kfs, int32_t n_kf, int32_t n_lm, const lba_obs* obs,
                         int32_t n_obs, const lba_prior* priors, int32_t n_priors, const int32_t* vel_kfs, int32_t n_vel,
                         int32_t nranks, int32_t* lm_rank, int32_t* prior_rank, int32_t* vel_rank, int32_t* panels_out,
                         int32_t* kf_rank);
/* LBA_FLAG_SUBTREE_SOLVE: per keyframe slot, the rank whose subtree holds it (-1: the top, every rank holds its
 * state; a keyframe of another rank's subtree keeps its old state on this rank: gather it from its owner). */
int  lba_kf_owner(const lba_problem* p, int32_t* owner);
/* The rank's share of the factorisation: out[0] its factorisation FLOPs (its subtree's columns + the top; the
 * whole system when the solve is replicated), out[1] the whole system's, out[2] bytes it all-reduces per LM trial
 * for the solve (split: the top tiles + bS + b_p; replicated: every tile + bS + b_p; 0 unpartitioned), out[3]
 * the replicated solve's bytes for comparison, out[4] panels of its subtree, out[5] panels of the top. */
int  lba_split_info(const lba_problem* p, double out[6]);

/* ---- window farm (BASELINE config 3): one LocalGPBA window per GPU (rank), windows cut
 * from one trajectory, so neighbours share keyframes and map points.  The reference runs one local BA at
 * a time (LocalMapping::Run -> Optimizer::LocalGPBA, src/LocalMapping.cc:131) and every window reads and
 * writes the shared map (src/Optimizer.cc:1380-1432); here the shared estimates are exchanged at window
 * boundaries instead, device to device:
 *   lba_set_farm*      the collective: RCCL over xGMI (lba_set_farm_rccl: ncclAllGather on the problem's
 *                      stream), an in-process group on one device (lba_set_farm_group, for tests), or any
 *                      sum all-reduce of the caller's (an all-gather as a sum over zero-padded slots);
 *   lba_farm_plan      after lba_set_problem, collective: which vertices this rank publishes (owner ==
 *                      rank) and, for every vertex another rank owns, where its estimate lands in the
 *                      exchange buffer (matched by global id once; no lookups at exchange time);
 *   lba_farm_exchange  collective, per window boundary: pack kernel -> all-gather -> unpack kernel on the
 *                      problem's stream; the received estimates are bit-exact copies of the owners'.
 * kf_owner / lm_owner: per vertex of this window, the rank that publishes it, or -1 for a vertex no other
 * window shares.  Keyframe time stamps and fixed flags are not exchanged (they are the same everywhere).
 * A vertex whose owner does not publish it (no such global id on that rank) keeps its own estimate; the
 * counts of published, received and unmatched vertices come back in out_counts[5] (may be NULL):
 * kf published, lm published, kf received, lm received, unmatched.  lba_set_problem drops the plan. */
int lba_set_farm(lba_problem* p, int32_t rank, int32_t nranks, lba_allreduce_fn fn, void* user);
int lba_set_farm_rccl(lba_problem* p, const void* id, int32_t rank, int32_t nranks);
int lba_set_farm_group(lba_problem* p, lba_group* g, int32_t rank);
int lba_farm_plan(lba_problem* p, const int64_t* kf_gid, const int32_t* kf_owner,
                  const int64_t* lm_gid, const int32_t* lm_owner, int32_t* out_counts);
int lba_farm_exchange(lba_problem* p);
/* Host-only form of the plan's matching (no device, no collective; tests): given every rank's published
 * global ids (pub_gid: nranks x cap, -1 padded) and this window's ids / owners, the source slot of every
 * received vertex: src[i] = owner * cap + position, or -1 (not a received vertex, or unmatched). */
int lba_farm_match(int32_t rank, int32_t nranks, int32_t cap, const int64_t* pub_gid,
                   const int64_t* gid, const int32_t* owner, int32_t n, int32_t* src);

/* Levenberg-Marquardt (OptimizationAlgorithmLevenberg::solve x iters).  stop_flag is polled
 * between iterations and trials like SparseOptimizer::terminate().  Returns iterations run
 * (>= 0) or an LBA_E_* code. */
int lba_optimize(lba_problem* p, int32_t iters, volatile const int32_t* stop_flag, lba_stats* out);

/* write-back: current (accepted) estimates */
int lba_get_state(lba_problem* p, lba_kf* kf_out, double* lm_out);
/* overwrite the current estimates (window-boundary exchange of shared keyframes/landmarks in a
 * multi-GPU window farm); either pointer may be NULL to keep that part.  Quaternions are
 * re-normalised like the Sophus cast. */
int lba_set_state(lba_problem* p, const lba_kf* kf_in, const double* lm_xyz);

/* Errors of the current estimate: robust chi2 sum, per-observation chi2 (e^T Omega e) and
 * the LocalGPBA depth test (both KF poses for GP edges, include/G2oTypes.h:305-314).
 * Any output pointer may be NULL. */
int lba_eval(lba_problem* p, double* chi2_robust, double* obs_chi2, uint8_t* depth_ok);
/* Per-observation chi2 of the last computed errors, without evaluating anything: after lba_optimize
 * the errors of its last trial state, accepted or not (g2o's e->chi2() after optimize(): the
 * _error of the last computeActiveErrors, src/Optimizer.cc:1300-1330). */
int lba_trial_chi2(lba_problem* p, double* obs_chi2);

/* Parity/debug entry points (no LM).  lba_linearize: computeActiveErrors + buildSystem at the
 * current estimate: residuals [n_obs*3] (unused components 0), H_pp dense [np*np] full
 * symmetric, b [np + 3*n_lm], H_ll [n_lm*9].  Any pointer may be NULL.  Returns np. */
int lba_linearize(lba_problem* p, double* residuals, double* H_pp, double* b, double* H_ll);
/* One damped solve at lambda on the last linearisation: dx [np + 3*n_lm] (poses then
 * landmarks), BlockSolver::solve with setLambda/restoreDiagonal (block_solver.hpp:354-486). */
int lba_solve_step(lba_problem* p, double lambda, double* dx);
/* The trial state of the last lba_solve_step: the current estimate with that step applied by the device's update
 * (VertexPoseVel / VertexSBAPointXYZ oplus, src/G2oTypes.cc:41-46, sparse_optimizer.cpp:422-435), i.e. what g2o's
 * LM evaluates after push() + update() (optimization_algorithm_levenberg.cpp:94-103); the current estimate is not
 * changed.  Same layout as lba_get_state. */
int lba_trial_state(lba_problem* p, lba_kf* kf_out, double* lm_out);
/* Diagnostics: the host preprocessing of lba_set_problem alone (device order, pairs, tiles, slabs; no device,
 * no GPU needed) on the given window; phase_ms: wall ms of the order/pairs, tiles and slots/state phases;
 * counts: device landmarks, pose blocks, pose dimension, tiles, a 32-bit fingerprint of the tiling and slab
 * layout (the same for any LBA_SETUP_THREADS).  Returns LBA_OK or the error lba_set_problem would return. */
int lba_setup_host_profile(const lba_config* cfg, const lba_kf* kfs, int32_t n_kf, const double* lm_xyz, int32_t n_lm,
                           const lba_obs* obs, int32_t n_obs, const lba_prior* priors, int32_t n_priors,
                           const int32_t* vel_kfs, int32_t n_vel, const lba_cam* cams, int32_t n_cam,
                           double phase_ms[3], int32_t counts[5]);
/* Diagnostics: `passes` back-to-back parallel passes of lba_set_problem's host thread pool, of 1..max_pieces
 * pieces each (short and long passes alternating); returns the number of pieces that did not run exactly once
 * in their own pass or were still running when their pass returned (0 when the pool is sound).  No device. */
int lba_debug_pool_stress(int32_t passes, int32_t max_pieces);
/* Diagnostics: the Lie-group primitives of the kernels (Sophus SE3 exp / log, Thirdparty/Sophus/sophus/se3.hpp:
 * 223-252,761-781; RightJacobianPose3 / RightJacobianPose3Inv, src/Pose3utils.cc:5-46, small-angle branches
 * included) evaluated on `device` for n records in[13 n] = {xi[6], q[4] (x,y,z,w), t[3]}: out[85 n] =
 * {exp(xi) q[4] t[3], log(q, t)[6], Jr(xi)[36], Jr^-1(xi)[36]} (row-major). */
int lba_debug_lie(int32_t device, int32_t n, const double* in, double* out);
/* Diagnostics: set the problem's device fault word to `code` (1 factorisation, 2 assembly, 4 trial evaluation:
 * the waits of one launch that gave up), as a bounded in-launch wait does when it times out.  The next call that
 * reads the word (lba_optimize, lba_linearize, lba_solve_step, lba_eval) fails with LBA_E_TIMEOUT and clears it,
 * so the failure path can be tested without a hang.  No LM work. */
int lba_debug_inject_fault(lba_problem* p, int32_t code);
/* How the reduced camera system is solved (after lba_set_problem), at the granularity of panels of
 * CHOL_NB = 32 rows: out[0] panels of the loop-closure tail (rows that reach back to the first panels,
 * ordered last), out[1] panels, out[2] stored 32 x 32 tiles of the factor L (fill-in included), out[3] 1
 * for the substitution (band) solve, 0 for the L^-1-tile solve, out[4] panels on the factorisation's
 * dependent chain (the depth of the elimination tree), out[5] levels of the nested dissection, out[6]
 * tiles of the lower triangle of S (the pattern before fill-in), out[7] fill-in tiles (out[2] - out[6]). */
int lba_solver_info(const lba_problem* p, int32_t out[8]);
/* The launch fusions the set-up chose (diagnostics and tests): out[0] 1 when the trial evaluation runs inside
 * k_update (the whole grid resident at once), out[1] 1 when the pose samples' expansion and the assembly of S
 * run as one launch (k_exp_asm), out[2] 1 for the fp32-residual kernels, out[3] the k_update grid. */
int lba_kernel_modes(const lba_problem* p, int32_t out[4]);
/* Algorithmic FLOPs of one solve of the reduced camera system, from the symbolic structure of L:
 * out[0] the tile factorisation (per column with m tiles below the diagonal: potrf + m trsm + m(m+1)/2
 * trailing tile updates), out[1] the forward and back substitutions. */
int lba_solver_flops(const lba_problem* p, double out[2]);
/* Device memory (bytes) the problem's buffers hold: the reduced system and its factor are packed envelope
 * tiles (O(envelope), not O(npose^2)); the dense H_pp of lba_linearize is allocated only when asked for.
 * LBA_E_ARG (< 0) for a null problem. */
int64_t lba_device_bytes(const lba_problem* p);
/* Wall time (ms) of the last lba_set_problem's phases: [0] activity, GP pairs and landmark order, [1] tiles,
 * [2] slab slots and device-order records, [3] host -> device upload, [4] the solve's layout (envelope plan,
 * flow tasks).  Writes min(n, phases) values and returns that count; LBA_E_ARG for a null problem. */
int lba_setup_phases(const lba_problem* p, double* ms, int32_t n);
/* Dimension of the pose system (12 * number of non-fixed KFs + 6 * number of free extrinsics). */
int lba_pose_dim(const lba_problem* p);
/* Current camera extrinsics (write-back of the VertexExtrinsic estimates, src/Optimizer.cc:1419-1428):
 * the cameras passed to lba_set_problem with Tbc (q, t) replaced by the estimate for free ones. */
int lba_get_cams(lba_problem* p, lba_cam* cams_out);

/* ---- tracking: Optimizer::PoseGPOptimizationFromeLastFrame (src/Optimizer.cc:369-686), SURVEY.md §8(f)3.
 * Per frame: vertices prev (pFrame->mpPrevFrame, fixed = the `fix` argument) and cur (pFrame), the map
 * points fixed; EdgeMonoGPOnlyPose for the asynchronous cameras (LBA_MONO_GP: the GP pose between prev
 * and cur at the camera's time stamp), EdgeMonoOnlyPose / EdgeStereoOnlyPose for the reference camera
 * (LBA_MONO / LBA_STEREO at cur), EdgeGaussianPrior(prev, cur) and EdgeVelocity on both.  Four rounds
 * of optimize(10) on the level-0 edges with re-classification between them (chi2 5.991 mono, 15.6 /
 * 9.8 / 7.815 / 7.815 stereo, x1.5 for points tracked closer than 10 m, depth test), the robust kernel
 * dropped after round 3.  A batch of frames runs as one launch, one workgroup per frame. */
typedef struct lba_track_obs {
    int32_t kind;           /* LBA_MONO_GP, LBA_MONO or LBA_STEREO */
    int32_t cam;            /* mmpKeyToCam[i]; the reference camera (n_cam - 1) for LBA_MONO / LBA_STEREO */
    int32_t outlier;        /* in: pFrame->mvbOutlier[i] (edge level 1); out: the last round's classification */
    int32_t close;          /* mvpMapPoints[i]->mvTrackDepth[cam] < 10 */
    double  t;              /* pFrame->mvTimeStamps[cam] (GP kinds) */
    double  z[3];           /* u, v (, u_right) */
    double  w;              /* invSigma2 / unc2 */
    double  Xw[3];          /* pMP->GetWorldPos() widened to double (fixed) */
} lba_track_obs;

typedef struct lba_track_frame {
    lba_kf  prev;           /* VertexPoseVel(pFrame->mpPrevFrame); prev.fixed = fix.  Not written back */
    lba_kf  cur;            /* VertexPoseVel(pFrame); out: the optimised pose and velocity (SetPose / SetVelocity) */
    int32_t obs0, n_obs;    /* the frame's observations in the batch array */
    int32_t n_good;         /* out: nInitialCorrespondences - nBad, the reference's return value */
    int32_t iterations;     /* out: LM iterations over the rounds */
} lba_track_frame;

typedef struct lba_tracker lba_tracker;   /* device buffers + stream, reused across calls */
int  lba_tracker_create(lba_tracker** out, const lba_config* cfg);   /* qc, Huber deltas, tau, device */
void lba_tracker_destroy(lba_tracker* t);
int  lba_track(lba_tracker* t, lba_track_frame* frames, int32_t n_frames, lba_track_obs* obs, int32_t n_obs,
               const lba_cam* cams, int32_t n_cam);

#ifdef __cplusplus
}
#endif
#endif /* AMC_LBA_H */
