/*
 * lba_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of AMC-SLAM's GP local-BA hot path, used as the parity checker for the
 * HIP product (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg).  Nothing in the
 * shipped library links or calls this code.  See lba_oracle.c for the per-function citations.
 *
 * Parity status: pinned by the vendored Sophus sympy package (exp/log fixtures generated in
 * the build container, tests/golden/make_golden.py), by the four-scalar GP identity, and by
 * central differences on the exact Jacobian blocks.  The Eigen boundary (6x6 inverse, LDLT) is
 * "parity unpinned" (SURVEY.md §8(c)): restated from Eigen 3.3's published algorithms.
 */
#ifndef LBA_ORACLE_H
#define LBA_ORACLE_H

#include "../include/amc_lba.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_problem orc_problem;

orc_problem* orc_create(const lba_config* cfg,
                        const lba_kf* kfs, int n_kf, const double* lm_xyz, int n_lm,
                        const lba_obs* obs, int n_obs, const lba_prior* priors, int n_priors,
                        const int* vel_kfs, int n_vel, const lba_cam* cams, int n_cam);
void   orc_destroy(orc_problem* p);
int    orc_pose_dim(const orc_problem* p);
int    orc_lm_dim(const orc_problem* p);

/* computeActiveErrors + activeRobustChi2; residuals [n_obs*3], obs_chi2 [n_obs] may be NULL */
double orc_compute_errors(orc_problem* p, double* residuals, double* obs_chi2);
/* buildSystem at the current estimate (errors recomputed first).  H_pp [np*np] full
 * symmetric, b [np + nl], H_ll [n_lm*9] (landmark array order; inactive landmarks 0). */
int    orc_build_system(orc_problem* p, double* H_pp, double* b, double* H_ll);
/* setLambda + BlockSolver::solve + restoreDiagonal on the last buildSystem; dx [np + nl] */
int    orc_solve(orc_problem* p, double lambda, double* dx);
/* r = (H + lambda I) dx - b on the last buildSystem (full pose + landmark system, O(nnz)); r [np + nl] */
void   orc_normal_residual(const orc_problem* p, double lambda, const double* dx, double* r);
/* Full LM: returns iterations; stats may be NULL */
int    orc_optimize(orc_problem* p, int iters, lba_stats* stats);
void   orc_get_state(const orc_problem* p, lba_kf* kfs, double* lm_xyz);
void   orc_depth_ok(const orc_problem* p, unsigned char* ok);
void   orc_last_obs_chi2(const orc_problem* p, double* obs_chi2);
void   orc_get_cams(const orc_problem* p, lba_cam* cams);   /* camera extrinsics (VertexExtrinsic estimates) */

/* single-edge evaluation at the current estimate: err[3], J[3*27] row-major with columns
 * [KF_a pose(6) vel(6) | KF_b pose(6) vel(6) | point(3)] (GP kinds), or
 * [0 | KF pose(6) vel(6) | point(3)] for EdgeMono/EdgeStereo.  Returns error dimension. */
int    orc_obs_linearize(orc_problem* p, int obs_index, double* err, double* J);
/* prior edge: err[12], Ji[144], Jj[144] */
int    orc_prior_linearize(orc_problem* p, int prior_index, double* err, double* Ji, double* Jj);

/* Optimizer::PoseGPOptimizationFromeLastFrame on one frame (include/amc_lba.h lba_track_*): updates
 * fr->cur, tob[].outlier, fr->n_good (returned), fr->iterations */
int    orc_track_pose(const lba_config* cfg, lba_track_frame* fr, lba_track_obs* tob, int n,
                      const lba_cam* cams, int n_cam);

/* Lie / GP primitives for golden-vector tests */
void   orc_se3_exp(const double xi[6], double q[4], double t[3]);
void   orc_se3_log(const double q[4], const double t[3], double xi[6]);
void   orc_so3_exp(const double w[3], double q[4]);
void   orc_so3_log(const double q[4], double w[3]);
void   orc_right_jac_pose3(const double xi[6], double J[36]);
void   orc_right_jac_pose3_inv(const double xi[6], double J[36]);
void   orc_left_jac_pose3_q(const double xi[6], double Q[9]);
/* GaussianProcess::QueryPose (11-arg form) with Qc [36]:  outputs T (q,t), At1 [72], Pt1 [72],
 * dT (q,t), xi12 [6] */
void   orc_gp_query_pose(const double qc[36],
                         const double q1[4], const double t1[3], const double q2[4], const double t2[3],
                         const double v1[6], const double v2[6], double time1, double time2, double t,
                         double qo[4], double to[3], double At1[72], double Pt1[72],
                         double dq[4], double dt[3], double xi12[6]);
/* Dense LDLT solve as LinearSolverDense (Eigen pivoted LDLT): returns 1 if isPositive */
int    orc_ldlt_solve(int n, const double* A, const double* b, double* x);

#ifdef __cplusplus
}
#endif
#endif
