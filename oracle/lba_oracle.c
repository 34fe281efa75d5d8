/*
 * lba_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker and CPU baseline, never shipped).
 *
 * A line-by-line C restatement of the reference CPU path behind Optimizer::LocalGPBA:
 *   Sophus SO3/SE3          Thirdparty/Sophus/sophus/so3.hpp, se3.hpp, common.hpp:94
 *   Pose3utils              src/Pose3utils.cc:5-73,111-119
 *   GaussianProcess         include/GaussianProcess.h:20-48, src/GaussianProcess.cc:5-42
 *   Pinhole                 src/CameraModels/Pinhole.cpp:35-41,71-81
 *   edges                   src/G2oTypes.cc:25-118,225-495, include/G2oTypes.h:147-519
 *   g2o quadratic forms     Thirdparty/g2o/g2o/core/base_multi_edge.hpp:35-48,170-222,
 *                           base_binary_edge.hpp:54-120, base_unary_edge.hpp:42-72,
 *                           base_edge.h:58-61,96-102, robust_kernel_impl.cpp:65-90
 *   block Schur             Thirdparty/g2o/g2o/core/block_solver.hpp:354-604
 *   dense LDLT              Thirdparty/g2o/g2o/solvers/linear_solver_dense.h:65-113 (Eigen LDLT,
 *                           restated from Eigen 3.3 LDLT.h: ldlt_inplace<Lower>::unblocked)
 *   Levenberg-Marquardt     Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-194,
 *                           sparse_optimizer.cpp:61-114,354-435
 *
 * The GP interpolation deliberately follows the reference's 12x12 matrix path (Qi, QiInv,
 * Transition products) rather than the four-scalar closed form the HIP product uses, so the
 * two implementations are independent.  Row-major storage throughout.
 */
#include "lba_oracle.h"

#include <float.h>
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define SOPHUS_EPS 1e-10   /* Sophus::Constants<double>::epsilon(), common.hpp:94 */

/* ------------------------------------------------------------------ dense helpers */
static void mat_mul(double* C, const double* A, const double* B, int m, int k, int n) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int l = 0; l < k; ++l) s += A[i * k + l] * B[l * n + j];
            C[i * n + j] = s;
        }
}
static void mat_tr(double* T, const double* A, int m, int n) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) T[j * m + i] = A[i * n + j];
}
static void mat_eye(double* A, int n) {
    memset(A, 0, sizeof(double) * n * n);
    for (int i = 0; i < n; ++i) A[i * n + i] = 1.0;
}
static void mat_scale(double* A, double s, int n) { for (int i = 0; i < n; ++i) A[i] *= s; }
static void set_block(double* A, int lda, int r0, int c0, const double* B, int m, int n) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) A[(r0 + i) * lda + c0 + j] = B[i * n + j];
}
static void get_block(double* B, const double* A, int lda, int r0, int c0, int m, int n) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) B[i * n + j] = A[(r0 + i) * lda + c0 + j];
}
static void hat3(double* H, const double* w) {   /* Sophus::SO3::hat / Skew */
    H[0] = 0.0;   H[1] = -w[2]; H[2] = w[1];
    H[3] = w[2];  H[4] = 0.0;   H[5] = -w[0];
    H[6] = -w[1]; H[7] = w[0];  H[8] = 0.0;
}
/* Eigen PartialPivLU inverse (used by Matrix::inverse() for sizes > 4) */
static int lu_inverse(double* Ainv, const double* A, int n) {
    double* LU = (double*)malloc(sizeof(double) * n * n);
    int* perm = (int*)malloc(sizeof(int) * n);
    memcpy(LU, A, sizeof(double) * n * n);
    for (int i = 0; i < n; ++i) perm[i] = i;
    int ok = 1;
    for (int k = 0; k < n; ++k) {
        int piv = k;
        double best = fabs(LU[k * n + k]);
        for (int i = k + 1; i < n; ++i)
            if (fabs(LU[i * n + k]) > best) { best = fabs(LU[i * n + k]); piv = i; }
        if (best == 0.0) ok = 0;
        if (piv != k) {
            for (int j = 0; j < n; ++j) { double t = LU[k * n + j]; LU[k * n + j] = LU[piv * n + j]; LU[piv * n + j] = t; }
            int t = perm[k]; perm[k] = perm[piv]; perm[piv] = t;
        }
        if (LU[k * n + k] != 0.0)
            for (int i = k + 1; i < n; ++i) {
                LU[i * n + k] /= LU[k * n + k];
                for (int j = k + 1; j < n; ++j) LU[i * n + j] -= LU[i * n + k] * LU[k * n + j];
            }
    }
    for (int c = 0; c < n; ++c) {   /* solve LU x = P e_c */
        double* x = (double*)malloc(sizeof(double) * n);
        for (int i = 0; i < n; ++i) x[i] = (perm[i] == c) ? 1.0 : 0.0;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < i; ++j) x[i] -= LU[i * n + j] * x[j];
        for (int i = n - 1; i >= 0; --i) {
            for (int j = i + 1; j < n; ++j) x[i] -= LU[i * n + j] * x[j];
            x[i] /= LU[i * n + i];
        }
        for (int i = 0; i < n; ++i) Ainv[i * n + c] = x[i];
        free(x);
    }
    free(LU);
    free(perm);
    return ok;
}
/* Eigen compute_inverse<3,3> (cofactor / adjugate form, InverseImpl.h) */
static double cof3(const double* m, int i, int j) {
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m[i1 * 3 + j1] * m[i2 * 3 + j2] - m[i1 * 3 + j2] * m[i2 * 3 + j1];
}
static void inverse3(double* r, const double* m) {
    double c0 = cof3(m, 0, 0), c1 = cof3(m, 1, 0), c2 = cof3(m, 2, 0);
    double det = c0 * m[0] + c1 * m[3] + c2 * m[6];
    double invdet = 1.0 / det;
    r[0] = c0 * invdet; r[1] = c1 * invdet; r[2] = c2 * invdet;
    r[3] = cof3(m, 0, 1) * invdet; r[4] = cof3(m, 1, 1) * invdet; r[5] = cof3(m, 2, 1) * invdet;
    r[6] = cof3(m, 0, 2) * invdet; r[7] = cof3(m, 1, 2) * invdet; r[8] = cof3(m, 2, 2) * invdet;
}

/* ------------------------------------------------------------------ Sophus SO3 / SE3 */
typedef struct { double x, y, z, w; } quat;
typedef struct { quat q; double t[3]; } se3;

static quat q_normalized(quat q) {   /* SO3Base::normalize, so3.hpp:297-303 */
    double len = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= len; q.y /= len; q.z /= len; q.w /= len;
    return q;
}
static quat so3_mul(quat a, quat b) {   /* so3.hpp:325-339, ctor normalises (:481-487) */
    quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return q_normalized(r);
}
static quat so3_inv(quat q) {   /* so3.hpp:229-231: SO3(conjugate) normalises */
    quat r = {-q.x, -q.y, -q.z, q.w};
    return q_normalized(r);
}
static void so3_act(const quat* q, const double* p, double* out) {   /* so3.hpp:358-367 */
    double uv[3] = {q->y * p[2] - q->z * p[1], q->z * p[0] - q->x * p[2], q->x * p[1] - q->y * p[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    double c[3] = {q->y * uv[2] - q->z * uv[1], q->z * uv[0] - q->x * uv[2], q->x * uv[1] - q->y * uv[0]};
    for (int i = 0; i < 3; ++i) out[i] = p[i] + q->w * uv[i] + c[i];
}
static void so3_matrix(const quat* q, double* R) {   /* Eigen QuaternionBase::toRotationMatrix */
    double tx = 2 * q->x, ty = 2 * q->y, tz = 2 * q->z;
    double twx = tx * q->w, twy = ty * q->w, twz = tz * q->w;
    double txx = tx * q->x, txy = ty * q->x, txz = tz * q->x;
    double tyy = ty * q->y, tyz = tz * q->y, tzz = tz * q->z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
static quat so3_exp_theta(const double* w, double* theta) {   /* so3.hpp:583-618 */
    double theta_sq = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double imag, real;
    if (theta_sq < SOPHUS_EPS * SOPHUS_EPS) {
        *theta = 0.0;
        double theta_po4 = theta_sq * theta_sq;
        imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_po4;
        real = 1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_po4;
    } else {
        *theta = sqrt(theta_sq);
        double half = 0.5 * (*theta);
        imag = sin(half) / (*theta);
        real = cos(half);
    }
    quat q = {imag * w[0], imag * w[1], imag * w[2], real};
    return q;
}
static void so3_log_theta(const quat* q, double* w, double* theta) {   /* so3.hpp:247-290 */
    double squared_n = q->x * q->x + q->y * q->y + q->z * q->z;
    double qw = q->w, f;
    if (squared_n < SOPHUS_EPS * SOPHUS_EPS) {
        double squared_w = qw * qw;
        f = 2.0 / qw - (2.0 / 3.0) * squared_n / (qw * squared_w);
        *theta = 2.0 * squared_n / qw;
    } else {
        double n = sqrt(squared_n);
        if (fabs(qw) < SOPHUS_EPS)
            f = (qw > 0 ? M_PI : -M_PI) / n;
        else
            f = 2.0 * atan(n / qw) / n;
        *theta = f * n;
    }
    w[0] = f * q->x; w[1] = f * q->y; w[2] = f * q->z;
}
static se3 se3_mul(const se3* a, const se3* b) {   /* se3.hpp:304-308 */
    se3 r;
    r.q = so3_mul(a->q, b->q);
    double tb[3];
    so3_act(&a->q, b->t, tb);
    for (int i = 0; i < 3; ++i) r.t[i] = a->t[i] + tb[i];
    return r;
}
static se3 se3_inv(const se3* a) {   /* se3.hpp:208-211 */
    se3 r;
    r.q = so3_inv(a->q);
    double mt[3] = {-a->t[0], -a->t[1], -a->t[2]};
    so3_act(&r.q, mt, r.t);
    return r;
}
static void se3_act(const se3* T, const double* p, double* out) {   /* se3.hpp:321-324 */
    so3_act(&T->q, p, out);
    for (int i = 0; i < 3; ++i) out[i] += T->t[i];
}
static se3 se3_exp(const double* a) {   /* se3.hpp:761-781 */
    double theta;
    se3 r;
    r.q = so3_exp_theta(a + 3, &theta);
    double Om[9], Om2[9], V[9];
    hat3(Om, a + 3);
    mat_mul(Om2, Om, Om, 3, 3, 3);
    if (theta < SOPHUS_EPS) {
        so3_matrix(&r.q, V);
    } else {
        double th2 = theta * theta;
        double c1 = (1.0 - cos(theta)) / th2, c2 = (theta - sin(theta)) / (th2 * theta);
        for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0 ? 1.0 : 0.0) + c1 * Om[i] + c2 * Om2[i];
    }
    mat_mul(r.t, V, a, 3, 3, 1);
    return r;
}
static void se3_log(const se3* T, double* xi) {   /* se3.hpp:223-252 */
    double theta, w[3];
    so3_log_theta(&T->q, w, &theta);
    xi[3] = w[0]; xi[4] = w[1]; xi[5] = w[2];
    double Om[9], Om2[9], Vinv[9];
    hat3(Om, w);
    mat_mul(Om2, Om, Om, 3, 3, 3);
    double c;
    if (fabs(theta) < SOPHUS_EPS) {
        c = 1.0 / 12.0;
    } else {
        double half = 0.5 * theta;
        c = (1.0 - theta * cos(half) / (2.0 * sin(half))) / (theta * theta);
    }
    for (int i = 0; i < 9; ++i) Vinv[i] = (i % 4 == 0 ? 1.0 : 0.0) - 0.5 * Om[i] + c * Om2[i];
    mat_mul(xi, Vinv, T->t, 3, 3, 1);
}
static void se3_adj(const se3* T, double* A) {   /* se3.hpp:103-111 */
    double R[9], tR[9], H[9];
    so3_matrix(&T->q, R);
    hat3(H, T->t);
    mat_mul(tR, H, R, 3, 3, 3);
    memset(A, 0, sizeof(double) * 36);
    set_block(A, 6, 0, 0, R, 3, 3);
    set_block(A, 6, 3, 3, R, 3, 3);
    set_block(A, 6, 0, 3, tR, 3, 3);
}

/* ------------------------------------------------------------------ Pose3utils (src/Pose3utils.cc) */
static void left_jac_pose3_q(const double* xi, double* Q) {   /* :5-24 */
    const double* omega = xi + 3;
    const double* rho = xi;
    double theta = sqrt(omega[0] * omega[0] + omega[1] * omega[1] + omega[2] * omega[2]);
    double X[9], Y[9], XY[9], YX[9], XYX[9], XXY[9], YXX[9], XYXX[9], XXYX[9];
    hat3(X, omega);
    hat3(Y, rho);
    mat_mul(XY, X, Y, 3, 3, 3);
    mat_mul(YX, Y, X, 3, 3, 3);
    mat_mul(XYX, X, YX, 3, 3, 3);
    mat_mul(XXY, X, XY, 3, 3, 3);    /* X * XY */
    mat_mul(YXX, YX, X, 3, 3, 3);    /* YX * X */
    mat_mul(XYXX, XYX, X, 3, 3, 3);  /* XYX * X */
    mat_mul(XXYX, X, XYX, 3, 3, 3);  /* X * XYX */
    double a, b, c;
    if (fabs(theta) > 1e-5) {
        double s = sin(theta), co = cos(theta);
        double t2 = theta * theta, t3 = t2 * theta, t4 = t3 * theta, t5 = t4 * theta;
        a = (theta - s) / t3;
        b = (1.0 - 0.5 * t2 - co) / t4;
        c = 0.5 * ((1.0 - 0.5 * t2 - co) / t4 - 3.0 * (theta - s - t3 / 6.0) / t5);
    } else {   /* reference's small-angle branch, signs as written */
        a = 1.0 / 6.0;
        b = 1.0 / 24.0;
        c = 0.5 * (1.0 / 24.0 + 3.0 / 120.0);
    }
    for (int i = 0; i < 9; ++i)
        Q[i] = 0.5 * Y[i] + a * (XY[i] + YX[i] + XYX[i]) - b * (XXY[i] + YXX[i] - 3.0 * XYX[i]) - c * (XYXX[i] + XXYX[i]);
}
static void left_jac_rot3(const double* w, double* J) {   /* :48-59 */
    double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    if (th2 <= DBL_EPSILON) { mat_eye(J, 3); return; }
    double th = sqrt(th2);
    double d[3] = {w[0] / th, w[1] / th, w[2] / th};
    double s = sin(th), A[9];
    hat3(A, w);
    for (int i = 0; i < 9; ++i) A[i] /= th;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            J[i * 3 + j] = (i == j ? s / th : 0.0) + (1.0 - s / th) * d[i] * d[j] + (1.0 - cos(th)) / th * A[i * 3 + j];
}
static void left_jac_rot3_inv(const double* w, double* J) {   /* :61-73 */
    double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    if (th2 <= DBL_EPSILON) { mat_eye(J, 3); return; }
    double th = sqrt(th2);
    double d[3] = {w[0] / th, w[1] / th, w[2] / th};
    double h = th / 2.0, cot = 1.0 / tan(h), A[9];
    hat3(A, w);
    for (int i = 0; i < 9; ++i) A[i] /= th;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            J[i * 3 + j] = (i == j ? h * cot : 0.0) + (1.0 - h * cot) * d[i] * d[j] - h * A[i * 3 + j];
}
static void left_jac_pose3(const double* xi, double* J) {   /* :26-31 */
    double Q[9], Jr[9];
    left_jac_pose3_q(xi, Q);
    left_jac_rot3(xi + 3, Jr);
    memset(J, 0, sizeof(double) * 36);
    set_block(J, 6, 0, 0, Jr, 3, 3);
    set_block(J, 6, 0, 3, Q, 3, 3);
    set_block(J, 6, 3, 3, Jr, 3, 3);
}
static void left_jac_pose3_inv(const double* xi, double* J) {   /* :36-42 */
    double Q[9], Ji[9], T1[9], T2[9];
    left_jac_pose3_q(xi, Q);
    left_jac_rot3_inv(xi + 3, Ji);
    mat_mul(T1, Ji, Q, 3, 3, 3);
    mat_mul(T2, T1, Ji, 3, 3, 3);
    mat_scale(T2, -1.0, 9);
    memset(J, 0, sizeof(double) * 36);
    set_block(J, 6, 0, 0, Ji, 3, 3);
    set_block(J, 6, 0, 3, T2, 3, 3);
    set_block(J, 6, 3, 3, Ji, 3, 3);
}
static void right_jac_pose3(const double* xi, double* J) {   /* :32-34 */
    double m[6];
    for (int i = 0; i < 6; ++i) m[i] = -xi[i];
    left_jac_pose3(m, J);
}
static void right_jac_pose3_inv(const double* xi, double* J) {   /* :44-46 */
    double m[6];
    for (int i = 0; i < 6; ++i) m[i] = -xi[i];
    left_jac_pose3_inv(m, J);
}
static void se3_ad(const double* v, double* A) {   /* se3Adj, :111-119 */
    double Hw[9], Hv[9];
    hat3(Hw, v + 3);
    hat3(Hv, v);
    memset(A, 0, sizeof(double) * 36);
    set_block(A, 6, 0, 0, Hw, 3, 3);
    set_block(A, 6, 0, 3, Hv, 3, 3);
    set_block(A, 6, 3, 3, Hw, 3, 3);
}

/* ------------------------------------------------------------------ GaussianProcess */
typedef struct { double Qc[36], QcInv[36]; } gp_t;

static void gp_qi(const gp_t* gp, double dt, double* M) {   /* GaussianProcess.h:20-29 */
    double dt2 = dt * dt, dt3 = dt2 * dt;
    memset(M, 0, sizeof(double) * 144);
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double q = gp->Qc[i * 6 + j];
            M[i * 12 + j] = 1.0 / 3.0 * dt3 * q;
            M[i * 12 + 6 + j] = 1.0 / 2.0 * dt2 * q;
            M[(6 + i) * 12 + j] = 1.0 / 2.0 * dt2 * q;
            M[(6 + i) * 12 + 6 + j] = dt * q;
        }
}
static void gp_qi_inv(const gp_t* gp, double dt, double* M) {   /* GaussianProcess.h:31-41 */
    double dt2 = dt * dt, dt3 = dt2 * dt;
    memset(M, 0, sizeof(double) * 144);
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double q = gp->QcInv[i * 6 + j];
            M[i * 12 + j] = 12.0 / dt3 * q;
            M[i * 12 + 6 + j] = -6.0 / dt2 * q;
            M[(6 + i) * 12 + j] = -6.0 / dt2 * q;
            M[(6 + i) * 12 + 6 + j] = 4.0 / dt * q;
        }
}
static void gp_transition(double t1, double t2, double* M) {   /* GaussianProcess.h:44-48 */
    mat_eye(M, 12);
    for (int i = 0; i < 6; ++i) M[i * 12 + 6 + i] = (t2 - t1);
}
/* QueryPose, 11-argument form (src/GaussianProcess.cc:23-42); the 7-arg form (:5-21) is the
 * same computation without the extra outputs. */
static se3 gp_query_pose(const gp_t* gp, const se3* pose1, const se3* pose2, const double* v1, const double* v2,
                         double t1, double t2, double t, double* At1, double* Pt1, se3* dT, double* xi12) {
    double Qi[144], PhiT[144], Phi[144], QiInv[144], tmp[144], Pt[144], At[144], Phi1t[144], Phi12[144];
    gp_qi(gp, t - t1, Qi);
    gp_transition(t, t2, Phi);
    mat_tr(PhiT, Phi, 12, 12);
    gp_qi_inv(gp, t2 - t1, QiInv);
    mat_mul(tmp, Qi, PhiT, 12, 12, 12);
    mat_mul(Pt, tmp, QiInv, 12, 12, 12);
    gp_transition(t1, t, Phi1t);
    gp_transition(t1, t2, Phi12);
    mat_mul(tmp, Pt, Phi12, 12, 12, 12);
    for (int i = 0; i < 144; ++i) At[i] = Phi1t[i] - tmp[i];
    get_block(At1, At, 12, 0, 0, 6, 12);
    get_block(Pt1, Pt, 12, 0, 0, 6, 12);
    double x1[12], x2[12], Jri[36];
    memset(x1, 0, sizeof(x1));
    for (int i = 0; i < 6; ++i) x1[6 + i] = v1[i];
    se3 p1i = se3_inv(pose1);
    se3 dp = se3_mul(&p1i, pose2);
    se3_log(&dp, xi12);
    for (int i = 0; i < 6; ++i) x2[i] = xi12[i];
    right_jac_pose3_inv(xi12, Jri);
    mat_mul(x2 + 6, Jri, v2, 6, 6, 1);
    double a[6], b[6], xi[6];
    mat_mul(a, At1, x1, 6, 12, 1);
    mat_mul(b, Pt1, x2, 6, 12, 1);
    for (int i = 0; i < 6; ++i) xi[i] = a[i] + b[i];
    *dT = se3_exp(xi);
    return se3_mul(pose1, dT);
}

/* ------------------------------------------------------------------ Pinhole (Pinhole.cpp) */
/* the camera and its VertexExtrinsic (include/G2oTypes.h:83-102): Tbc is the vertex estimate; ext_free
 * marks it optimisable (bExtrinsic, src/Optimizer.cc:1228-1240), with its EdgeExtrinsicPrior
 * R_ = mRbc_ini^-1 and information (include/G2oTypes.h:470-494, src/Optimizer.cc:990-993) */
typedef struct { se3 Tbc; double fx, fy, cx, cy; int ext_free, hidx; quat Rini_inv; double info[9]; } cam_t;

static void pin_project(const cam_t* c, const double* X, double* uv) {   /* :35-41 */
    uv[0] = c->fx * X[0] / X[2] + c->cx;
    uv[1] = c->fy * X[1] / X[2] + c->cy;
}
static void pin_project_jac(const cam_t* c, const double* X, double* J) {   /* :71-81 */
    J[0] = c->fx / X[2]; J[1] = 0.0; J[2] = -c->fx * X[0] / (X[2] * X[2]);
    J[3] = 0.0; J[4] = c->fy / X[2]; J[5] = -c->fy * X[1] / (X[2] * X[2]);
}

/* ------------------------------------------------------------------ problem */
typedef struct { se3 Twb; double vel[6]; double time, bf; int fixed; } kf_t;

struct orc_problem {
    lba_config cfg;
    gp_t gp;
    int n_kf, n_lm, n_obs, n_prior, n_vel, n_cam;
    kf_t* kf;          /* current estimate */
    double* lm;        /* [n_lm*3] */
    kf_t* kf_bak;      /* push/pop backup (BaseVertex::push/pop, base_vertex.h:96-98) */
    double* lm_bak;
    lba_obs* obs;
    lba_prior* pri;
    int* vel;
    cam_t* cam;
    se3* cam_bak;      /* extrinsic estimates, push/pop */
    /* index mapping (SparseOptimizer::buildIndexMapping, sparse_optimizer.cpp:166-190): keyframe blocks
     * (12 wide) then free extrinsics (6 wide, VertexExtrinsic ids iniMPid + c + 1 follow every KF id) */
    int* poff;         /* per pose block: offset in the pose system */
    int* pdim;         /* per pose block: 12 or 6 */
    int* kf_hidx;      /* pose block index or -1 */
    int* lm_hidx;      /* landmark block index or -1 */
    int np, nl;        /* pose dim (12 * #KF blocks + 6 * #free extrinsics), landmark dim (3*#lm blocks) */
    int n_pose_blocks, n_lm_blocks;
    /* per-edge errors */
    double* obs_err;   /* [n_obs*3] */
    double* obs_rho0;  /* [n_obs] robust chi2 of each observation (summed in order after the parallel pass) */
    double* obs_J;     /* [JCHUNK*3*JC] Jacobians of a chunk of observations (filled in parallel, used in order) */
    double* pri_err;   /* [n_prior*12] */
    double* vel_err;   /* [n_vel] */
    /* Hessian (BlockSolver, block_solver.hpp) */
    /* Hpp as g2o's SparseBlockMatrix holds it (sparse_block_matrix.h:40-231): the upper blocks (hi <= hj) of
     * its structural pattern (every pose block's diagonal, the pose pairs of every edge), pdim[hi] x pdim[hj]
     * row-major in 144-double slots; block rows hpp_rowptr[hi] .. hpp_rowptr[hi + 1] - 1, columns hpp_col
     * ascending.  O(blocks), so the normal equations of a 5000-keyframe global BA (np = 59988) fit. */
    int* hpp_rowptr;
    int* hpp_col;
    double* hpp_blk;
    int hpp_nblk;
    double* Hll;       /* [n_lm_blocks*9] */
    int* hpl_start;    /* per landmark block: range into hpl_pose/hpl_blk */
    int* hpl_pose;     /* pose block index, ascending within a landmark */
    double* hpl_blk;   /* 12x3 blocks (an extrinsic's block uses its first 6 rows) */
    double* b;         /* [np + nl] */
    double* x;         /* [np + nl], persistent like BlockSolver::_x */
    double* diag_bak;  /* setLambda backup */
    /* LM */
    double lambda, ni;
    int nBad;
};

static int cmp_int(const void* a, const void* b) {
    const int x = *(const int*)a, y = *(const int*)b;
    return (x > y) - (x < y);
}

static se3 mk_se3(const double* q, const double* t) {
    se3 r;
    r.q.x = q[0]; r.q.y = q[1]; r.q.z = q[2]; r.q.w = q[3];
    r.t[0] = t[0]; r.t[1] = t[1]; r.t[2] = t[2];
    /* the reference widens float poses with Sophus cast<double>(), whose SO3 constructor
     * re-normalises the quaternion (so3.hpp:167-168, :481-487) */
    r.q = q_normalized(r.q);
    return r;
}
static int obs_dim(int kind) { return (kind == LBA_STEREO_GP || kind == LBA_STEREO) ? 3 : 2; }
static int is_gp(int kind) { return kind == LBA_MONO_GP || kind == LBA_STEREO_GP; }
static double obs_delta(const orc_problem* p, int kind) {
    return obs_dim(kind) == 3 ? p->cfg.huber_stereo : p->cfg.huber_mono;
}

/* RobustKernelHuber::robustify (robust_kernel_impl.cpp:76-90) */
static void huber(double e, double delta, double* rho) {
    double dsqr = delta * delta;
    if (e <= dsqr) { rho[0] = e; rho[1] = 1.0; rho[2] = 0.0; }
    else {
        double sqrte = sqrt(e);
        rho[0] = 2 * sqrte * delta - dsqr;
        rho[1] = delta / sqrte;
        rho[2] = -0.5 * rho[1] / e;
    }
}

/* EdgeMonoGPExtrinsic/EdgeMonoGP/EdgeStereoGP computeError (src/G2oTypes.cc:225-256,369-387)
 * and EdgeMono/EdgeStereo computeError (include/G2oTypes.h:423-468, PoseVelocity::Project
 * src/G2oTypes.cc:48-63). */
static void obs_error(const orc_problem* p, const lba_obs* o, double* e) {
    const cam_t* c = &p->cam[o->cam];
    const double* Xw = p->lm + 3 * o->lm;
    double Xc[3], uv[2];
    if (is_gp(o->kind)) {
        const kf_t* f1 = &p->kf[o->kf_a];
        const kf_t* f2 = &p->kf[o->kf_b];
        double At1[72], Pt1[72], xi12[6];
        se3 dT;
        se3 Twb = gp_query_pose(&p->gp, &f1->Twb, &f2->Twb, f1->vel, f2->vel, f1->time, f2->time, o->t, At1, Pt1, &dT, xi12);
        se3 Twc = se3_mul(&Twb, &c->Tbc);
        se3 Tcw = se3_inv(&Twc);
        se3_act(&Tcw, Xw, Xc);
        pin_project(c, Xc, uv);
        e[0] = o->z[0] - uv[0];
        e[1] = o->z[1] - uv[1];
        if (o->kind == LBA_STEREO_GP) {
            double invZ = 1 / Xc[2];
            e[2] = o->z[2] - (uv[0] - f1->bf * invZ);
        } else e[2] = 0.0;
    } else {
        const kf_t* f = &p->kf[o->kf_b];
        se3 Twc = se3_mul(&f->Twb, &c->Tbc);
        se3 Tcw = se3_inv(&Twc);
        se3_act(&Tcw, Xw, Xc);
        pin_project(c, Xc, uv);
        e[0] = o->z[0] - uv[0];
        e[1] = o->z[1] - uv[1];
        if (o->kind == LBA_STEREO) {
            double invZ = 1 / Xc[2];
            e[2] = o->z[2] - (uv[0] - f->bf * invZ);
        } else e[2] = 0.0;
    }
}

/* linearizeOplus of the reprojection edges (src/G2oTypes.cc:258-314,316-367,389-443,445-495).
 * J is [dim x JC]: cols 0-11 KF_a, 12-23 KF_b, 24-26 point, 27-32 the camera extrinsic
 * (EdgeMonoGPExtrinsic's _jacobianOplus[3] = -proj_jac [-I, Skew(Xc)], src/G2oTypes.cc:310-313). */
#define JC 33
#define JCHUNK 65536   /* observations whose Jacobians are held at once (build_system) */
static void obs_jacobian(const orc_problem* p, const lba_obs* o, double* J) {
    const cam_t* c = &p->cam[o->cam];
    const double* Xw = p->lm + 3 * o->lm;
    int dim = obs_dim(o->kind);
    memset(J, 0, sizeof(double) * dim * JC);
    se3 Tcb = se3_inv(&c->Tbc);
    double Rcb[9], Rwb[9], Rbw[9], Xb[3], Xc[3], pj[6], proj[9];
    if (is_gp(o->kind)) {
        const kf_t* f1 = &p->kf[o->kf_a];
        const kf_t* f2 = &p->kf[o->kf_b];
        double At1[72], Pt1[72], xi12[6];
        se3 dT;
        se3 Twb = gp_query_pose(&p->gp, &f1->Twb, &f2->Twb, f1->vel, f2->vel, f1->time, f2->time, o->t, At1, Pt1, &dT, xi12);
        so3_matrix(&Twb.q, Rwb);
        mat_tr(Rbw, Rwb, 3, 3);
        se3 Tbw = se3_inv(&Twb);
        se3_act(&Tbw, Xw, Xb);
        se3_act(&Tcb, Xb, Xc);
        pin_project_jac(c, Xc, pj);
        memcpy(proj, pj, sizeof(pj));
        if (dim == 3) {
            double inv_z2 = 1.0 / (Xc[2] * Xc[2]);
            proj[6] = pj[0]; proj[7] = pj[1]; proj[8] = pj[2] + f1->bf * inv_z2;
        }
        double S[18], SX[9], RS[9];
        so3_matrix(&Tcb.q, Rcb);
        hat3(SX, Xb);
        mat_mul(RS, Rcb, SX, 3, 3, 3);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) { S[i * 6 + j] = -Rcb[i * 3 + j]; S[i * 6 + 3 + j] = RS[i * 3 + j]; }
        double J1[18];
        mat_mul(J1, proj, S, dim, 3, 6);
        mat_scale(J1, -1.0, dim * 6);
        double dxi[6], mdxi[6], AddT[36], Jr_dxi[36], Jr_inv[36], ad_v2[36], adT12[36], adT12inv[36];
        se3_log(&dT, dxi);
        for (int i = 0; i < 6; ++i) mdxi[i] = -dxi[i];
        se3 emd = se3_exp(mdxi);
        se3_adj(&emd, AddT);
        right_jac_pose3(dxi, Jr_dxi);
        right_jac_pose3_inv(xi12, Jr_inv);
        se3_ad(f2->vel, ad_v2);
        se3 eT12 = se3_exp(xi12);
        se3_adj(&eT12, adT12);
        lu_inverse(adT12inv, adT12, 6);
        double JinT1[72], JinV1[72], JinT2[72], JinV2[72], top[36], bot[36];
        mat_mul(top, Jr_inv, adT12inv, 6, 6, 6);
        mat_scale(top, -1.0, 36);
        mat_mul(bot, ad_v2, top, 6, 6, 6);
        mat_scale(bot, -0.5, 36);
        set_block(JinT1, 6, 0, 0, top, 6, 6);
        set_block(JinT1, 6, 6, 0, bot, 6, 6);
        memset(JinV1, 0, sizeof(JinV1));
        for (int i = 0; i < 6; ++i) JinV1[(6 + i) * 6 + i] = 1.0;
        mat_mul(bot, ad_v2, Jr_inv, 6, 6, 6);
        mat_scale(bot, -0.5, 36);
        set_block(JinT2, 6, 0, 0, Jr_inv, 6, 6);
        set_block(JinT2, 6, 6, 0, bot, 6, 6);
        memset(JinV2, 0, sizeof(JinV2));
        set_block(JinV2, 6, 6, 0, Jr_inv, 6, 6);
        /* _jacobianOplus[0] = [J1 (Jr_dxi Pt1 JinT1 + Ad_dT) | J1 Jr_dxi At1 JinV1] */
        double JP[72], JPJ[36], J1Jr[18], J1JrA[36], blk[18];
        mat_mul(JP, Jr_dxi, Pt1, 6, 6, 12);
        mat_mul(JPJ, JP, JinT1, 6, 12, 6);
        for (int i = 0; i < 36; ++i) JPJ[i] += AddT[i];
        mat_mul(blk, J1, JPJ, dim, 6, 6);
        set_block(J, JC, 0, 0, blk, dim, 6);
        mat_mul(J1Jr, J1, Jr_dxi, dim, 6, 6);
        mat_mul(J1JrA, J1Jr, At1, dim, 6, 12);
        mat_mul(blk, J1JrA, JinV1, dim, 12, 6);
        set_block(J, JC, 0, 6, blk, dim, 6);
        /* Jj1 = J1 Jr_dxi Pt1; _jacobianOplus[1] = [Jj1 JinT2 | Jj1 JinV2] */
        double Jj1[36];
        mat_mul(Jj1, J1Jr, Pt1, dim, 6, 12);
        mat_mul(blk, Jj1, JinT2, dim, 12, 6);
        set_block(J, JC, 0, 12, blk, dim, 6);
        mat_mul(blk, Jj1, JinV2, dim, 12, 6);
        set_block(J, JC, 0, 18, blk, dim, 6);
        /* _jacobianOplus[2] = -proj_jac Rcb Rbw */
        double PR[9], PRR[9];
        mat_mul(PR, proj, Rcb, dim, 3, 3);
        mat_mul(PRR, PR, Rbw, dim, 3, 3);
        mat_scale(PRR, -1.0, dim * 3);
        set_block(J, JC, 0, 24, PRR, dim, 3);
        if (o->kind == LBA_MONO_GP) {   /* SE3deriv2 = [-I, Skew(Xc)]; J_ext = -proj_jac SE3deriv2 */
            double S2[18], SXc[9], PE[18];
            hat3(SXc, Xc);
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) { S2[i * 6 + j] = (i == j) ? -1.0 : 0.0; S2[i * 6 + 3 + j] = SXc[i * 3 + j]; }
            mat_mul(PE, proj, S2, dim, 3, 6);
            mat_scale(PE, -1.0, dim * 6);
            set_block(J, JC, 0, 27, PE, dim, 6);
        }
    } else {
        const kf_t* f = &p->kf[o->kf_b];
        so3_matrix(&f->Twb.q, Rwb);
        mat_tr(Rbw, Rwb, 3, 3);
        se3 Tbw = se3_inv(&f->Twb);
        se3_act(&Tbw, Xw, Xb);
        se3_act(&Tcb, Xb, Xc);
        pin_project_jac(c, Xc, pj);
        memcpy(proj, pj, sizeof(pj));
        if (dim == 3) {
            double inv_z2 = 1.0 / (Xc[2] * Xc[2]);
            proj[6] = pj[0]; proj[7] = pj[1]; proj[8] = pj[2] + f->bf * inv_z2;
        }
        double S[18], SX[9], RS[9], blk[18];
        so3_matrix(&Tcb.q, Rcb);
        hat3(SX, Xb);
        mat_mul(RS, Rcb, SX, 3, 3, 3);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) { S[i * 6 + j] = -Rcb[i * 3 + j]; S[i * 6 + 3 + j] = RS[i * 3 + j]; }
        mat_mul(blk, proj, S, dim, 3, 6);
        mat_scale(blk, -1.0, dim * 6);
        set_block(J, JC, 0, 12, blk, dim, 6);   /* velocity columns stay zero */
        double PR[9], PRR[9];
        mat_mul(PR, proj, Rcb, dim, 3, 3);
        mat_mul(PRR, PR, Rbw, dim, 3, 3);
        mat_scale(PRR, -1.0, dim * 3);
        set_block(J, JC, 0, 24, PRR, dim, 3);
    }
}

/* EdgeGaussianPrior computeError (include/G2oTypes.h:155-163) */
static void prior_error(const orc_problem* p, const lba_prior* e, double* err) {
    const kf_t* f1 = &p->kf[e->kf_a];
    const kf_t* f2 = &p->kf[e->kf_b];
    se3 i1 = se3_inv(&f1->Twb);
    se3 T = se3_mul(&i1, &f2->Twb);
    double dxi[6], Jri[36], r[6];
    se3_log(&T, dxi);
    for (int i = 0; i < 6; ++i) err[i] = dxi[i] - (f2->time - f1->time) * f1->vel[i];
    right_jac_pose3_inv(dxi, Jri);
    mat_mul(r, Jri, f2->vel, 6, 6, 1);
    for (int i = 0; i < 6; ++i) err[6 + i] = r[i] - f1->vel[i];
}
/* EdgeGaussianPrior::linearizeOplus (src/G2oTypes.cc:100-118) */
static void prior_jacobian(const orc_problem* p, const lba_prior* e, double* Ji, double* Jj) {
    const kf_t* f1 = &p->kf[e->kf_a];
    const kf_t* f2 = &p->kf[e->kf_b];
    se3 i1 = se3_inv(&f1->Twb);
    se3 T = se3_mul(&i1, &f2->Twb);
    double xi[6], Jri[36], adv2[36], AdT[36], AdTinv[36], top[36], bot[36];
    se3_log(&T, xi);
    right_jac_pose3_inv(xi, Jri);
    se3_ad(f2->vel, adv2);
    se3_adj(&T, AdT);
    lu_inverse(AdTinv, AdT, 6);
    memset(Ji, 0, sizeof(double) * 144);
    memset(Jj, 0, sizeof(double) * 144);
    mat_mul(top, Jri, AdTinv, 6, 6, 6);
    mat_scale(top, -1.0, 36);
    mat_mul(bot, adv2, top, 6, 6, 6);
    mat_scale(bot, -0.5, 36);
    set_block(Ji, 12, 0, 0, top, 6, 6);
    set_block(Ji, 12, 6, 0, bot, 6, 6);
    double dt = f2->time - f1->time;
    for (int i = 0; i < 6; ++i) { Ji[i * 12 + 6 + i] = -dt; Ji[(6 + i) * 12 + 6 + i] = -1.0; }
    mat_mul(bot, adv2, Jri, 6, 6, 6);
    mat_scale(bot, -0.5, 36);
    set_block(Jj, 12, 0, 0, Jri, 6, 6);
    set_block(Jj, 12, 6, 0, bot, 6, 6);
    set_block(Jj, 12, 6, 6, Jri, 6, 6);
}

/* EdgeExtrinsicPrior (include/G2oTypes.h:479-491): e = (R_ * T.so3()).log(); Jacobian block (0, 3) =
 * RightJacobianSO3(e).inverse() (src/G2oTypes.cc:575-591; Eigen's 3x3 inverse), block (0, 0) zero */
static void ext_prior_error(const cam_t* c, double* e) {
    quat q = so3_mul(c->Rini_inv, c->Tbc.q);
    double th;
    so3_log_theta(&q, e, &th);
}
static void ext_prior_jacobian(const double* e, double* J /* 3 x 6 */) {
    const double x = e[0], y = e[1], z = e[2];
    const double d2 = x * x + y * y + z * z, d = sqrt(d2);
    double Jr[9], W[9] = {0.0, -z, y, z, 0.0, -x, -y, x, 0.0}, WW[9], Ji[9];
    mat_eye(Jr, 3);
    if (!(d < 1e-5)) {
        mat_mul(WW, W, W, 3, 3, 3);
        for (int i = 0; i < 9; ++i) Jr[i] = Jr[i] - W[i] * (1.0 - cos(d)) / d2 + WW[i] * (d - sin(d)) / (d2 * d);
    }
    inverse3(Ji, Jr);
    memset(J, 0, sizeof(double) * 18);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) J[i * 6 + 3 + j] = Ji[i * 3 + j];
}

/* ------------------------------------------------------------------ construction */
orc_problem* orc_create(const lba_config* cfg, const lba_kf* kfs, int n_kf, const double* lm_xyz, int n_lm,
                        const lba_obs* obs, int n_obs, const lba_prior* priors, int n_priors,
                        const int* vel_kfs, int n_vel, const lba_cam* cams, int n_cam) {
    orc_problem* p = (orc_problem*)calloc(1, sizeof(orc_problem));
    p->cfg = *cfg;
    memcpy(p->gp.Qc, cfg->qc, sizeof(p->gp.Qc));
    lu_inverse(p->gp.QcInv, p->gp.Qc, 6);   /* GaussianProcess(Qc): mQcInv(Qc.inverse()) */
    p->n_kf = n_kf; p->n_lm = n_lm; p->n_obs = n_obs; p->n_prior = n_priors; p->n_vel = n_vel; p->n_cam = n_cam;
    p->kf = (kf_t*)calloc(n_kf > 0 ? n_kf : 1, sizeof(kf_t));
    p->kf_bak = (kf_t*)calloc(n_kf > 0 ? n_kf : 1, sizeof(kf_t));
    for (int i = 0; i < n_kf; ++i) {
        p->kf[i].Twb = mk_se3(kfs[i].q, kfs[i].t);
        memcpy(p->kf[i].vel, kfs[i].vel, sizeof(double) * 6);
        p->kf[i].time = kfs[i].time;
        p->kf[i].bf = kfs[i].bf;
        p->kf[i].fixed = kfs[i].fixed;
    }
    p->lm = (double*)malloc(sizeof(double) * 3 * (n_lm > 0 ? n_lm : 1));
    p->lm_bak = (double*)malloc(sizeof(double) * 3 * (n_lm > 0 ? n_lm : 1));
    memcpy(p->lm, lm_xyz, sizeof(double) * 3 * n_lm);
    p->obs = (lba_obs*)malloc(sizeof(lba_obs) * (n_obs > 0 ? n_obs : 1));
    memcpy(p->obs, obs, sizeof(lba_obs) * n_obs);
    p->pri = (lba_prior*)malloc(sizeof(lba_prior) * (n_priors > 0 ? n_priors : 1));
    memcpy(p->pri, priors, sizeof(lba_prior) * n_priors);
    p->vel = (int*)malloc(sizeof(int) * (n_vel > 0 ? n_vel : 1));
    memcpy(p->vel, vel_kfs, sizeof(int) * n_vel);
    p->cam = (cam_t*)malloc(sizeof(cam_t) * (n_cam > 0 ? n_cam : 1));
    p->cam_bak = (se3*)malloc(sizeof(se3) * (n_cam > 0 ? n_cam : 1));
    for (int c = 0; c < n_cam; ++c) {
        p->cam[c].Tbc = mk_se3(cams[c].q, cams[c].t);
        p->cam[c].fx = cams[c].fx; p->cam[c].fy = cams[c].fy;
        p->cam[c].cx = cams[c].cx; p->cam[c].cy = cams[c].cy;
        p->cam[c].ext_free = cams[c].ext_free != 0;
        p->cam[c].hidx = -1;
        /* EdgeExtrinsicPrior(mRbc_ini[c].cast<double>()): R_(R.inverse()) */
        quat ri = {cams[c].rbc_ini[0], cams[c].rbc_ini[1], cams[c].rbc_ini[2], cams[c].rbc_ini[3]};
        p->cam[c].Rini_inv = so3_inv(q_normalized(ri));
        memcpy(p->cam[c].info, cams[c].rbc_info, sizeof(double) * 9);
    }
    /* active vertices: touched by at least one edge that is not all-fixed
     * (SparseOptimizer::initializeOptimization, sparse_optimizer.cpp:197-267) */
    int* kf_act = (int*)calloc(n_kf > 0 ? n_kf : 1, sizeof(int));
    int* lm_act = (int*)calloc(n_lm > 0 ? n_lm : 1, sizeof(int));
    for (int i = 0; i < n_obs; ++i) {   /* the landmark is never fixed: every obs edge is active */
        lm_act[obs[i].lm] = 1;
        kf_act[obs[i].kf_b] = 1;
        if (is_gp(obs[i].kind)) kf_act[obs[i].kf_a] = 1;
    }
    for (int i = 0; i < n_priors; ++i)
        if (!(kfs[priors[i].kf_a].fixed && kfs[priors[i].kf_b].fixed)) { kf_act[priors[i].kf_a] = 1; kf_act[priors[i].kf_b] = 1; }
    for (int i = 0; i < n_vel; ++i)
        if (!kfs[vel_kfs[i]].fixed) kf_act[vel_kfs[i]] = 1;
    p->kf_hidx = (int*)malloc(sizeof(int) * (n_kf > 0 ? n_kf : 1));
    p->lm_hidx = (int*)malloc(sizeof(int) * (n_lm > 0 ? n_lm : 1));
    int np = 0, nl = 0;
    for (int i = 0; i < n_kf; ++i) p->kf_hidx[i] = (kf_act[i] && !kfs[i].fixed) ? np++ : -1;
    for (int i = 0; i < n_lm; ++i) p->lm_hidx[i] = lm_act[i] ? nl++ : -1;
    const int npk = np;
    for (int c = 0; c < n_cam; ++c)   /* a free extrinsic is active through its prior edge */
        if (p->cam[c].ext_free) p->cam[c].hidx = np++;
    free(kf_act);
    free(lm_act);
    p->n_pose_blocks = np;
    p->n_lm_blocks = nl;
    p->poff = (int*)malloc(sizeof(int) * (np > 0 ? np : 1));
    p->pdim = (int*)malloc(sizeof(int) * (np > 0 ? np : 1));
    for (int h = 0; h < np; ++h) {
        p->poff[h] = h < npk ? 12 * h : 12 * npk + 6 * (h - npk);
        p->pdim[h] = h < npk ? 12 : 6;
    }
    p->np = 12 * npk + 6 * (np - npk);
    p->nl = 3 * nl;
    p->obs_err = (double*)calloc(3 * (n_obs > 0 ? n_obs : 1), sizeof(double));
    p->obs_rho0 = (double*)calloc(n_obs > 0 ? n_obs : 1, sizeof(double));
    p->obs_J = (double*)calloc((size_t)3 * 33 * JCHUNK, sizeof(double));
    p->pri_err = (double*)calloc(12 * (n_priors > 0 ? n_priors : 1), sizeof(double));
    p->vel_err = (double*)calloc((n_vel > 0 ? n_vel : 1), sizeof(double));
    p->Hll = (double*)calloc(9 * (nl > 0 ? nl : 1), sizeof(double));
    /* the pose vertices of every edge (hessian indices, -1 for fixed / absent), for the patterns below */
#define OBS_POSE_VERTS(o, hs)                                                                   \
    do {                                                                                        \
        (hs)[0] = p->kf[(o)->kf_b].fixed ? -1 : p->kf_hidx[(o)->kf_b];                           \
        (hs)[1] = is_gp((o)->kind) && !p->kf[(o)->kf_a].fixed ? p->kf_hidx[(o)->kf_a] : -1;       \
        (hs)[2] = (o)->kind == LBA_MONO_GP ? p->cam[(o)->cam].hidx : -1;                         \
    } while (0)
    /* Hpp pattern: per block row the partner columns (candidates with duplicates, counted then filled),
     * each row's list sorted and made unique */
    {
        int* cnt = (int*)calloc(np + 1, sizeof(int));
        for (int pass = 0; pass < 2; ++pass) {
            int* fill = pass ? (int*)calloc(np + 1, sizeof(int)) : NULL;
            int* cand = pass ? (int*)malloc(sizeof(int) * (cnt[np] > 0 ? cnt[np] : 1)) : NULL;
#define HPP_CAND(a, b)                                                                          \
            do {                                                                                \
                const int lo_ = (a) < (b) ? (a) : (b), hi_ = (a) < (b) ? (b) : (a);             \
                if (pass) cand[cnt[lo_] + fill[lo_]++] = hi_; else cnt[lo_ + 1]++;               \
            } while (0)
            for (int h = 0; h < np; ++h) HPP_CAND(h, h);
            for (int i = 0; i < n_priors; ++i) {
                if (kfs[priors[i].kf_a].fixed && kfs[priors[i].kf_b].fixed) continue;
                const int a = kfs[priors[i].kf_a].fixed ? -1 : p->kf_hidx[priors[i].kf_a];
                const int b = kfs[priors[i].kf_b].fixed ? -1 : p->kf_hidx[priors[i].kf_b];
                if (a >= 0 && b >= 0) HPP_CAND(a, b);
            }
            for (int i = 0; i < n_obs; ++i) {
                int hs[3];
                OBS_POSE_VERTS(&obs[i], hs);
                for (int x = 0; x < 3; ++x)
                    for (int y = x + 1; y < 3; ++y)
                        if (hs[x] >= 0 && hs[y] >= 0) HPP_CAND(hs[x], hs[y]);
            }
#undef HPP_CAND
            if (!pass) {
                for (int h = 0; h < np; ++h) cnt[h + 1] += cnt[h];
                continue;
            }
            p->hpp_rowptr = (int*)calloc(np + 1, sizeof(int));
            int nb = 0;
            for (int h = 0; h < np; ++h) {
                int* r = cand + cnt[h];
                const int m = cnt[h + 1] - cnt[h];
                qsort(r, m, sizeof(int), cmp_int);
                int u = 0;
                for (int k = 0; k < m; ++k)
                    if (u == 0 || r[u - 1] != r[k]) r[u++] = r[k];
                nb += u;
                p->hpp_rowptr[h + 1] = nb;
                fill[h] = u;
            }
            p->hpp_nblk = nb;
            p->hpp_col = (int*)malloc(sizeof(int) * (nb > 0 ? nb : 1));
            for (int h = 0; h < np; ++h) memcpy(p->hpp_col + p->hpp_rowptr[h], cand + cnt[h], sizeof(int) * fill[h]);
            p->hpp_blk = (double*)calloc((size_t)144 * (nb > 0 ? nb : 1), sizeof(double));
            free(fill);
            free(cand);
        }
        free(cnt);
    }
    /* Hpl pattern: one 12x3 block per (pose block, landmark block) pair, pose blocks ascending per landmark
     * (the observations grouped by landmark, each landmark's pose blocks sorted and made unique) */
    p->hpl_start = (int*)calloc(nl + 1, sizeof(int));
    {
        int* lo_start = (int*)calloc(nl + 1, sizeof(int));
        for (int i = 0; i < n_obs; ++i) lo_start[p->lm_hidx[obs[i].lm] + 1] += 3;
        for (int l = 0; l < nl; ++l) lo_start[l + 1] += lo_start[l];
        int* lfill = (int*)calloc(nl + 1, sizeof(int));
        int* cand = (int*)malloc(sizeof(int) * (lo_start[nl] > 0 ? lo_start[nl] : 1));
        for (int i = 0; i < n_obs; ++i) {
            const int l = p->lm_hidx[obs[i].lm];
            int hs[3];
            OBS_POSE_VERTS(&obs[i], hs);
            for (int x = 0; x < 3; ++x)
                if (hs[x] >= 0) cand[lo_start[l] + lfill[l]++] = hs[x];
        }
        for (int l = 0; l < nl; ++l) {
            int* r = cand + lo_start[l];
            qsort(r, lfill[l], sizeof(int), cmp_int);
            int u = 0;
            for (int k = 0; k < lfill[l]; ++k)
                if (u == 0 || r[u - 1] != r[k]) r[u++] = r[k];
            lfill[l] = u;
            p->hpl_start[l + 1] = p->hpl_start[l] + u;
        }
        int npairs = p->hpl_start[nl];
        p->hpl_pose = (int*)malloc(sizeof(int) * (npairs > 0 ? npairs : 1));
        p->hpl_blk = (double*)calloc(36 * (size_t)(npairs > 0 ? npairs : 1), sizeof(double));
        for (int l = 0; l < nl; ++l) memcpy(p->hpl_pose + p->hpl_start[l], cand + lo_start[l], sizeof(int) * lfill[l]);
        free(cand);
        free(lfill);
        free(lo_start);
    }
#undef OBS_POSE_VERTS
    p->b = (double*)calloc(p->np + p->nl + 1, sizeof(double));
    p->x = (double*)calloc(p->np + p->nl + 1, sizeof(double));
    p->diag_bak = (double*)calloc(p->np + p->nl + 1, sizeof(double));
    p->lambda = -1.0;
    p->ni = 2.0;
    return p;
}

void orc_destroy(orc_problem* p) {
    if (!p) return;
    free(p->kf); free(p->kf_bak); free(p->lm); free(p->lm_bak); free(p->obs); free(p->pri); free(p->vel);
    free(p->cam); free(p->cam_bak); free(p->poff); free(p->pdim); free(p->kf_hidx); free(p->lm_hidx); free(p->obs_err); free(p->obs_rho0); free(p->obs_J); free(p->pri_err); free(p->vel_err);
    free(p->hpp_rowptr); free(p->hpp_col); free(p->hpp_blk); free(p->Hll); free(p->hpl_start); free(p->hpl_pose); free(p->hpl_blk); free(p->b); free(p->x);
    free(p->diag_bak);
    free(p);
}
int orc_pose_dim(const orc_problem* p) { return p->np; }
int orc_lm_dim(const orc_problem* p) { return p->nl; }

/* ------------------------------------------------------------------ errors */
static double chi2_of(const double* e, int dim, double w) {   /* BaseEdge::chi2, base_edge.h:58-61 */
    double s = 0.0;
    for (int i = 0; i < dim; ++i) s += e[i] * (w * e[i]);
    return s;
}
static double prior_chi2(const orc_problem* p, const lba_prior* e, const double* err) {
    const kf_t* f1 = &p->kf[e->kf_a];
    const kf_t* f2 = &p->kf[e->kf_b];
    double Om[144], Oe[12];
    gp_qi_inv(&p->gp, f2->time - f1->time, Om);
    mat_mul(Oe, Om, err, 12, 12, 1);
    double s = 0.0;
    for (int i = 0; i < 12; ++i) s += err[i] * Oe[i];
    return s;
}
static int prior_active(const orc_problem* p, const lba_prior* e) {
    return !(p->kf[e->kf_a].fixed && p->kf[e->kf_b].fixed);
}

/* SparseOptimizer::computeActiveErrors + activeRobustChi2 (sparse_optimizer.cpp:61-114) */
static double compute_errors(orc_problem* p) {
    double chi = 0.0, rho[3];
    for (int i = 0; i < p->n_vel; ++i) {   /* EdgeVelocity: e = Vel(2), info QcInv(2,2) */
        const kf_t* f = &p->kf[p->vel[i]];
        if (f->fixed) continue;
        p->vel_err[i] = f->vel[2];
        chi += p->vel_err[i] * (p->gp.QcInv[2 * 6 + 2] * p->vel_err[i]);
    }
    for (int i = 0; i < p->n_prior; ++i) {
        if (!prior_active(p, &p->pri[i])) continue;
        prior_error(p, &p->pri[i], p->pri_err + 12 * i);
        double c = prior_chi2(p, &p->pri[i], p->pri_err + 12 * i);
        if (p->cfg.huber_prior > 0) { huber(c, p->cfg.huber_prior, rho); chi += rho[0]; }
        else chi += c;
    }
    for (int c = 0; c < p->n_cam; ++c) {   /* EdgeExtrinsicPrior: active when its vertex is free */
        if (!p->cam[c].ext_free) continue;
        double e[3], Oe[3];
        ext_prior_error(&p->cam[c], e);
        mat_mul(Oe, p->cam[c].info, e, 3, 3, 1);
        chi += e[0] * Oe[0] + e[1] * Oe[1] + e[2] * Oe[2];
    }
    /* per observation in parallel (the OpenMP build, liblba_oracle_omp.so: g2o's computeActiveErrors
     * with G2O_USE_OPENMP, sparse_optimizer.cpp:61-114), then summed in edge order (bitwise the serial
     * build's result) */
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int i = 0; i < p->n_obs; ++i) {
        const lba_obs* o = &p->obs[i];
        double* e = p->obs_err + 3 * i;
        double r3[3];
        obs_error(p, o, e);
        huber(chi2_of(e, obs_dim(o->kind), o->w), obs_delta(p, o->kind), r3);
        p->obs_rho0[i] = r3[0];
    }
    for (int i = 0; i < p->n_obs; ++i) chi += p->obs_rho0[i];
    return chi;
}

double orc_compute_errors(orc_problem* p, double* residuals, double* obs_chi2) {
    double chi = compute_errors(p);
    for (int i = 0; i < p->n_obs; ++i) {
        if (residuals) memcpy(residuals + 3 * i, p->obs_err + 3 * i, 3 * sizeof(double));
        if (obs_chi2) obs_chi2[i] = chi2_of(p->obs_err + 3 * i, obs_dim(p->obs[i].kind), p->obs[i].w);
    }
    return chi;
}

/* chi2 of the stored errors (the last compute_errors: after orc_optimize its last trial state), nothing
 * recomputed: g2o's e->chi2() after optimize() (base_edge.h:58-61) */
void orc_last_obs_chi2(const orc_problem* p, double* obs_chi2) {
    for (int i = 0; i < p->n_obs; ++i) obs_chi2[i] = chi2_of(p->obs_err + 3 * i, obs_dim(p->obs[i].kind), p->obs[i].w);
}

/* ------------------------------------------------------------------ buildSystem */
/* the stored upper block (hi <= hj) of Hpp: pdim[hi] x pdim[hj], row-major */
static double* hpp_block(const orc_problem* p, int hi, int hj) {
    int a = p->hpp_rowptr[hi], b = p->hpp_rowptr[hi + 1];
    while (a < b) {
        const int m = (a + b) >> 1;
        if (p->hpp_col[m] < hj) a = m + 1;
        else b = m;
    }
    if (a == p->hpp_rowptr[hi + 1] || p->hpp_col[a] != hj) {
        fprintf(stderr, "oracle: Hpp block (%d, %d) outside the pattern\n", hi, hj);
        abort();
    }
    return p->hpp_blk + (size_t)144 * a;
}
/* add an (i,j) pose-pose block contribution (pdim[i] x pdim[j], row-major) into the upper triangle of Hpp */
static void hpp_add(orc_problem* p, int hi, int hj, const double* blk) {
    const int di = p->pdim[hi], dj = p->pdim[hj];
    if (hi <= hj) {
        double* B = hpp_block(p, hi, hj);
        for (int r = 0; r < di; ++r)
            for (int c = 0; c < dj; ++c) B[r * dj + c] += blk[r * dj + c];
    } else {   /* transposed block (hessianRowMajor) */
        double* B = hpp_block(p, hj, hi);
        for (int r = 0; r < di; ++r)
            for (int c = 0; c < dj; ++c) B[c * di + r] += blk[r * dj + c];
    }
}
/* element (i, i) of Hpp */
static double* hpp_diag(const orc_problem* p, int h, int r) {
    return hpp_block(p, h, h) + r * p->pdim[h] + r;
}
/* the upper blocks of Hpp into a dense n x n (upper block triangle, the lower part untouched) */
static void hpp_dense_upper(const orc_problem* p, double* H) {
    const size_t n = (size_t)p->np;
    for (int hi = 0; hi < p->n_pose_blocks; ++hi)
        for (int k = p->hpp_rowptr[hi]; k < p->hpp_rowptr[hi + 1]; ++k) {
            const int hj = p->hpp_col[k], di = p->pdim[hi], dj = p->pdim[hj];
            const double* B = p->hpp_blk + (size_t)144 * k;
            for (int r = 0; r < di; ++r)
                for (int c = 0; c < dj; ++c) H[(p->poff[hi] + r) * n + p->poff[hj] + c] = B[r * dj + c];
        }
}
static double* hpl_block(orc_problem* p, int hp, int hl) {
    for (int k = p->hpl_start[hl]; k < p->hpl_start[hl + 1]; ++k)
        if (p->hpl_pose[k] == hp) return p->hpl_blk + 36 * k;
    return NULL;
}

static void build_system(orc_problem* p) {
    memset(p->hpp_blk, 0, sizeof(double) * 144 * (size_t)p->hpp_nblk);
    memset(p->Hll, 0, sizeof(double) * 9 * p->n_lm_blocks);
    memset(p->hpl_blk, 0, sizeof(double) * 36 * p->hpl_start[p->n_lm_blocks]);
    memset(p->b, 0, sizeof(double) * (p->np + p->nl));
    double rho[3];
    /* edges in insertion order of LocalGPBA: velocity, priors, observations */
    for (int i = 0; i < p->n_vel; ++i) {   /* BaseUnaryEdge::constructQuadraticForm (base_unary_edge.hpp:42-72) */
        int k = p->vel[i];
        int h = p->kf_hidx[k];
        if (p->kf[k].fixed || h < 0) continue;
        double om = p->gp.QcInv[2 * 6 + 2];
        double e = p->vel_err[i];
        /* J = [0_{1x6}, A], A = e_2 -> only column 8 */
        p->b[p->poff[h] + 8] -= om * e;
        *hpp_diag(p, h, 8) += om;
    }
    for (int i = 0; i < p->n_prior; ++i) {   /* BaseBinaryEdge::constructQuadraticForm (base_binary_edge.hpp:54-120) */
        const lba_prior* e = &p->pri[i];
        if (!prior_active(p, e)) continue;
        double Ji[144], Jj[144], Om[144], W[144], r[12];
        prior_jacobian(p, e, Ji, Jj);
        gp_qi_inv(&p->gp, p->kf[e->kf_b].time - p->kf[e->kf_a].time, Om);
        const double* err = p->pri_err + 12 * i;
        double wgt = 1.0;
        if (p->cfg.huber_prior > 0) {
            huber(prior_chi2(p, e, err), p->cfg.huber_prior, rho);
            wgt = rho[1];
        }
        for (int k = 0; k < 144; ++k) W[k] = wgt * Om[k];
        mat_mul(r, Om, err, 12, 12, 1);
        for (int k = 0; k < 12; ++k) r[k] = -r[k] * wgt;   /* omega_r = -Omega e (* rho') */
        int hi = p->kf_hidx[e->kf_a], hj = p->kf_hidx[e->kf_b];
        double AT[144], AtW[144], blk[144], g[12];
        if (!p->kf[e->kf_a].fixed && hi >= 0) {
            mat_tr(AT, Ji, 12, 12);
            mat_mul(g, AT, r, 12, 12, 1);
            for (int k = 0; k < 12; ++k) p->b[p->poff[hi] + k] += g[k];
            mat_mul(AtW, AT, W, 12, 12, 12);
            mat_mul(blk, AtW, Ji, 12, 12, 12);
            hpp_add(p, hi, hi, blk);
            if (!p->kf[e->kf_b].fixed && hj >= 0) {
                mat_mul(blk, AtW, Jj, 12, 12, 12);
                hpp_add(p, hi, hj, blk);
            }
        }
        if (!p->kf[e->kf_b].fixed && hj >= 0) {
            mat_tr(AT, Jj, 12, 12);
            mat_mul(g, AT, r, 12, 12, 1);
            for (int k = 0; k < 12; ++k) p->b[p->poff[hj] + k] += g[k];
            mat_mul(AtW, AT, W, 12, 12, 12);
            mat_mul(blk, AtW, Jj, 12, 12, 12);
            hpp_add(p, hj, hj, blk);
        }
    }
    for (int c = 0; c < p->n_cam; ++c) {   /* EdgeExtrinsicPrior (BaseUnaryEdge, base_unary_edge.hpp:42-72) */
        const cam_t* cm = &p->cam[c];
        if (!cm->ext_free) continue;
        double e[3], J[18], JT[18], JtO[18], blk[36], Oe[3], g[6];
        ext_prior_error(cm, e);
        ext_prior_jacobian(e, J);
        mat_tr(JT, J, 3, 6);
        mat_mul(JtO, JT, cm->info, 6, 3, 3);
        mat_mul(blk, JtO, J, 6, 3, 6);
        hpp_add(p, cm->hidx, cm->hidx, blk);
        mat_mul(Oe, cm->info, e, 3, 3, 1);
        mat_mul(g, JT, Oe, 6, 3, 1);
        for (int k = 0; k < 6; ++k) p->b[p->poff[cm->hidx] + k] -= g[k];
    }
    /* the observations' Jacobians in parallel (the OpenMP build: g2o's linearizeOplus over the active
     * edges, block_solver.hpp:378-380), then accumulated in edge order (bitwise the serial build's) */
    for (int c0 = 0; c0 < p->n_obs; c0 += JCHUNK) {   /* (chunks: the Jacobians of all 6M observations of
                                                         * config 4 would take 4.7 GB) */
    const int c1 = p->n_obs - c0 < JCHUNK ? p->n_obs : c0 + JCHUNK;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int i = c0; i < c1; ++i) obs_jacobian(p, &p->obs[i], p->obs_J + (size_t)3 * JC * (i - c0));
    for (int i = c0; i < c1; ++i) {
        const lba_obs* o = &p->obs[i];
        int dim = obs_dim(o->kind);
        const double* e = p->obs_err + 3 * i;
        const double* J = p->obs_J + (size_t)3 * JC * (i - c0);
        huber(chi2_of(e, dim, o->w), obs_delta(p, o->kind), rho);
        double s = rho[1] * o->w;                    /* robustInformation = rho' * Omega */
        double om_r[3];
        for (int d = 0; d < dim; ++d) om_r[d] = -(o->w * e[d]) * rho[1];
        int hl = p->lm_hidx[o->lm];
        /* vertices in edge order: GP edges (KF_a, KF_b, pt[, extrinsic]), binary edges (KF_b, pt);
         * vk: KF index, -1 the point, -2 - c the extrinsic of camera c */
        int vk[4], vc[4], vd[4], nv = 0;
        if (is_gp(o->kind)) { vk[nv] = o->kf_a; vc[nv] = 0; vd[nv++] = 12; }
        vk[nv] = o->kf_b; vc[nv] = 12; vd[nv++] = 12;
        vk[nv] = -1; vc[nv] = 24; vd[nv++] = 3;
        if (o->kind == LBA_MONO_GP) { vk[nv] = -2 - o->cam; vc[nv] = 27; vd[nv++] = 6; }
#define VHIDX(v) ((v) >= 0 ? (p->kf[v].fixed ? -1 : p->kf_hidx[v]) : ((v) == -1 ? hl : p->cam[-2 - (v)].hidx))
        for (int a = 0; a < nv; ++a) {
            int ha = VHIDX(vk[a]);
            if (ha < 0) continue;
            int da = vd[a];
            double AtO[36], gb[12];   /* AtO = A^T (s I) : [da x dim] */
            for (int r = 0; r < da; ++r)
                for (int d = 0; d < dim; ++d) AtO[r * dim + d] = J[d * JC + vc[a] + r] * s;
            for (int r = 0; r < da; ++r) {
                double acc = 0.0;
                for (int d = 0; d < dim; ++d) acc += J[d * JC + vc[a] + r] * om_r[d];
                gb[r] = acc;
            }
            double blk[144];
            for (int r = 0; r < da; ++r)
                for (int c = 0; c < da; ++c) {
                    double acc = 0.0;
                    for (int d = 0; d < dim; ++d) acc += AtO[r * dim + d] * J[d * JC + vc[a] + c];
                    blk[r * da + c] = acc;
                }
            if (vk[a] != -1) {
                for (int r = 0; r < da; ++r) p->b[p->poff[ha] + r] += gb[r];
                hpp_add(p, ha, ha, blk);
            } else {
                for (int r = 0; r < 3; ++r) p->b[p->np + 3 * ha + r] += gb[r];
                for (int r = 0; r < 9; ++r) p->Hll[9 * ha + r] += blk[r];
            }
            for (int c2 = a + 1; c2 < nv; ++c2) {
                int hb = VHIDX(vk[c2]);
                if (hb < 0) continue;
                int db = vd[c2];
                double ob[144];
                for (int r = 0; r < da; ++r)
                    for (int c = 0; c < db; ++c) {
                        double acc = 0.0;
                        for (int d = 0; d < dim; ++d) acc += AtO[r * dim + d] * J[d * JC + vc[c2] + c];
                        ob[r * db + c] = acc;
                    }
                if (vk[a] != -1 && vk[c2] != -1) hpp_add(p, ha, hb, ob);
                else if (vk[c2] == -1) {   /* (pose, point): Hpl */
                    double* B = hpl_block(p, ha, hl);
                    for (int r = 0; r < da * 3; ++r) B[r] += ob[r];
                } else {   /* (point, extrinsic): stored as the extrinsic's Hpl block (pose index first) */
                    double* B = hpl_block(p, hb, hl);
                    for (int r = 0; r < db; ++r)
                        for (int c = 0; c < 3; ++c) B[r * 3 + c] += ob[c * db + r];
                }
            }
        }
    }
    }
}

static void mirror_upper(double* H, int n) {
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j) H[(size_t)i * n + j] = H[(size_t)j * n + i];
}

int orc_build_system(orc_problem* p, double* H_pp, double* b, double* H_ll) {
    compute_errors(p);
    build_system(p);
    if (H_pp) {
        memset(H_pp, 0, sizeof(double) * (size_t)p->np * p->np);
        hpp_dense_upper(p, H_pp);
        mirror_upper(H_pp, p->np);
    }
    if (b) memcpy(b, p->b, sizeof(double) * (p->np + p->nl));
    if (H_ll) {
        memset(H_ll, 0, sizeof(double) * 9 * p->n_lm);
        for (int l = 0; l < p->n_lm; ++l)
            if (p->lm_hidx[l] >= 0) memcpy(H_ll + 9 * l, p->Hll + 9 * p->lm_hidx[l], 9 * sizeof(double));
    }
    return p->np;
}

/* ------------------------------------------------------------------ Eigen LDLT (pivoted) */
/* Eigen 3.3 LDLT.h ldlt_inplace<Lower>::unblocked + LDLT::solve; returns isPositive() */
static int ldlt_solve_inplace(int n, double* A /*full symmetric, destroyed*/, const double* b, double* x) {
    int* tr = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
    double* temp = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
    enum { ZeroSign, PositiveSemiDef, NegativeSemiDef, Indefinite } sign = ZeroSign;
#define M(i, j) A[(size_t)(i) * n + (j)]
    for (int k = 0; k < n; ++k) {
        int big = k;
        double bv = fabs(M(k, k));
        for (int i = k + 1; i < n; ++i)
            if (fabs(M(i, i)) > bv) { bv = fabs(M(i, i)); big = i; }
        tr[k] = big;
        if (k != big) {
            int s = n - big - 1;
            for (int j = 0; j < k; ++j) { double t = M(k, j); M(k, j) = M(big, j); M(big, j) = t; }
            for (int j = 0; j < s; ++j) { double t = M(big + 1 + j, k); M(big + 1 + j, k) = M(big + 1 + j, big); M(big + 1 + j, big) = t; }
            { double t = M(k, k); M(k, k) = M(big, big); M(big, big) = t; }
            for (int i = k + 1; i < big; ++i) { double t = M(i, k); M(i, k) = M(big, i); M(big, i) = t; }
        }
        int rs = n - k - 1;
        if (k > 0) {
            for (int j = 0; j < k; ++j) temp[j] = M(j, j) * M(k, j);
            double d = 0.0;
            for (int j = 0; j < k; ++j) d += M(k, j) * temp[j];
            M(k, k) -= d;
            for (int i = 0; i < rs; ++i) {
                double s2 = 0.0;
                for (int j = 0; j < k; ++j) s2 += M(k + 1 + i, j) * temp[j];
                M(k + 1 + i, k) -= s2;
            }
        }
        double akk = M(k, k);
        int valid = fabs(akk) > 0.0;
        if (rs > 0 && valid)
            for (int i = 0; i < rs; ++i) M(k + 1 + i, k) /= akk;
        if (sign == PositiveSemiDef) { if (akk < 0) sign = Indefinite; }
        else if (sign == NegativeSemiDef) { if (akk > 0) sign = Indefinite; }
        else if (sign == ZeroSign) { if (akk > 0) sign = PositiveSemiDef; else if (akk < 0) sign = NegativeSemiDef; }
    }
    int positive = (sign == PositiveSemiDef || sign == ZeroSign);
    if (positive && x) {
        for (int i = 0; i < n; ++i) x[i] = b[i];
        for (int k = 0; k < n; ++k) { double t = x[k]; x[k] = x[tr[k]]; x[tr[k]] = t; }   /* P b */
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < i; ++j) x[i] -= M(i, j) * x[j];
        for (int i = 0; i < n; ++i) {
            double d = M(i, i);
            if (fabs(d) > DBL_MIN) x[i] /= d; else x[i] = 0.0;
        }
        for (int i = n - 1; i >= 0; --i)
            for (int j = i + 1; j < n; ++j) x[i] -= M(j, i) * x[j];
        for (int k = n - 1; k >= 0; --k) { double t = x[k]; x[k] = x[tr[k]]; x[tr[k]] = t; }
    }
#undef M
    free(tr);
    free(temp);
    return positive;
}

int orc_ldlt_solve(int n, const double* A, const double* b, double* x) {
    double* W = (double*)malloc(sizeof(double) * (size_t)n * n);
    memcpy(W, A, sizeof(double) * (size_t)n * n);
    int ok = ldlt_solve_inplace(n, W, b, x);
    free(W);
    return ok;
}

/* ------------------------------------------------------------------ BlockSolver::solve */
static void set_lambda(orc_problem* p, double lambda) {   /* block_solver.hpp:564-589 */
    int n = p->np;
    for (int h = 0; h < p->n_pose_blocks; ++h)
        for (int r = 0; r < p->pdim[h]; ++r) {
            double* d = hpp_diag(p, h, r);
            p->diag_bak[p->poff[h] + r] = *d;
            *d += lambda;
        }
    for (int l = 0; l < p->n_lm_blocks; ++l)
        for (int d = 0; d < 3; ++d) { p->diag_bak[n + 3 * l + d] = p->Hll[9 * l + 4 * d]; p->Hll[9 * l + 4 * d] += lambda; }
}
static void restore_diagonal(orc_problem* p) {   /* block_solver.hpp:592-604 */
    int n = p->np;
    for (int h = 0; h < p->n_pose_blocks; ++h)
        for (int r = 0; r < p->pdim[h]; ++r) *hpp_diag(p, h, r) = p->diag_bak[p->poff[h] + r];
    for (int l = 0; l < p->n_lm_blocks; ++l)
        for (int d = 0; d < 3; ++d) p->Hll[9 * l + 4 * d] = p->diag_bak[n + 3 * l + d];
}
/* block_solver.hpp:354-486 with LinearSolverDense (linear_solver_dense.h:65-113) */
static int block_solve(orc_problem* p) {
    int n = p->np, nlb = p->n_lm_blocks;
    double* S = (double*)malloc(sizeof(double) * ((size_t)n * n + 1));
    double* coeff = (double*)calloc(n + 1, sizeof(double));
    double* Dinv = (double*)malloc(sizeof(double) * 9 * (nlb > 0 ? nlb : 1));
    double* dbl = (double*)malloc(sizeof(double) * 3 * (nlb > 0 ? nlb : 1));
    memset(S, 0, sizeof(double) * (size_t)n * n);
    hpp_dense_upper(p, S);   /* Hschur = Hpp (upper blocks used) */
    /* (the OpenMP build: landmark inverses in parallel; the Schur complement with every pose block row
     * owned by one thread that walks the landmarks in order, so each entry of S and coeff receives its
     * terms in the serial order: bitwise the serial build's; block_solver.hpp:381-432,527) */
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int l = 0; l < nlb; ++l) {
        inverse3(Dinv + 9 * l, p->Hll + 9 * l);
        mat_mul(dbl + 3 * l, Dinv + 9 * l, p->b + n + 3 * l, 3, 3, 1);
    }
#ifdef _OPENMP
#pragma omp parallel
#endif
    {
#ifdef _OPENMP
    const int nth = omp_get_num_threads(), th = omp_get_thread_num();
#else
    const int nth = 1, th = 0;
#endif
    for (int l = 0; l < nlb; ++l) {
        double* Di = Dinv + 9 * l;
        const double* db = dbl + 3 * l;
        for (int k1 = p->hpl_start[l]; k1 < p->hpl_start[l + 1]; ++k1) {
            int i1 = p->hpl_pose[k1];
            if (i1 % nth != th) continue;
            const double* Bi = p->hpl_blk + 36 * k1;
            const int d1 = p->pdim[i1], o1 = p->poff[i1];
            double BD[36], Bb[12];
            mat_mul(BD, Bi, Di, d1, 3, 3);
            mat_mul(Bb, Bi, db, d1, 3, 1);
            for (int r = 0; r < d1; ++r) coeff[o1 + r] += Bb[r];
            for (int k2 = k1; k2 < p->hpl_start[l + 1]; ++k2) {
                int i2 = p->hpl_pose[k2];
                const double* Bj = p->hpl_blk + 36 * k2;
                for (int r = 0; r < d1; ++r)
                    for (int c = 0; c < p->pdim[i2]; ++c) {
                        double acc = 0.0;
                        for (int a = 0; a < 3; ++a) acc += BD[r * 3 + a] * Bj[c * 3 + a];
                        S[(size_t)(o1 + r) * n + p->poff[i2] + c] -= acc;
                    }
            }
        }
    }
    }
    mirror_upper(S, n);
    double* bs = (double*)malloc(sizeof(double) * (n + 1));
    for (int i = 0; i < n; ++i) bs[i] = p->b[i] - coeff[i];
    double* xp = (double*)malloc(sizeof(double) * (n + 1));
    int ok = ldlt_solve_inplace(n, S, bs, xp);
    if (ok) {
        memcpy(p->x, xp, sizeof(double) * n);
        /* landmarks: xl = Dinv (bl - Hpl^T xp) */
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
        for (int l = 0; l < nlb; ++l) {
            double cl[3];
            for (int d = 0; d < 3; ++d) cl[d] = p->b[n + 3 * l + d];
            for (int k = p->hpl_start[l]; k < p->hpl_start[l + 1]; ++k) {
                int i1 = p->hpl_pose[k];
                const double* B = p->hpl_blk + 36 * k;
                for (int d = 0; d < 3; ++d) {
                    double acc = 0.0;
                    for (int r = 0; r < p->pdim[i1]; ++r) acc += B[r * 3 + d] * (-p->x[p->poff[i1] + r]);
                    cl[d] += acc;
                }
            }
            mat_mul(p->x + n + 3 * l, Dinv + 9 * l, cl, 3, 3, 1);
        }
    }
    free(S); free(coeff); free(Dinv); free(dbl); free(bs); free(xp);
    return ok;
}

int orc_solve(orc_problem* p, double lambda, double* dx) {
    set_lambda(p, lambda);
    int ok = block_solve(p);
    restore_diagonal(p);
    if (dx) memcpy(dx, p->x, sizeof(double) * (p->np + p->nl));
    return ok;
}

/* Size-independent check of a damped step (the linear system block_solver.hpp:354-486 solves):
 * r = (H + lambda I) dx - b over the full [pose | landmark] system of the last buildSystem, with
 * H's upper Hpp, Hpl and Hll blocks (block_solver.hpp:564-589 for the damping).  O(nnz), so the
 * GPU step can be checked at sizes where the dense pivoted LDLT takes too long. */
void orc_normal_residual(const orc_problem* p, double lambda, const double* dx, double* r) {
    const int n = p->np, nlb = p->n_lm_blocks;
    for (int i = 0; i < n + p->nl; ++i) r[i] = -p->b[i];
    for (int hi = 0; hi < p->n_pose_blocks; ++hi)
        for (int k = p->hpp_rowptr[hi]; k < p->hpp_rowptr[hi + 1]; ++k) {
            const int hj = p->hpp_col[k], di = p->pdim[hi], dj = p->pdim[hj], oi = p->poff[hi], oj = p->poff[hj];
            const double* B = p->hpp_blk + (size_t)144 * k;
            for (int a = 0; a < di; ++a)
                for (int c = 0; c < dj; ++c) {
                    const double v = B[a * dj + c];
                    if (hi == hj && c < a) continue;        /* a diagonal block's upper triangle */
                    if (hi == hj && c == a) { r[oi + a] += (v + lambda) * dx[oi + a]; continue; }
                    r[oi + a] += v * dx[oj + c];
                    r[oj + c] += v * dx[oi + a];
                }
        }
    for (int l = 0; l < nlb; ++l) {
        const double* xl = dx + n + 3 * l;
        double* rl = r + n + 3 * l;
        for (int d = 0; d < 3; ++d)
            for (int e = 0; e < 3; ++e) rl[d] += (p->Hll[9 * l + 3 * d + e] + (d == e ? lambda : 0.0)) * xl[e];
        for (int k = p->hpl_start[l]; k < p->hpl_start[l + 1]; ++k) {
            const int i1 = p->hpl_pose[k];
            const double* B = p->hpl_blk + 36 * k;
            for (int a = 0; a < p->pdim[i1]; ++a)
                for (int d = 0; d < 3; ++d) {
                    r[p->poff[i1] + a] += B[a * 3 + d] * xl[d];
                    rl[d] += B[a * 3 + d] * dx[p->poff[i1] + a];
                }
        }
    }
}

/* The same over |H + lambda I| |dx| + |b| (d): the componentwise (Oettli-Prager) backward error of the step is
 * max_i |r_i| / d_i, which a backward-stable solve keeps near n eps however ill-conditioned the system is. */
void orc_normal_residual_abs(const orc_problem* p, double lambda, const double* dx, double* d) {
    const int n = p->np, nlb = p->n_lm_blocks;
    for (int i = 0; i < n + p->nl; ++i) d[i] = fabs(p->b[i]);
    for (int hi = 0; hi < p->n_pose_blocks; ++hi)
        for (int k = p->hpp_rowptr[hi]; k < p->hpp_rowptr[hi + 1]; ++k) {
            const int hj = p->hpp_col[k], di = p->pdim[hi], dj = p->pdim[hj], oi = p->poff[hi], oj = p->poff[hj];
            const double* B = p->hpp_blk + (size_t)144 * k;
            for (int a = 0; a < di; ++a)
                for (int c = 0; c < dj; ++c) {
                    const double v = fabs(B[a * dj + c]);
                    if (hi == hj && c < a) continue;
                    if (hi == hj && c == a) { d[oi + a] += fabs(B[a * dj + c] + lambda) * fabs(dx[oi + a]); continue; }
                    d[oi + a] += v * fabs(dx[oj + c]);
                    d[oj + c] += v * fabs(dx[oi + a]);
                }
        }
    for (int l = 0; l < nlb; ++l) {
        const double* xl = dx + n + 3 * l;
        double* dl = d + n + 3 * l;
        for (int a = 0; a < 3; ++a)
            for (int e = 0; e < 3; ++e) dl[a] += fabs(p->Hll[9 * l + 3 * a + e] + (a == e ? lambda : 0.0)) * fabs(xl[e]);
        for (int k = p->hpl_start[l]; k < p->hpl_start[l + 1]; ++k) {
            const int i1 = p->hpl_pose[k];
            const double* B = p->hpl_blk + 36 * k;
            for (int a = 0; a < p->pdim[i1]; ++a)
                for (int e = 0; e < 3; ++e) {
                    d[p->poff[i1] + a] += fabs(B[a * 3 + e]) * fabs(xl[e]);
                    dl[e] += fabs(B[a * 3 + e]) * fabs(dx[p->poff[i1] + a]);
                }
        }
    }
}

/* ------------------------------------------------------------------ LM */
static void push_state(orc_problem* p) {
    memcpy(p->kf_bak, p->kf, sizeof(kf_t) * p->n_kf);
    memcpy(p->lm_bak, p->lm, sizeof(double) * 3 * p->n_lm);
    for (int c = 0; c < p->n_cam; ++c) p->cam_bak[c] = p->cam[c].Tbc;
}
static void pop_state(orc_problem* p) {
    memcpy(p->kf, p->kf_bak, sizeof(kf_t) * p->n_kf);
    memcpy(p->lm, p->lm_bak, sizeof(double) * 3 * p->n_lm);
    for (int c = 0; c < p->n_cam; ++c) p->cam[c].Tbc = p->cam_bak[c];
}
/* SparseOptimizer::update (sparse_optimizer.cpp:422-435), VertexPoseVel::oplusImpl
 * (PoseVelocity::Update src/G2oTypes.cc:41-46), VertexSBAPointXYZ::oplusImpl */
static void apply_update(orc_problem* p, const double* x) {
    for (int k = 0; k < p->n_kf; ++k) {
        int h = p->kf_hidx[k];
        if (h < 0) continue;
        se3 d = se3_exp(x + p->poff[h]);
        p->kf[k].Twb = se3_mul(&p->kf[k].Twb, &d);
        for (int i = 0; i < 6; ++i) p->kf[k].vel[i] += x[p->poff[h] + 6 + i];
    }
    for (int c = 0; c < p->n_cam; ++c) {   /* VertexExtrinsic::oplusImpl: T <- T exp(d) (include/G2oTypes.h:97-99) */
        if (p->cam[c].hidx < 0) continue;
        se3 d = se3_exp(x + p->poff[p->cam[c].hidx]);
        p->cam[c].Tbc = se3_mul(&p->cam[c].Tbc, &d);
    }
    for (int l = 0; l < p->n_lm; ++l) {
        int h = p->lm_hidx[l];
        if (h < 0) continue;
        for (int i = 0; i < 3; ++i) p->lm[3 * l + i] += x[p->np + 3 * h + i];
    }
}
static double compute_lambda_init(const orc_problem* p) {   /* levenberg.cpp:171-185 */
    if (p->cfg.lambda_init > 0) return p->cfg.lambda_init;
    double m = 0.0;
    for (int h = 0; h < p->n_pose_blocks; ++h)
        for (int r = 0; r < p->pdim[h]; ++r) m = fmax(m, fabs(*hpp_diag(p, h, r)));
    for (int l = 0; l < p->n_lm_blocks; ++l)
        for (int d = 0; d < 3; ++d) m = fmax(m, fabs(p->Hll[9 * l + 4 * d]));
    return p->cfg.tau * m;
}
static double compute_scale(const orc_problem* p) {   /* levenberg.cpp:187-194 */
    double s = 0.0;
    for (int j = 0; j < p->np + p->nl; ++j) s += p->x[j] * (p->lambda * p->x[j] + p->b[j]);
    return s;
}

/* OptimizationAlgorithmLevenberg::solve (levenberg.cpp:61-169) */
static int lm_iteration(orc_problem* p, int iteration, int* trials, int* fails, double* last_chi) {
    double currentChi = compute_errors(p);
    double tempChi = currentChi, iniChi = currentChi;
    build_system(p);
    if (iteration == 0) { p->lambda = compute_lambda_init(p); p->ni = 2.0; p->nBad = 0; }
    double rho = 0.0;
    int qmax = 0;
    do {
        push_state(p);
        set_lambda(p, p->lambda);
        int ok2 = block_solve(p);
        apply_update(p, p->x);
        restore_diagonal(p);
        tempChi = compute_errors(p);
        *last_chi = tempChi;   /* activeRobustChi2() of the last computed errors (the stats' chi2_final) */
        if (!ok2) { tempChi = DBL_MAX; (*fails)++; }
        rho = currentChi - tempChi;
        double scale = compute_scale(p) + 1e-3;
        rho /= scale;
        if (rho > 0 && isfinite(tempChi)) {
            double alpha = 1. - pow((2 * rho - 1), 3);
            alpha = fmin(alpha, 2. / 3.);
            double sf = fmax(1. / 3., alpha);
            p->lambda *= sf;
            p->ni = 2;
            currentChi = tempChi;
        } else {
            p->lambda *= p->ni;
            p->ni *= 2;
            pop_state(p);
        }
        qmax++;
    } while (rho < 0 && qmax < p->cfg.max_trials);
    *trials += qmax;
    if (qmax == p->cfg.max_trials || rho == 0) return LBA_RESULT_TERMINATE;
    if (p->cfg.early_stop) {
        if ((iniChi - currentChi) * 1e3 < iniChi) p->nBad++;
        else p->nBad = 0;
        if (p->nBad >= 3) return LBA_RESULT_TERMINATE;
    }
    return LBA_RESULT_OK;
}

int orc_optimize(orc_problem* p, int iters, lba_stats* st) {
    lba_stats s;
    memset(&s, 0, sizeof(s));
    if (p->np + p->nl == 0) return LBA_E_EMPTY;
    s.chi2_initial = compute_errors(p);
    int it = 0, res = LBA_RESULT_OK;
    double last = s.chi2_initial;
    for (int i = 0; i < iters; ++i) {
        res = lm_iteration(p, i, &s.trials, &s.solve_failures, &last);
        ++it;
        /* early_stop == 0 (benchmark mode): every Terminate is ignored so the iteration
         * count is fixed */
        if (res != LBA_RESULT_OK && p->cfg.early_stop) break;
    }
    s.iterations = it;
    s.result = res;
    s.chi2_final = last;
    s.lambda_final = p->lambda;
    if (st) *st = s;
    return it;
}

void orc_get_state(const orc_problem* p, lba_kf* kfs, double* lm_xyz) {
    if (kfs)
        for (int i = 0; i < p->n_kf; ++i) {
            const kf_t* f = &p->kf[i];
            kfs[i].q[0] = f->Twb.q.x; kfs[i].q[1] = f->Twb.q.y; kfs[i].q[2] = f->Twb.q.z; kfs[i].q[3] = f->Twb.q.w;
            memcpy(kfs[i].t, f->Twb.t, sizeof(double) * 3);
            memcpy(kfs[i].vel, f->vel, sizeof(double) * 6);
            kfs[i].time = f->time;
            kfs[i].bf = f->bf;
            kfs[i].fixed = f->fixed;
            kfs[i].pad = 0;
        }
    if (lm_xyz) memcpy(lm_xyz, p->lm, sizeof(double) * 3 * p->n_lm);
}

/* Test hooks for a caller-driven LM (tests/test_gpu_configs.py: config 4 trial by trial): set the estimates (the
 * inverse of orc_get_state; time, bf and fixed flags stay the set-up's), and apply a step dx [np + 3 nl] to them with
 * SparseOptimizer::update's oplus (apply_update above, sparse_optimizer.cpp:422-435). */
void orc_set_state(orc_problem* p, const lba_kf* kfs, const double* lm_xyz) {
    if (kfs)
        for (int i = 0; i < p->n_kf; ++i) {
            kf_t* f = &p->kf[i];
            f->Twb.q.x = kfs[i].q[0]; f->Twb.q.y = kfs[i].q[1]; f->Twb.q.z = kfs[i].q[2]; f->Twb.q.w = kfs[i].q[3];
            memcpy(f->Twb.t, kfs[i].t, sizeof(double) * 3);
            memcpy(f->vel, kfs[i].vel, sizeof(double) * 6);
        }
    if (lm_xyz) memcpy(p->lm, lm_xyz, sizeof(double) * 3 * p->n_lm);
}
void orc_apply_step(orc_problem* p, const double* dx) { apply_update(p, dx); }

void orc_get_cams(const orc_problem* p, lba_cam* cams) {   /* cams holds the set-up cameras; Tbc updated */
    for (int c = 0; c < p->n_cam; ++c) {
        const se3* T = &p->cam[c].Tbc;
        cams[c].q[0] = T->q.x; cams[c].q[1] = T->q.y; cams[c].q[2] = T->q.z; cams[c].q[3] = T->q.w;
        memcpy(cams[c].t, T->t, sizeof(double) * 3);
    }
}

/* isDepthPositive (src/G2oTypes.cc:65-81; GP edges test both KF poses, include/G2oTypes.h:305-314) */
void orc_depth_ok(const orc_problem* p, unsigned char* ok) {
    for (int i = 0; i < p->n_obs; ++i) {
        const lba_obs* o = &p->obs[i];
        const cam_t* c = &p->cam[o->cam];
        int good = 1;
        int ks[2] = {o->kf_b, is_gp(o->kind) ? o->kf_a : -1};
        for (int s = 0; s < 2; ++s) {
            if (ks[s] < 0) continue;
            se3 Twc = se3_mul(&p->kf[ks[s]].Twb, &c->Tbc);
            se3 Tcw = se3_inv(&Twc);
            double Xc[3];
            se3_act(&Tcw, p->lm + 3 * o->lm, Xc);
            if (!(Xc[2] > 0)) good = 0;
        }
        ok[i] = (unsigned char)good;
    }
}

int orc_obs_linearize(orc_problem* p, int i, double* err, double* J) {
    const lba_obs* o = &p->obs[i];
    double e[3];
    obs_error(p, o, e);
    if (err) memcpy(err, e, sizeof(e));
    if (J) {   /* the public layout keeps the 27 vertex columns (KF_a, KF_b, point) */
        double Jf[3 * JC];
        obs_jacobian(p, o, Jf);
        for (int d = 0; d < obs_dim(o->kind); ++d) memcpy(J + 27 * d, Jf + JC * d, sizeof(double) * 27);
    }
    return obs_dim(o->kind);
}
int orc_prior_linearize(orc_problem* p, int i, double* err, double* Ji, double* Jj) {
    double e[12], a[144], b[144];
    prior_error(p, &p->pri[i], e);
    prior_jacobian(p, &p->pri[i], a, b);
    if (err) memcpy(err, e, sizeof(e));
    if (Ji) memcpy(Ji, a, sizeof(a));
    if (Jj) memcpy(Jj, b, sizeof(b));
    return 12;
}

/* ------------------------------------------------------------------ primitive exports */
void orc_se3_exp(const double xi[6], double q[4], double t[3]) {
    se3 T = se3_exp(xi);
    q[0] = T.q.x; q[1] = T.q.y; q[2] = T.q.z; q[3] = T.q.w;
    memcpy(t, T.t, sizeof(double) * 3);
}
void orc_se3_log(const double q[4], const double t[3], double xi[6]) {
    se3 T = mk_se3(q, t);
    se3_log(&T, xi);
}
void orc_so3_exp(const double w[3], double q[4]) {
    double th;
    quat r = so3_exp_theta(w, &th);
    q[0] = r.x; q[1] = r.y; q[2] = r.z; q[3] = r.w;
}
void orc_so3_log(const double q[4], double w[3]) {
    quat r = {q[0], q[1], q[2], q[3]};
    double th;
    so3_log_theta(&r, w, &th);
}
void orc_right_jac_pose3(const double xi[6], double J[36]) { right_jac_pose3(xi, J); }
void orc_right_jac_pose3_inv(const double xi[6], double J[36]) { right_jac_pose3_inv(xi, J); }
void orc_left_jac_pose3_q(const double xi[6], double Q[9]) { left_jac_pose3_q(xi, Q); }
void orc_gp_query_pose(const double qc[36], const double q1[4], const double t1[3], const double q2[4], const double t2[3],
                       const double v1[6], const double v2[6], double time1, double time2, double t,
                       double qo[4], double to[3], double At1[72], double Pt1[72], double dq[4], double dt[3], double xi12[6]) {
    gp_t gp;
    memcpy(gp.Qc, qc, sizeof(gp.Qc));
    lu_inverse(gp.QcInv, gp.Qc, 6);
    se3 P1 = mk_se3(q1, t1), P2 = mk_se3(q2, t2), dT;
    se3 T = gp_query_pose(&gp, &P1, &P2, v1, v2, time1, time2, t, At1, Pt1, &dT, xi12);
    qo[0] = T.q.x; qo[1] = T.q.y; qo[2] = T.q.z; qo[3] = T.q.w;
    memcpy(to, T.t, sizeof(double) * 3);
    dq[0] = dT.q.x; dq[1] = dT.q.y; dq[2] = dT.q.z; dq[3] = dT.q.w;
    memcpy(dt, dT.t, sizeof(double) * 3);
}

/* ------------------------------------------------------------------ tracking-side pose optimisation
 * Optimizer::PoseGPOptimizationFromeLastFrame (src/Optimizer.cc:369-686): two frame vertices
 * (prev: fixed = `fix`, cur), the map points constant (EdgeMonoGPOnlyPose / EdgeMonoOnlyPose /
 * EdgeStereoOnlyPose, src/G2oTypes.cc:162-223, include/G2oTypes.h:186-270: the reprojection edges of
 * this file with the point columns dropped), EdgeGaussianPrior(prev, cur), EdgeVelocity on both;
 * BlockSolverX + LinearSolverDense + Levenberg without a user lambda (:373-381).  Four rounds of
 * initializeOptimization(0) + optimize(10) with the re-classification of :575-672 in between.
 * Per-edge chi2 follows g2o: e->chi2() of an active edge is the error of the last computeActiveErrors
 * (the last trial state, even a rejected one); outliers get computeError() at the current state. */
typedef struct {
    orc_problem* p;
    const int* level;
    int robust;
    int fixprev;
    double* ob_chi2;
} trk_t;

static int trk_dof0(const trk_t* T) { return T->fixprev ? 12 : 0; }

static double trk_errors(trk_t* T) {   /* computeActiveErrors + activeRobustChi2 over level 0 */
    orc_problem* p = T->p;
    double chi = 0.0, rho[3];
    for (int k = 0; k < 2; ++k) {   /* EdgeVelocity (inactive on a fixed vertex) */
        if (p->kf[k].fixed) continue;
        double e = p->kf[k].vel[2];
        chi += e * (p->gp.QcInv[2 * 6 + 2] * e);
    }
    {
        double err[12];
        prior_error(p, &p->pri[0], err);
        chi += prior_chi2(p, &p->pri[0], err);
    }
    for (int i = 0; i < p->n_obs; ++i) {
        if (T->level[i]) continue;
        const lba_obs* o = &p->obs[i];
        double e[3];
        obs_error(p, o, e);
        double c = chi2_of(e, obs_dim(o->kind), o->w);
        T->ob_chi2[i] = c;
        if (T->robust) { huber(c, obs_delta(p, o->kind), rho); chi += rho[0]; }
        else chi += c;
    }
    return chi;
}

/* buildSystem over the level-0 edges: H [24 x 24], b [24] = -J^T rho' Omega e */
static void trk_build(trk_t* T, double* H, double* b) {
    orc_problem* p = T->p;
    memset(H, 0, sizeof(double) * 576);
    memset(b, 0, sizeof(double) * 24);
    double rho[3];
    for (int i = 0; i < p->n_obs; ++i) {
        if (T->level[i]) continue;
        const lba_obs* o = &p->obs[i];
        int dim = obs_dim(o->kind);
        double e[3], J[3 * JC];
        obs_error(p, o, e);
        obs_jacobian(p, o, J);
        double c = chi2_of(e, dim, o->w), s = o->w;
        if (T->robust) { huber(c, obs_delta(p, o->kind), rho); s *= rho[1]; }
        for (int r = 0; r < dim; ++r)
            for (int a = 0; a < 24; ++a) {
                double ja = J[r * JC + a];
                if (ja == 0.0) continue;
                b[a] -= ja * s * e[r];
                for (int c2 = 0; c2 < 24; ++c2) H[a * 24 + c2] += ja * s * J[r * JC + c2];
            }
    }
    {   /* EdgeGaussianPrior(prev, cur), info QiInv(dt) */
        double e[12], Ji[144], Jj[144], Jf[288], Om[144], OJ[288];
        prior_error(p, &p->pri[0], e);
        prior_jacobian(p, &p->pri[0], Ji, Jj);
        for (int r = 0; r < 12; ++r)
            for (int c = 0; c < 12; ++c) { Jf[r * 24 + c] = Ji[r * 12 + c]; Jf[r * 24 + 12 + c] = Jj[r * 12 + c]; }
        gp_qi_inv(&p->gp, p->kf[1].time - p->kf[0].time, Om);
        mat_mul(OJ, Om, Jf, 12, 12, 24);
        for (int a = 0; a < 24; ++a) {
            double s = 0.0;
            for (int r = 0; r < 12; ++r) {
                double oe = 0.0;
                for (int q = 0; q < 12; ++q) oe += Om[r * 12 + q] * e[q];
                s += Jf[r * 24 + a] * oe;
            }
            b[a] -= s;
            for (int c = 0; c < 24; ++c) {
                double h = 0.0;
                for (int r = 0; r < 12; ++r) h += Jf[r * 24 + a] * OJ[r * 24 + c];
                H[a * 24 + c] += h;
            }
        }
    }
    for (int k = 0; k < 2; ++k) {   /* EdgeVelocity: d e / d vel_z = 1 */
        if (p->kf[k].fixed) continue;
        double om = p->gp.QcInv[2 * 6 + 2];
        H[(12 * k + 8) * 24 + 12 * k + 8] += om;
        b[12 * k + 8] -= om * p->kf[k].vel[2];
    }
}

static int trk_lm_iteration(trk_t* T, int iteration, double* lambda, double* ni, int* nbad, int* trials) {
    orc_problem* p = T->p;
    const int d0 = trk_dof0(T), n = 24 - d0;
    double H[576], b[24], A[576], x[24];
    double currentChi = trk_errors(T), tempChi = currentChi, iniChi = currentChi;
    trk_build(T, H, b);
    if (iteration == 0) {   /* computeLambdaInit over the active vertices */
        double m = 0.0;
        for (int i = d0; i < 24; ++i) m = fmax(m, fabs(H[i * 24 + i]));
        *lambda = p->cfg.lambda_init > 0 ? p->cfg.lambda_init : p->cfg.tau * m;
        *ni = 2.0;
        *nbad = 0;
    }
    double rho = 0.0;
    int qmax = 0;
    kf_t bak[2];
    do {
        memcpy(bak, p->kf, sizeof(bak));
        for (int i = 0; i < n; ++i) {
            for (int j = 0; j < n; ++j) A[i * n + j] = H[(d0 + i) * 24 + d0 + j];
            A[i * n + i] += *lambda;
        }
        int ok2 = ldlt_solve_inplace(n, A, b + d0, x);
        if (ok2) {
            for (int k = T->fixprev ? 1 : 0; k < 2; ++k) {
                const double* dx = x + 12 * k - d0;
                se3 d = se3_exp(dx);
                p->kf[k].Twb = se3_mul(&p->kf[k].Twb, &d);
                for (int i = 0; i < 6; ++i) p->kf[k].vel[i] += dx[6 + i];
            }
        }
        tempChi = trk_errors(T);
        if (!ok2) tempChi = DBL_MAX;
        rho = currentChi - tempChi;
        double scale = 1e-3;
        if (ok2)
            for (int i = 0; i < n; ++i) scale += x[i] * (*lambda * x[i] + b[d0 + i]);
        rho /= scale;
        if (rho > 0 && isfinite(tempChi)) {
            double alpha = 1. - pow((2 * rho - 1), 3);
            alpha = fmin(alpha, 2. / 3.);
            *lambda *= fmax(1. / 3., alpha);
            *ni = 2;
            currentChi = tempChi;
        } else {
            *lambda *= *ni;
            *ni *= 2;
            memcpy(p->kf, bak, sizeof(bak));
        }
        qmax++;
    } while (rho < 0 && qmax < p->cfg.max_trials);
    *trials += qmax;
    if (qmax == p->cfg.max_trials || rho == 0) return LBA_RESULT_TERMINATE;
    if ((iniChi - currentChi) * 1e3 < iniChi) (*nbad)++;
    else *nbad = 0;
    if (*nbad >= 3) return LBA_RESULT_TERMINATE;
    return LBA_RESULT_OK;
}

static int trk_depth_ok(const orc_problem* p, int i) {   /* isDepthPositive (include/G2oTypes.h:203-206, 260-266) */
    const lba_obs* o = &p->obs[i];
    const cam_t* c = &p->cam[o->cam];
    int ks[2] = {o->kf_b, is_gp(o->kind) ? o->kf_a : -1};
    for (int s = 0; s < 2; ++s) {
        if (ks[s] < 0) continue;
        se3 Twc = se3_mul(&p->kf[ks[s]].Twb, &c->Tbc);
        se3 Tcw = se3_inv(&Twc);
        double Xc[3];
        se3_act(&Tcw, p->lm + 3 * o->lm, Xc);
        if (!(Xc[2] > 0)) return 0;
    }
    return 1;
}

int orc_track_pose(const lba_config* cfg, lba_track_frame* fr, lba_track_obs* tob, int n, const lba_cam* cams, int n_cam) {
    lba_kf kfs[2] = {fr->prev, fr->cur};
    kfs[1].fixed = 0;
    double* lm = (double*)malloc(sizeof(double) * 3 * (n > 0 ? n : 1));
    lba_obs* ob = (lba_obs*)calloc(n > 0 ? n : 1, sizeof(lba_obs));
    int* level = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
    double* chi2 = (double*)calloc(n > 0 ? n : 1, sizeof(double));
    for (int i = 0; i < n; ++i) {
        memcpy(lm + 3 * i, tob[i].Xw, sizeof(double) * 3);
        ob[i].kind = tob[i].kind;
        ob[i].kf_a = tob[i].kind == LBA_MONO_GP ? 0 : -1;
        ob[i].kf_b = 1;
        ob[i].lm = i;
        ob[i].cam = tob[i].cam;
        ob[i].t = tob[i].t;
        memcpy(ob[i].z, tob[i].z, sizeof(double) * 3);
        ob[i].w = tob[i].w;
        level[i] = tob[i].outlier ? 1 : 0;
    }
    lba_prior pri = {0, 1};
    int vel[2] = {0, 1};
    orc_problem* p = orc_create(cfg, kfs, 2, lm, n, ob, n, &pri, 1, vel, 2, cams, n_cam);
    trk_t T = {p, level, 1, fr->prev.fixed != 0, chi2};
    static const float chi2Mono[4] = {5.991f, 5.991f, 5.991f, 5.991f};
    static const float chi2Stereo[4] = {15.6f, 9.8f, 7.815f, 7.815f};
    int nBad = 0, iters = 0, trials = 0;
    for (int it = 0; it < 4; ++it) {
        double lambda = 0.0, ni = 2.0;
        int nbad_lm = 0;
        for (int k = 0; k < 10; ++k) {   /* optimize(its[it] = 10) */
            int r = trk_lm_iteration(&T, k, &lambda, &ni, &nbad_lm, &trials);
            ++iters;
            if (r != LBA_RESULT_OK && p->cfg.early_stop) break;
        }
        nBad = 0;
        const float chi2close = (float)(1.5 * chi2Mono[it]);
        for (int i = 0; i < n; ++i) {
            if (level[i]) {   /* e->computeError() at the current state */
                double e[3];
                obs_error(p, &p->obs[i], e);
                chi2[i] = chi2_of(e, obs_dim(p->obs[i].kind), p->obs[i].w);
            }
            const float c2 = (float)chi2[i];
            int out;
            if (tob[i].kind == LBA_STEREO) out = c2 > chi2Stereo[it];
            else {
                const int bclose = tob[i].close != 0;
                out = (c2 > chi2Mono[it] && !bclose) || (bclose && c2 > chi2close) || !trk_depth_ok(p, i);
            }
            level[i] = out;
            nBad += out;
        }
        if (it == 2) T.robust = 0;
        if (n + 3 < 10) break;   /* optimizer.edges().size() < 10 */
    }
    for (int i = 0; i < n; ++i) tob[i].outlier = level[i];
    const kf_t* c = &p->kf[1];
    fr->cur.q[0] = c->Twb.q.x; fr->cur.q[1] = c->Twb.q.y; fr->cur.q[2] = c->Twb.q.z; fr->cur.q[3] = c->Twb.q.w;
    memcpy(fr->cur.t, c->Twb.t, sizeof(double) * 3);
    memcpy(fr->cur.vel, c->vel, sizeof(double) * 6);
    fr->n_good = n - nBad;
    fr->iterations = iters;
    orc_destroy(p);
    free(lm); free(ob); free(level); free(chi2);
    return fr->n_good;
}
