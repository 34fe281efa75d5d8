// lba_math.hpp — fp64 Lie-group / GP / projection math for the MI355X local-BA kernels.
//
// Every function is LBA_HD (host+device) so the exact code the kernels run can also be
// checked on the CPU against the oracle (tests/test_math_host.py builds a host harness).
// Formulas follow the published algorithms the reference uses:
//   Sophus SO3/SE3 (Thirdparty/Sophus/sophus/so3.hpp:247-290,297-303,325-339,358-367,583-618;
//   se3.hpp:103-111,208-211,223-252,304-308,761-781; epsilon 1e-10 common.hpp:94),
//   Pose3utils (src/Pose3utils.cc:5-73,111-119), Pinhole (src/CameraModels/Pinhole.cpp:35-81).
// The GP interpolation uses the closed form of QueryPose's 12x12 products
// (src/GaussianProcess.cc:5-42): Pt1 = [l1 I, l2 I], At1 = [(1-l1) I, p2 I] with
// s = tau/T, l1 = 3s^2 - 2s^3, l2 = tau^2 (tau - T)/T^2, p2 = tau (1 - s)^2.
// Storage is row-major; tangent order is [translation; rotation].
#pragma once

#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define LBA_HD __host__ __device__ __forceinline__
#else
#define LBA_HD static inline
#endif

namespace lba {

constexpr double kEps = 1e-10;   // Sophus::Constants<double>::epsilon()

struct Quat { double x, y, z, w; };

// ---------------------------------------------------------------- small dense helpers
LBA_HD void hat3(const double* w, double* H) {
    H[0] = 0.0;   H[1] = -w[2]; H[2] = w[1];
    H[3] = w[2];  H[4] = 0.0;   H[5] = -w[0];
    H[6] = -w[1]; H[7] = w[0];  H[8] = 0.0;
}
LBA_HD void mul33(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            C[i * 3 + j] = A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j] + A[i * 3 + 2] * B[2 * 3 + j];
}
LBA_HD void mul33v(const double* A, const double* v, double* o) {
    o[0] = A[0] * v[0] + A[1] * v[1] + A[2] * v[2];
    o[1] = A[3] * v[0] + A[4] * v[1] + A[5] * v[2];
    o[2] = A[6] * v[0] + A[7] * v[1] + A[8] * v[2];
}
LBA_HD void mul33tv(const double* A, const double* v, double* o) {   // A^T v
    o[0] = A[0] * v[0] + A[3] * v[1] + A[6] * v[2];
    o[1] = A[1] * v[0] + A[4] * v[1] + A[7] * v[2];
    o[2] = A[2] * v[0] + A[5] * v[1] + A[8] * v[2];
}
// C[m x n] = A[m x k] * B[k x n]
LBA_HD void matmul(const double* A, const double* B, double* C, int m, int k, int n) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int l = 0; l < k; ++l) s += A[i * k + l] * B[l * n + j];
            C[i * n + j] = s;
        }
}

// ---------------------------------------------------------------- SO3 (unit quaternion)
LBA_HD Quat qnormalize(Quat q) {
    const double len = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    return Quat{q.x / len, q.y / len, q.z / len, q.w / len};
}
// Sophus SO3 product: Hamilton product, then normalisation by the SO3 constructor
LBA_HD Quat qmul(const Quat& a, const Quat& b) {
    Quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return qnormalize(r);
}
LBA_HD Quat qinv(const Quat& q) { return qnormalize(Quat{-q.x, -q.y, -q.z, q.w}); }
// rotate p by q (Sophus SO3::operator* on points)
LBA_HD void qrot(const Quat& q, const double* p, double* o) {
    double uv0 = q.y * p[2] - q.z * p[1], uv1 = q.z * p[0] - q.x * p[2], uv2 = q.x * p[1] - q.y * p[0];
    uv0 += uv0; uv1 += uv1; uv2 += uv2;
    o[0] = p[0] + q.w * uv0 + (q.y * uv2 - q.z * uv1);
    o[1] = p[1] + q.w * uv1 + (q.z * uv0 - q.x * uv2);
    o[2] = p[2] + q.w * uv2 + (q.x * uv1 - q.y * uv0);
}
// Eigen toRotationMatrix
LBA_HD void qmat(const Quat& q, double* R) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
// (sh / ch: sin and cos of the half angle theta / 2, when theta >= epsilon; one sincos for both, which
// se3_exp reuses for its V matrix)
LBA_HD Quat so3_exp(const double* w, double* theta_out, double* sh_out = nullptr, double* ch_out = nullptr) {
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double imag, real, th;
    if (th2 < kEps * kEps) {
        th = 0.0;
        const double th4 = th2 * th2;
        imag = 0.5 - (1.0 / 48.0) * th2 + (1.0 / 3840.0) * th4;
        real = 1.0 - (1.0 / 8.0) * th2 + (1.0 / 384.0) * th4;
    } else {
        th = sqrt(th2);
        const double h = 0.5 * th;
        double sh, ch;
        sincos(h, &sh, &ch);
        imag = sh / th;
        real = ch;
        if (sh_out) { *sh_out = sh; *ch_out = ch; }
    }
    *theta_out = th;
    return Quat{imag * w[0], imag * w[1], imag * w[2], real};
}
// (cot_half: cot(theta / 2) = w / |v| outside the small-angle branch: theta = 2 atan(|v| / w), so
// se3_log needs no sin / cos of the half angle)
LBA_HD void so3_log(const Quat& q, double* w, double* theta_out, double* cot_half = nullptr) {
    const double sn = q.x * q.x + q.y * q.y + q.z * q.z;
    double f;
    if (sn < kEps * kEps) {
        const double w2 = q.w * q.w;
        f = 2.0 / q.w - (2.0 / 3.0) * sn / (q.w * w2);
        *theta_out = 2.0 * sn / q.w;
    } else {
        const double n = sqrt(sn);
        if (fabs(q.w) < kEps)
            f = (q.w > 0 ? M_PI : -M_PI) / n;
        else
            f = 2.0 * atan(n / q.w) / n;
        *theta_out = f * n;
        if (cot_half) *cot_half = q.w / n;
    }
    w[0] = f * q.x; w[1] = f * q.y; w[2] = f * q.z;
}

// ---------------------------------------------------------------- SE3 = (q, t)
struct SE3 { Quat q; double t[3]; };

LBA_HD SE3 se3_mul(const SE3& a, const SE3& b) {
    SE3 r;
    r.q = qmul(a.q, b.q);
    double tb[3];
    qrot(a.q, b.t, tb);
    r.t[0] = a.t[0] + tb[0]; r.t[1] = a.t[1] + tb[1]; r.t[2] = a.t[2] + tb[2];
    return r;
}
LBA_HD SE3 se3_inv(const SE3& a) {
    SE3 r;
    r.q = qinv(a.q);
    const double mt[3] = {-a.t[0], -a.t[1], -a.t[2]};
    qrot(r.q, mt, r.t);
    return r;
}
LBA_HD SE3 se3_exp(const double* a) {
    SE3 r;
    double th, sh = 0.0, ch = 1.0;
    r.q = so3_exp(a + 3, &th, &sh, &ch);
    double Om[9], Om2[9], V[9];
    hat3(a + 3, Om);
    mul33(Om, Om, Om2);
    if (th < kEps) {
        qmat(r.q, V);
    } else {
        // 1 - cos(th) = 2 sin^2(th / 2), sin(th) = 2 sin(th / 2) cos(th / 2): the half-angle pair of
        // so3_exp (Sophus evaluates cos(th) and sin(th) again; equal up to rounding)
        const double th2 = th * th;
        const double c1 = 2.0 * sh * sh / th2, c2 = (th - 2.0 * sh * ch) / (th2 * th);
        for (int i = 0; i < 9; ++i) V[i] = ((i & 3) == 0 ? 1.0 : 0.0) + c1 * Om[i] + c2 * Om2[i];
    }
    mul33v(V, a, r.t);
    return r;
}
LBA_HD void se3_log(const SE3& T, double* xi) {
    double th, w[3], cot_h = 0.0;
    so3_log(T.q, w, &th, &cot_h);
    xi[3] = w[0]; xi[4] = w[1]; xi[5] = w[2];
    double Om[9], Om2[9], Vi[9];
    hat3(w, Om);
    mul33(Om, Om, Om2);
    double c;
    if (fabs(th) < kEps) {
        c = 1.0 / 12.0;
    } else {
        c = (1.0 - 0.5 * th * cot_h) / (th * th);   // (1 - th cos(h) / (2 sin(h))) / th^2, h = th / 2
    }
    for (int i = 0; i < 9; ++i) Vi[i] = ((i & 3) == 0 ? 1.0 : 0.0) - 0.5 * Om[i] + c * Om2[i];
    mul33v(Vi, T.t, xi);
}
// Ad(T) = [R, t^R; 0, R] (6x6)
LBA_HD void se3_adj(const SE3& T, double* A) {
    double R[9], H[9], tR[9];
    qmat(T.q, R);
    hat3(T.t, H);
    mul33(H, R, tR);
    for (int i = 0; i < 36; ++i) A[i] = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            A[i * 6 + j] = R[i * 3 + j];
            A[(3 + i) * 6 + 3 + j] = R[i * 3 + j];
            A[i * 6 + 3 + j] = tR[i * 3 + j];
        }
}

// ---------------------------------------------------------------- Pose3utils
// The Pose3utils Jacobians below take sin / cos of the rotation angle th = |w| (and cot(th / 2)) from ONE
// sincos of the half angle: sin(th) = 2 sh ch, cos(th) = 1 - 2 sh^2, cot(th / 2) = ch / sh (the reference
// evaluates sin, cos and tan separately; the values agree up to rounding).
struct AngleSC { double th2, th, s, c, sh, ch; };
LBA_HD AngleSC angle_sc(const double* w) {
    AngleSC a;
    a.th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    a.th = sqrt(a.th2);
    sincos(0.5 * a.th, &a.sh, &a.ch);
    a.s = 2.0 * a.sh * a.ch;
    a.c = 1.0 - 2.0 * a.sh * a.sh;
    return a;
}
// LeftJacobianPose3Q (src/Pose3utils.cc:5-24), including the reference's small-angle branch
LBA_HD void left_jac_q(const double* xi, const AngleSC& g, double* Q) {
    const double* om = xi + 3;
    const double th = g.th;
    double X[9], Y[9], XY[9], YX[9], XYX[9], T1[9], T2[9], T3[9], T4[9];
    hat3(om, X);
    hat3(xi, Y);
    mul33(X, Y, XY);
    mul33(Y, X, YX);
    mul33(X, YX, XYX);
    double a, b, c;
    if (fabs(th) > 1e-5) {
        const double s = g.s, co = g.c;
        const double t2 = th * th, t3 = t2 * th, t4 = t3 * th, t5 = t4 * th;
        a = (th - s) / t3;
        b = (1.0 - 0.5 * t2 - co) / t4;
        c = 0.5 * ((1.0 - 0.5 * t2 - co) / t4 - 3.0 * (th - s - t3 / 6.0) / t5);
    } else {
        a = 1.0 / 6.0;
        b = 1.0 / 24.0;
        c = 0.5 * (1.0 / 24.0 + 3.0 / 120.0);
    }
    mul33(X, XY, T1);    // X*XY
    mul33(YX, X, T2);    // YX*X
    mul33(XYX, X, T3);   // XYX*X
    mul33(X, XYX, T4);   // X*XYX
    for (int i = 0; i < 9; ++i)
        Q[i] = 0.5 * Y[i] + a * (XY[i] + YX[i] + XYX[i]) - b * (T1[i] + T2[i] - 3.0 * XYX[i]) - c * (T3[i] + T4[i]);
}
// LeftJacobianRot3 (:48-59)
LBA_HD void left_jac_rot3(const double* w, const AngleSC& g, double* J) {
    const double th2 = g.th2;
    if (th2 <= 2.220446049250313e-16) {
        for (int i = 0; i < 9; ++i) J[i] = ((i & 3) == 0) ? 1.0 : 0.0;
        return;
    }
    const double th = g.th;
    const double d[3] = {w[0] / th, w[1] / th, w[2] / th};
    const double s = g.s;
    const double c1 = s / th, c2 = 1.0 - s / th, c3 = (2.0 * g.sh * g.sh) / th;   // (1 - cos th) / th
    double A[9];
    hat3(w, A);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            J[i * 3 + j] = (i == j ? c1 : 0.0) + c2 * d[i] * d[j] + c3 * (A[i * 3 + j] / th);
}
// LeftJacobianRot3Inv (:61-73)
LBA_HD void left_jac_rot3_inv(const double* w, const AngleSC& g, double* J) {
    const double th2 = g.th2;
    if (th2 <= 2.220446049250313e-16) {
        for (int i = 0; i < 9; ++i) J[i] = ((i & 3) == 0) ? 1.0 : 0.0;
        return;
    }
    const double th = g.th;
    const double d[3] = {w[0] / th, w[1] / th, w[2] / th};
    const double h = th / 2.0, hc = h * (g.ch / g.sh);   // h / tan(h)
    double A[9];
    hat3(w, A);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            J[i * 3 + j] = (i == j ? hc : 0.0) + (1.0 - hc) * d[i] * d[j] - h * (A[i * 3 + j] / th);
}
// Right Jacobian of SE(3) as blocks: Jr(xi) = LeftJacobianPose3(-xi) = [J, Q; 0, J]
LBA_HD void right_jac_blocks(const double* xi, double* J, double* Q) {
    const double m[6] = {-xi[0], -xi[1], -xi[2], -xi[3], -xi[4], -xi[5]};
    const AngleSC g = angle_sc(m + 3);
    left_jac_q(m, g, Q);
    left_jac_rot3(m + 3, g, J);
}
// Inverse right Jacobian: Jr^-1(xi) = LeftJacobianPose3Inv(-xi) = [Ji, -Ji Q Ji; 0, Ji] (6x6)
LBA_HD void right_jac_inv(const double* xi, double* Jr) {
    const double m[6] = {-xi[0], -xi[1], -xi[2], -xi[3], -xi[4], -xi[5]};
    double Q[9], Ji[9], T[9], U[9];
    const AngleSC g = angle_sc(m + 3);
    left_jac_q(m, g, Q);
    left_jac_rot3_inv(m + 3, g, Ji);
    mul33(Ji, Q, T);
    mul33(T, Ji, U);
    for (int i = 0; i < 36; ++i) Jr[i] = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            Jr[i * 6 + j] = Ji[i * 3 + j];
            Jr[(3 + i) * 6 + 3 + j] = Ji[i * 3 + j];
            Jr[i * 6 + 3 + j] = -U[i * 3 + j];
        }
}
// se3Adj(v) = [w^, v^; 0, w^] (:111-119)
LBA_HD void se3_ad(const double* v, double* A) {
    double Hw[9], Hv[9];
    hat3(v + 3, Hw);
    hat3(v, Hv);
    for (int i = 0; i < 36; ++i) A[i] = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            A[i * 6 + j] = Hw[i * 3 + j];
            A[(3 + i) * 6 + 3 + j] = Hw[i * 3 + j];
            A[i * 6 + 3 + j] = Hv[i * 3 + j];
        }
}

// ---------------------------------------------------------------- GP closed form
struct GPScalars { double l1, l2, p2; };
LBA_HD GPScalars gp_scalars(double t1, double t2, double t) {
    const double T = t2 - t1, tau = t - t1, s = tau / T, om = 1.0 - s;
    GPScalars g;
    g.l1 = s * s * (3.0 - 2.0 * s);
    g.l2 = tau * tau * (tau - T) / (T * T);
    g.p2 = tau * om * om;
    return g;
}

// Per GP KF-pair quantities (depend on the two KF states only), staged once per pair.
struct GPPair {
    double T1q[4], T1t[3];   // Twb of KF_a
    double v1[6];            // velocity of KF_a
    double xi12[6];          // log(T1^-1 T2)
    double w2[6];            // Jr^-1(xi12) v2
    double G1a[36];          // A1 = -Jr^-1(xi12) Ad(exp(xi12))^-1
    double G1b[36];          // B1 = -1/2 ad(v2) A1
    double G2a[36];          // C  = Jr^-1(xi12)
    double G2b[36];          // D  = -1/2 ad(v2) C
    double t1, t2;
};

// full = false: only what the interpolated pose needs (T1, v1, xi12, w2; residual evaluation)
LBA_HD void gp_pair_build(const SE3& Ta, const double* va, const SE3& Tb, const double* vb, double ta, double tb,
                          GPPair* P, bool full = true) {
    P->T1q[0] = Ta.q.x; P->T1q[1] = Ta.q.y; P->T1q[2] = Ta.q.z; P->T1q[3] = Ta.q.w;
    for (int i = 0; i < 3; ++i) P->T1t[i] = Ta.t[i];
    for (int i = 0; i < 6; ++i) P->v1[i] = va[i];
    const SE3 Tai = se3_inv(Ta);
    const SE3 T12 = se3_mul(Tai, Tb);
    se3_log(T12, P->xi12);
    right_jac_inv(P->xi12, P->G2a);
    matmul(P->G2a, vb, P->w2, 6, 6, 1);
    P->t1 = ta;
    P->t2 = tb;
    if (!full) return;
    // Ad(exp(xi12))^-1 = Ad(exp(xi12)^-1) = Ad(T12^-1): exp(log(T12)) is T12 up to rounding, so the
    // reference's exp + general 6x6 inverse (src/G2oTypes.cc:292) is the adjoint of the inverse pair pose
    double AdI[36], ad2[36];
    se3_adj(se3_inv(T12), AdI);
    matmul(P->G2a, AdI, P->G1a, 6, 6, 6);
    for (int i = 0; i < 36; ++i) P->G1a[i] = -P->G1a[i];
    se3_ad(vb, ad2);
    matmul(ad2, P->G1a, P->G1b, 6, 6, 6);
    matmul(ad2, P->G2a, P->G2b, 6, 6, 6);
    for (int i = 0; i < 36; ++i) { P->G1b[i] *= -0.5; P->G2b[i] *= -0.5; }
}

// ---------------------------------------------------------------- observation model
struct Cam { double q[4], t[3], fx, fy, cx, cy; };

// Derived camera quantities: Tcb = Tbc^-1 as rotation matrix + translation
struct CamD { double Rcb[9], tcb[3], fx, fy, cx, cy; };

LBA_HD void cam_derive(const Cam& c, CamD* d) {
    SE3 Tbc;
    Tbc.q = Quat{c.q[0], c.q[1], c.q[2], c.q[3]};
    Tbc.t[0] = c.t[0]; Tbc.t[1] = c.t[1]; Tbc.t[2] = c.t[2];
    const SE3 Tcb = se3_inv(Tbc);
    qmat(Tcb.q, d->Rcb);
    d->tcb[0] = Tcb.t[0]; d->tcb[1] = Tcb.t[1]; d->tcb[2] = Tcb.t[2];
    d->fx = c.fx; d->fy = c.fy; d->cx = c.cx; d->cy = c.cy;
}

// Camera record of a state (CAMD_STRIDE doubles): Rcb(9) tcb(3) fx fy cx cy, then the Jacobian factor of
// the camera's extrinsic vertex stored like a sample's N (column c at 16 + 6 c, 12 columns, the last six
// zero: the extrinsic occupies a 12-wide pose block whose second half is inert).  EdgeMonoGPExtrinsic's
// _jacobianOplus[3] = -P [-I, Xc^] (src/G2oTypes.cc:311-313) equals J1 Ad(Tbc) with J1 = P Rcb [I, -Xb^]
// the Jacobian w.r.t. the body pose sample: Rcb (tbc - Xb) = -Xc, so P Rcb [Rbc, (tbc - Xb)^ Rbc] = P [I, -Xc^].
constexpr int CAMREC_DOUBLES = 16 + 72;
LBA_HD void cam_record(const SE3& Tbc, double fx, double fy, double cx, double cy, double* o) {
    const SE3 Tcb = se3_inv(Tbc);
    qmat(Tcb.q, o);
    o[9] = Tcb.t[0]; o[10] = Tcb.t[1]; o[11] = Tcb.t[2];
    o[12] = fx; o[13] = fy; o[14] = cx; o[15] = cy;
    double A[36];
    se3_adj(Tbc, A);
    for (int c = 0; c < 12; ++c)
        for (int l = 0; l < 6; ++l) o[16 + 6 * c + l] = c < 6 ? A[l * 6 + c] : 0.0;
}

// EdgeExtrinsicPrior (include/G2oTypes.h:470-494): e = log(R_ Rbc) with R_ = Rbc_ini^-1 (qinv_ini, already
// inverted and normalised as the edge's constructor does), Jacobian w.r.t. the rotation half of the
// extrinsic's tangent: RightJacobianSO3(e)^-1 (src/G2oTypes.cc:575-591, Eigen 3x3 inverse); the
// translation half is zero.
LBA_HD void inv3(const double* m, double* r);
LBA_HD void ext_prior_error_jac(const Quat& qbc, const Quat& qinv_ini, double* e, double* Jrot) {
    double th;
    so3_log(qmul(qinv_ini, qbc), e, &th);
    if (!Jrot) return;
    const double x = e[0], y = e[1], z = e[2];
    const double d2 = x * x + y * y + z * z, d = sqrt(d2);
    double Jr[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (!(d < 1e-5)) {
        const double W[9] = {0.0, -z, y, z, 0.0, -x, -y, x, 0.0};
        double WW[9];
        mul33(W, W, WW);
        const double a = 1.0 - cos(d), b = d - sin(d), d3 = d2 * d;
        for (int i = 0; i < 9; ++i) Jr[i] = Jr[i] - W[i] * a / d2 + WW[i] * b / d3;
    }
    inv3(Jr, Jrot);
}

// GP pose sample: everything an observation at time t between (KF_a, KF_b) needs.  All observations
// of one camera of one keyframe share t, so a window has O(pairs x cameras) samples for O(obs) GP
// observations and the interpolation + Jacobian chain is evaluated once per sample.
//   T(t) = T1 exp(xi),  xi = p2 v1 + l1 xi12 + l2 Jr^-1(xi12) v2        (QueryPose, GaussianProcess.cc:23-42)
// The reference chain (src/G2oTypes.cc:258-314) J_a = [K (l1 A1 + l2 B1) + J1 Ad(exp(-xi)), p2 K],
// J_b = [K (l1 C + l2 D), l2 K C] with K = J1 Jr(xi) is refactored as J = J1 N with the 6x24 matrix
//   N = [Jr (l1 A1 + l2 B1) + Ad(exp(-xi)) | p2 Jr | Jr (l1 C + l2 D) | l2 Jr C].
constexpr int GPS_N = 6 * 24;
struct GPSample {
    double Rwb[9], twb[3];
    double N[GPS_N];   // stored transposed: N[c * 6 + l] = N(l, c), so one column is 48 contiguous bytes
};

// (dT_out: exp(xi), whose inverse gives the Ad(exp(-xi)) block of N)
LBA_HD void gp_sample_pose(const GPPair& P, double t, double* Rwb, double* twb, double* xi, GPScalars* g,
                           SE3* dT_out = nullptr) {
    *g = gp_scalars(P.t1, P.t2, t);
    for (int i = 0; i < 6; ++i) xi[i] = g->p2 * P.v1[i] + g->l1 * P.xi12[i] + g->l2 * P.w2[i];
    const SE3 dT = se3_exp(xi);
    if (dT_out) *dT_out = dT;
    SE3 T1;
    T1.q = Quat{P.T1q[0], P.T1q[1], P.T1q[2], P.T1q[3]};
    T1.t[0] = P.T1t[0]; T1.t[1] = P.T1t[1]; T1.t[2] = P.T1t[2];
    const SE3 T = se3_mul(T1, dT);
    qmat(T.q, Rwb);
    twb[0] = T.t[0]; twb[1] = T.t[1]; twb[2] = T.t[2];
}

LBA_HD void gp_sample_build(const GPPair& P, double t, GPSample* S) {
    double xi[6];
    GPScalars g;
    SE3 E;
    gp_sample_pose(P, t, S->Rwb, S->twb, xi, &g, &E);
    // Jr(xi) = [Jl, Q; 0, Jl] with Jl = LeftJacobianRot3(-w), Q = LeftJacobianPose3Q(-xi)
    double Jl[9], Q[9];
    right_jac_blocks(xi, Jl, Q);
    double Jr[36];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            Jr[i * 6 + j] = Jl[i * 3 + j];
            Jr[i * 6 + 3 + j] = Q[i * 3 + j];
            Jr[(3 + i) * 6 + j] = 0.0;
            Jr[(3 + i) * 6 + 3 + j] = Jl[i * 3 + j];
        }
    // Ad(exp(-xi)) = Ad(exp(xi)^-1) = [R', t'^ R'; 0, R']
    const SE3 Em = se3_inv(E);
    double Rm[9], Ht[9], tR[9];
    qmat(Em.q, Rm);
    hat3(Em.t, Ht);
    mul33(Ht, Rm, tR);
    double MA[36], MC[36];
    for (int i = 0; i < 36; ++i) {
        MA[i] = g.l1 * P.G1a[i] + g.l2 * P.G1b[i];
        MC[i] = g.l1 * P.G2a[i] + g.l2 * P.G2b[i];
    }
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c) {
            double na = 0.0, nb = 0.0, nc = 0.0;
            for (int l = 0; l < 6; ++l) {
                na += Jr[r * 6 + l] * MA[l * 6 + c];
                nb += Jr[r * 6 + l] * MC[l * 6 + c];
                nc += Jr[r * 6 + l] * P.G2a[l * 6 + c];
            }
            double ad = 0.0;
            if (r < 3) ad = (c < 3) ? Rm[r * 3 + c] : tR[r * 3 + c - 3];
            else if (c >= 3) ad = Rm[(r - 3) * 3 + c - 3];
            S->N[c * 6 + r] = na + ad;
            S->N[(6 + c) * 6 + r] = g.p2 * Jr[r * 6 + c];
            S->N[(12 + c) * 6 + r] = nb;
            S->N[(18 + c) * 6 + r] = g.l2 * nc;
        }
}

// Xb = Rwb^T (Xw - twb), Xc = Rcb Xb + tcb; residual e = z - pi(Xc) (3rd row u - bf/z)
template <int DIM>
LBA_HD void project_residual(const double* Rwb, const double* twb, const CamD& c, const double* Xw, const double* z,
                             double bf, double* Xb, double* Xc, double* e) {
    const double d[3] = {Xw[0] - twb[0], Xw[1] - twb[1], Xw[2] - twb[2]};
    mul33tv(Rwb, d, Xb);
    mul33v(c.Rcb, Xb, Xc);
    Xc[0] += c.tcb[0]; Xc[1] += c.tcb[1]; Xc[2] += c.tcb[2];
    const double u = c.fx * Xc[0] / Xc[2] + c.cx;
    const double v = c.fy * Xc[1] / Xc[2] + c.cy;
    e[0] = z[0] - u;
    e[1] = z[1] - v;
    if (DIM == 3) e[2] = z[2] - (u - bf * (1.0 / Xc[2]));
}

// Jacobian rows of one reprojection observation (DIM = 2 mono, 3 stereo) w.r.t. the body pose at
// the observation time and the point:
//   J1 = P Rcb [I, -Xb^] (DIM x 6, row-major), J_pt = -P Rcb Rwb^T (DIM x 3)
// (src/G2oTypes.cc:445-495; the GP edges chain J1 with their sample's factor N, see obs_jacobian).
template <int DIM>
LBA_HD void obs_j1(const double* Rwb, const CamD& c, const double* Xb, const double* Xc, double bf, double* J1,
                   double* Jp) {
    // projection Jacobian P (DIM x 3)
    const double iz = 1.0 / Xc[2];
    double Pj[9];
    Pj[0] = c.fx * iz; Pj[1] = 0.0; Pj[2] = -c.fx * Xc[0] / (Xc[2] * Xc[2]);
    Pj[3] = 0.0; Pj[4] = c.fy * iz; Pj[5] = -c.fy * Xc[1] / (Xc[2] * Xc[2]);
    if (DIM == 3) { Pj[6] = Pj[0]; Pj[7] = Pj[1]; Pj[8] = Pj[2] + bf * (1.0 / (Xc[2] * Xc[2])); }
    // M = P Rcb (DIM x 3);  J1 = [M, -M Xb^] ;  Jpt = -M Rwb^T
    double M[3 * DIM], H[9];
    for (int r = 0; r < DIM; ++r)
        for (int j = 0; j < 3; ++j)
            M[r * 3 + j] = Pj[r * 3 + 0] * c.Rcb[0 * 3 + j] + Pj[r * 3 + 1] * c.Rcb[1 * 3 + j] + Pj[r * 3 + 2] * c.Rcb[2 * 3 + j];
    hat3(Xb, H);
    for (int r = 0; r < DIM; ++r)
        for (int j = 0; j < 3; ++j) {
            J1[r * 6 + j] = M[r * 3 + j];
            J1[r * 6 + 3 + j] = -(M[r * 3 + 0] * H[0 * 3 + j] + M[r * 3 + 1] * H[1 * 3 + j] + M[r * 3 + 2] * H[2 * 3 + j]);
        }
    for (int r = 0; r < DIM; ++r)
        for (int j = 0; j < 3; ++j)   // -M Rwb^T : (M Rbw)_{rj} = sum_k M_rk Rwb_jk
            Jp[r * 3 + j] = -(M[r * 3 + 0] * Rwb[j * 3 + 0] + M[r * 3 + 1] * Rwb[j * 3 + 1] + M[r * 3 + 2] * Rwb[j * 3 + 2]);
}

// fp32-residual option (LBA_FLAG_F32_RESIDUAL, BASELINE configs[4]: "fp32 residuals + fp64 accumulate"): the
// same two functions with the projection, the residual and the Jacobian rows in fp32.  The world offset Xw - twb
// stays fp64 (a trajectory kilometres long would otherwise lose millimetres to fp32 rounding before the
// rotation); the results are widened to fp64 for the robust weight and every sum of J^T W J / J^T W e.
template <int DIM>
LBA_HD void project_residual_f32(const double* Rwb, const double* twb, const CamD& c, const double* Xw, const double* z,
                                 double bf, double* Xb, double* Xc, double* e) {
    const float d0 = (float)(Xw[0] - twb[0]), d1 = (float)(Xw[1] - twb[1]), d2 = (float)(Xw[2] - twb[2]);
    float xb[3], xc[3];
    for (int j = 0; j < 3; ++j) xb[j] = (float)Rwb[j] * d0 + (float)Rwb[3 + j] * d1 + (float)Rwb[6 + j] * d2;
    for (int i = 0; i < 3; ++i)
        xc[i] = (float)c.Rcb[i * 3] * xb[0] + (float)c.Rcb[i * 3 + 1] * xb[1] + (float)c.Rcb[i * 3 + 2] * xb[2] +
                (float)c.tcb[i];
    const float u = (float)c.fx * xc[0] / xc[2] + (float)c.cx;
    const float v = (float)c.fy * xc[1] / xc[2] + (float)c.cy;
    e[0] = (double)((float)z[0] - u);
    e[1] = (double)((float)z[1] - v);
    if (DIM == 3) e[2] = (double)((float)z[2] - (u - (float)bf * (1.0f / xc[2])));
    for (int k = 0; k < 3; ++k) {
        Xb[k] = (double)xb[k];
        Xc[k] = (double)xc[k];
    }
}
template <int DIM>
LBA_HD void obs_j1_f32(const double* Rwb, const CamD& c, const double* Xb, const double* Xc, double bf, double* J1,
                       double* Jp) {
    const float x0 = (float)Xc[0], x1 = (float)Xc[1], x2 = (float)Xc[2];
    const float iz = 1.0f / x2, fx = (float)c.fx, fy = (float)c.fy;
    float Pj[9];
    Pj[0] = fx * iz; Pj[1] = 0.0f; Pj[2] = -fx * x0 / (x2 * x2);
    Pj[3] = 0.0f; Pj[4] = fy * iz; Pj[5] = -fy * x1 / (x2 * x2);
    if (DIM == 3) { Pj[6] = Pj[0]; Pj[7] = Pj[1]; Pj[8] = Pj[2] + (float)bf * (1.0f / (x2 * x2)); }
    float M[3 * DIM];
    for (int r = 0; r < DIM; ++r)
        for (int j = 0; j < 3; ++j)
            M[r * 3 + j] = Pj[r * 3] * (float)c.Rcb[j] + Pj[r * 3 + 1] * (float)c.Rcb[3 + j] + Pj[r * 3 + 2] * (float)c.Rcb[6 + j];
    const float b0 = (float)Xb[0], b1 = (float)Xb[1], b2 = (float)Xb[2];
    const float H[9] = {0.0f, -b2, b1, b2, 0.0f, -b0, -b1, b0, 0.0f};
    for (int r = 0; r < DIM; ++r)
        for (int j = 0; j < 3; ++j) {
            J1[r * 6 + j] = (double)M[r * 3 + j];
            J1[r * 6 + 3 + j] = (double)(-(M[r * 3] * H[j] + M[r * 3 + 1] * H[3 + j] + M[r * 3 + 2] * H[6 + j]));
            Jp[r * 3 + j] = (double)(-(M[r * 3] * (float)Rwb[j * 3] + M[r * 3 + 1] * (float)Rwb[j * 3 + 1] +
                                      M[r * 3 + 2] * (float)Rwb[j * 3 + 2]));
        }
}
// the projection of the requested precision (F32: the fp32-residual option)
template <int DIM, bool F32>
LBA_HD void project_residual_p(const double* Rwb, const double* twb, const CamD& c, const double* Xw, const double* z,
                               double bf, double* Xb, double* Xc, double* e) {
    if constexpr (F32) project_residual_f32<DIM>(Rwb, twb, c, Xw, z, bf, Xb, Xc, e);
    else project_residual<DIM>(Rwb, twb, c, Xw, z, bf, Xb, Xc, e);
}
template <int DIM, bool F32>
LBA_HD void obs_j1_p(const double* Rwb, const CamD& c, const double* Xb, const double* Xc, double bf, double* J1,
                     double* Jp) {
    if constexpr (F32) obs_j1_f32<DIM>(Rwb, c, Xb, Xc, bf, J1, Jp);
    else obs_j1<DIM>(Rwb, c, Xb, Xc, bf, J1, Jp);
}

// Full Jacobian rows, columns [KF_a pose(6) vel(6) | KF_b pose(6) vel(6) | point(3)] (27):
//   GP edges: pose/vel columns = J1 N (N of the observation's GP sample, stored transposed);
//   EdgeMono/EdgeStereo: KF_b pose columns = J1, velocity columns 0.
// Output row r: pose/vel columns 0..23 at J[r*ldJ + c], point columns at J[r*ldJ + pcol + j]
// (host harness: ldJ 27, pcol 24).  The kernels keep J1 and reduce in the sample's space instead.
template <int DIM, typename OutT, typename NT, bool F32 = false>
LBA_HD void obs_jacobian(const double* Rwb, const CamD& c, const double* Xb, const double* Xc, double bf,
                         const NT* N, OutT* J, int ldJ, int pcol) {
    double J1[6 * DIM], Jp[3 * DIM];
    obs_j1_p<DIM, F32>(Rwb, c, Xb, Xc, bf, J1, Jp);
    for (int r = 0; r < DIM; ++r)
        for (int j = 0; j < 3; ++j) J[r * ldJ + pcol + j] = Jp[r * 3 + j];
    if (!N) {
        for (int r = 0; r < DIM; ++r) {
            for (int j = 0; j < 12; ++j) J[r * ldJ + j] = 0.0;
            for (int j = 0; j < 6; ++j) { J[r * ldJ + 12 + j] = J1[r * 6 + j]; J[r * ldJ + 18 + j] = 0.0; }
        }
        return;
    }
    for (int cc = 0; cc < 24; ++cc) {
        double n[6];
        for (int l = 0; l < 6; ++l) n[l] = N[cc * 6 + l];
        for (int r = 0; r < DIM; ++r) {
            const double* a = J1 + r * 6;
            J[r * ldJ + cc] = a[0] * n[0] + a[1] * n[1] + a[2] * n[2] + a[3] * n[3] + a[4] * n[4] + a[5] * n[5];
        }
    }
}

// Eigen compute_inverse<3,3>: adjugate / determinant (used by the Schur step,
// Thirdparty/g2o/g2o/core/block_solver.hpp:389)
LBA_HD void inv3(const double* m, double* r) {
    const double c00 = m[4] * m[8] - m[5] * m[7];
    const double c10 = m[7] * m[2] - m[8] * m[1];
    const double c20 = m[1] * m[5] - m[2] * m[4];
    const double invdet = 1.0 / (c00 * m[0] + c10 * m[3] + c20 * m[6]);
    r[0] = c00 * invdet; r[1] = c10 * invdet; r[2] = c20 * invdet;
    r[3] = (m[5] * m[6] - m[3] * m[8]) * invdet;
    r[4] = (m[8] * m[0] - m[6] * m[2]) * invdet;
    r[5] = (m[2] * m[3] - m[0] * m[5]) * invdet;
    r[6] = (m[3] * m[7] - m[4] * m[6]) * invdet;
    r[7] = (m[6] * m[1] - m[7] * m[0]) * invdet;
    r[8] = (m[0] * m[4] - m[1] * m[3]) * invdet;
}

// GaussianProcess::QiInv(dt) (include/GaussianProcess.h:31-41), 12x12 row-major
LBA_HD void qi_inv(const double* qcinv, double dt, double* Om) {
    const double dt2 = dt * dt, dt3 = dt2 * dt;
    const double a = 12.0 / dt3, b = -6.0 / dt2, c = 4.0 / dt;
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            const double q = qcinv[i * 6 + j];
            Om[i * 12 + j] = a * q;
            Om[i * 12 + 6 + j] = b * q;
            Om[(6 + i) * 12 + j] = b * q;
            Om[(6 + i) * 12 + 6 + j] = c * q;
        }
}

// EdgeGaussianPrior (include/G2oTypes.h:155-163, src/G2oTypes.cc:100-118):
//   e = [xi - dt v1 ; Jr^-1(xi) v2 - v1], xi = log(T1^-1 T2)
//   Ji = [-Jr^-1 Ad(T)^-1, -dt I ; -1/2 ad(v2)(-Jr^-1 Ad(T)^-1), -I],  Jj = [Jr^-1, 0 ; -1/2 ad(v2) Jr^-1, Jr^-1]
// Ji / Jj may be null (error only).
template <typename OutT>
LBA_HD void prior_error_jac(const SE3& Ta, const double* va, double ta, const SE3& Tb, const double* vb, double tb,
                            OutT* e, OutT* Ji, OutT* Jj) {
    const SE3 T = se3_mul(se3_inv(Ta), Tb);
    double xi[6], Jri[36];
    se3_log(T, xi);
    right_jac_inv(xi, Jri);
    const double dt = tb - ta;
    for (int i = 0; i < 6; ++i) {
        double s = 0.0;
        for (int k = 0; k < 6; ++k) s += Jri[i * 6 + k] * vb[k];
        e[i] = xi[i] - dt * va[i];
        e[6 + i] = s - va[i];
    }
    if (!Ji) return;
    double AdI[36], ad2[36], top[36];
    se3_adj(se3_inv(T), AdI);
    se3_ad(vb, ad2);
    matmul(Jri, AdI, top, 6, 6, 6);
    for (int i = 0; i < 144; ++i) { Ji[i] = 0.0; Jj[i] = 0.0; }
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double bi = 0.0, bj = 0.0;
            for (int k = 0; k < 6; ++k) { bi += ad2[i * 6 + k] * (-top[k * 6 + j]); bj += ad2[i * 6 + k] * Jri[k * 6 + j]; }
            Ji[i * 12 + j] = -top[i * 6 + j];
            Ji[(6 + i) * 12 + j] = -0.5 * bi;
            Jj[i * 12 + j] = Jri[i * 6 + j];
            Jj[(6 + i) * 12 + j] = -0.5 * bj;
            Jj[(6 + i) * 12 + 6 + j] = Jri[i * 6 + j];
        }
    for (int i = 0; i < 6; ++i) { Ji[i * 12 + 6 + i] = -dt; Ji[(6 + i) * 12 + 6 + i] = -1.0; }
}

// Huber (RobustKernelHuber::robustify, robust_kernel_impl.cpp:76-90): rho(e), rho'(e)
LBA_HD void huber(double e, double delta, double* r0, double* r1) {
    const double d2 = delta * delta;
    if (e <= d2) { *r0 = e; *r1 = 1.0; }
    else { const double s = sqrt(e); *r0 = 2 * s * delta - d2; *r1 = delta / s; }
}

}  // namespace lba
