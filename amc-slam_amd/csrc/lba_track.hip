// lba_track.hip — tracking-side pose optimisation on the GPU: Optimizer::PoseGPOptimizationFromeLastFrame
// (src/Optimizer.cc:369-686), SURVEY.md §8(f)3.
//
// The problem is tiny (two 12-dof frame vertices, the map points fixed, a few hundred to a few thousand
// reprojection edges) and latency-bound, so the whole call — four rounds of optimize(10) with the
// outlier re-classification between them — is ONE workgroup per frame in ONE launch: no host round trip
// per LM trial, and a batch of frames (cameras of a rig, agents, a replayed sequence) fills the chip.
// Inside a workgroup the edges are processed in the pose-sample space like k_linearize: every edge of
// an asynchronous camera sees the GP pose between the two frames at that camera's time stamp, so the
// frame has at most one sample per camera; J = J1 N with the sample's factor N (6 x 24), and
// sum J^T W J = N^T (sum J1^T W J1) N per sample.  Edges, Jacobians and GP maths are the ones of
// lba_math.hpp (src/G2oTypes.cc:162-223, include/G2oTypes.h:186-270); the LM loop is g2o's
// OptimizationAlgorithmLevenberg (optimization_algorithm_levenberg.cpp:61-194) without a user lambda.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/amc_lba.h"
#include "lba_math.hpp"

using namespace lba;

namespace {

constexpr int TR_THREADS = 256;
constexpr int TR_MAXS = 16;   // pose samples per frame: distinct camera time stamps + the frame's own pose
constexpr int CAMD_N = 16;    // Rcb(9) tcb(3) fx fy cx cy

struct TrackArgs {
    lba_track_frame* frames;
    lba_track_obs* obs;       // per frame, sorted by pose sample
    const int* obs_smp;       // per observation: the frame-local sample index
    const int* smp0;          // per frame: first sample (global index) [n_frames + 1]
    const int* smp_obs0;      // per sample: first observation; [smp_obs0[s], smp_obs0[s + 1])
    const double* smp_t;      // per sample: time stamp (GP samples)
    const int* smp_kf;        // per sample: 1 = the frame's own pose (reference camera)
    const double* camd;       // [n_cam][CAMD_N]
    double* chi2;             // per observation: e^T Omega e of the last evaluation (g2o's stale semantics)
    double qcinv[36];
    double huber_mono, huber_stereo, tau, lambda_init;
    int max_trials, early_stop;
};

__device__ __forceinline__ void load_camd(const double* c, CamD* d) {
    for (int i = 0; i < 9; ++i) d->Rcb[i] = c[i];
    for (int i = 0; i < 3; ++i) d->tcb[i] = c[9 + i];
    d->fx = c[12]; d->fy = c[13]; d->cx = c[14]; d->cy = c[15];
}

__device__ __forceinline__ SE3 kf_se3(const double* k) {
    SE3 T;
    T.q = Quat{k[0], k[1], k[2], k[3]};
    T.t[0] = k[4]; T.t[1] = k[5]; T.t[2] = k[6];
    return T;
}

template <int N>
__device__ __forceinline__ void block_sum_vec(double (&v)[N], double* red) {   // every thread gets the sums
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v[i] += __shfl_xor(v[i], o);
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < N; ++i) red[wave * N + i] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double s = 0.0;
        for (int w = 0; w < TR_THREADS / 64; ++w) s += red[w * N + i];   // fixed order: same bits everywhere
        v[i] = s;
    }
    __syncthreads();
}

struct TrackShared {
    double ks[2][2][16];       // [state buffer][KF a = prev, KF b = cur]: q t v time bf fixed
    GPPair gpp;
    double sR[TR_MAXS][12];    // sample poses Rwb twb
    double sN[TR_MAXS][144];   // sample factors N (transposed: N[c * 6 + l] = N(l, c))
    double H[576], bv[24], x[24];
    double Msh[28], MN[144];
    double prJ[288], prOJ[288], prOm[144], prE[12], prOe[12];
    double red[(TR_THREADS / 64) * 28];
    double scal[8];
    int flag[8];
};

// GP pair of the state `buf` and the frame's pose samples (jac: with their factors N)
__device__ void prep(const TrackArgs& A, TrackShared& S, int buf, bool jac, int s0, int ns) {
    const double* ka = S.ks[buf][0];
    const double* kb = S.ks[buf][1];
    if (threadIdx.x == 0) gp_pair_build(kf_se3(ka), ka + 7, kf_se3(kb), kb + 7, ka[13], kb[13], &S.gpp, jac);
    __syncthreads();
    const int si = threadIdx.x;
    if (si < ns) {
        const int s = s0 + si;
        double* R = S.sR[si];
        if (A.smp_kf[s]) {   // the frame's own pose: N = [0 | I 0]
            qmat(kf_se3(kb).q, R);
            R[9] = kb[4]; R[10] = kb[5]; R[11] = kb[6];
            if (jac)
                for (int e = 0; e < 144; ++e) S.sN[si][e] = ((e / 6) >= 12 && (e / 6) < 18 && (e % 6) == (e / 6) - 12) ? 1.0 : 0.0;
        } else if (jac) {
            GPSample G;
            gp_sample_build(S.gpp, A.smp_t[s], &G);
            for (int i = 0; i < 12; ++i) R[i] = i < 9 ? G.Rwb[i] : G.twb[i - 9];
            for (int e = 0; e < 144; ++e) S.sN[si][e] = G.N[e];
        } else {
            double xi[6];
            GPScalars g;
            gp_sample_pose(S.gpp, A.smp_t[s], R, R + 9, xi, &g);
        }
    }
    __syncthreads();
}

// residual of observation o at its sample pose; returns DIM
__device__ __forceinline__ int residual(const TrackArgs& A, const TrackShared& S, int o, int buf, double* e, double* Xb,
                                        double* Xc, CamD& cd) {
    const lba_track_obs& ob = A.obs[o];
    const double* R = S.sR[A.obs_smp[o]];
    load_camd(A.camd + (size_t)ob.cam * CAMD_N, &cd);
    const double bf = S.ks[buf][1][14];
    if (ob.kind == LBA_STEREO) {
        project_residual<3>(R, R + 9, cd, ob.Xw, ob.z, bf, Xb, Xc, e);
        return 3;
    }
    project_residual<2>(R, R + 9, cd, ob.Xw, ob.z, bf, Xb, Xc, e);
    e[2] = 0.0;
    return 2;
}

// motion prior + velocity edges: chi2 (and with jac the quadratic form into H / bv).  All threads.
__device__ double prior_terms(const TrackArgs& A, TrackShared& S, int buf, bool jac, int d0) {
    const double* ka = S.ks[buf][0];
    const double* kb = S.ks[buf][1];
    const int tid = threadIdx.x;
    if (tid == 0) {
        double Ji[144], Jj[144];
        prior_error_jac<double>(kf_se3(ka), ka + 7, ka[13], kf_se3(kb), kb + 7, kb[13], S.prE, jac ? Ji : nullptr,
                                jac ? Jj : nullptr);
        qi_inv(A.qcinv, kb[13] - ka[13], S.prOm);
        if (jac)
            for (int r = 0; r < 12; ++r)
                for (int c = 0; c < 12; ++c) { S.prJ[r * 24 + c] = Ji[r * 12 + c]; S.prJ[r * 24 + 12 + c] = Jj[r * 12 + c]; }
    }
    __syncthreads();
    if (tid < 12) {
        double s = 0.0;
        for (int q = 0; q < 12; ++q) s += S.prOm[tid * 12 + q] * S.prE[q];
        S.prOe[tid] = s;
    }
    if (jac)
        for (int e = tid; e < 288; e += TR_THREADS) {
            const int r = e / 24, c = e % 24;
            double s = 0.0;
            for (int q = 0; q < 12; ++q) s += S.prOm[r * 12 + q] * S.prJ[q * 24 + c];
            S.prOJ[e] = s;
        }
    __syncthreads();
    if (jac) {
        for (int e = tid; e < 300; e += TR_THREADS) {   // upper triangle (i <= j), then mirrored
            int i = 0, rem = e;
            while (rem >= 24 - i) { rem -= 24 - i; ++i; }
            const int j = i + rem;
            double h = 0.0;
            for (int r = 0; r < 12; ++r) h += S.prJ[r * 24 + i] * S.prOJ[r * 24 + j];
            S.H[i * 24 + j] += h;
        }
        if (tid < 24) {
            double s = 0.0;
            for (int r = 0; r < 12; ++r) s += S.prJ[r * 24 + tid] * S.prOe[r];
            S.bv[tid] -= s;
        }
        __syncthreads();
        if (tid == 0) {   // EdgeVelocity on each free vertex: e = vel_z, info QcInv(2,2)
            for (int k = (d0 == 12 ? 1 : 0); k < 2; ++k) {
                S.H[(12 * k + 8) * 24 + 12 * k + 8] += A.qcinv[14];
                S.bv[12 * k + 8] -= A.qcinv[14] * S.ks[buf][k][9];
            }
        }
        __syncthreads();
    }
    double chi = 0.0;
    for (int q = 0; q < 12; ++q) chi += S.prE[q] * S.prOe[q];
    for (int k = (d0 == 12 ? 1 : 0); k < 2; ++k) {
        const double v = S.ks[buf][k][9];
        chi += v * (A.qcinv[14] * v);
    }
    return chi;
}

// computeActiveErrors + activeRobustChi2 at the state `buf` (per-edge chi2 stored, stale semantics)
__device__ double evaluate(const TrackArgs& A, TrackShared& S, int f, int buf, bool robust, int d0, int s0, int ns) {
    prep(A, S, buf, false, s0, ns);
    const lba_track_frame& F = A.frames[f];
    double acc[1] = {0.0};
    for (int o = F.obs0 + threadIdx.x; o < F.obs0 + F.n_obs; o += TR_THREADS) {
        if (A.obs[o].outlier) continue;
        double e[3], Xb[3], Xc[3];
        CamD cd;
        const int dim = residual(A, S, o, buf, e, Xb, Xc, cd);
        double c = 0.0;
        for (int d = 0; d < dim; ++d) c += e[d] * (A.obs[o].w * e[d]);
        A.chi2[o] = c;
        double r0 = c, r1;
        if (robust) huber(c, dim == 3 ? A.huber_stereo : A.huber_mono, &r0, &r1);
        acc[0] += r0;
    }
    block_sum_vec<1>(acc, S.red);
    return acc[0] + prior_terms(A, S, buf, false, d0);
}

// computeActiveErrors + buildSystem at the state `buf`: H, bv (24-dof, both frames), returns the chi2
__device__ double linearize(const TrackArgs& A, TrackShared& S, int f, int buf, bool robust, int d0, int s0, int ns) {
    prep(A, S, buf, true, s0, ns);
    const int tid = threadIdx.x;
    for (int e = tid; e < 576; e += TR_THREADS) S.H[e] = 0.0;
    if (tid < 24) S.bv[tid] = 0.0;
    __syncthreads();
    double chi = 0.0;
    for (int si = 0; si < ns; ++si) {
        const int s = s0 + si;
        // sample-space partial: M = sum s J1^T J1 (upper 21), g = sum s J1^T e (6), robust chi2
        double v[28];
#pragma unroll
        for (int q = 0; q < 28; ++q) v[q] = 0.0;
        for (int o = A.smp_obs0[s] + tid; o < A.smp_obs0[s + 1]; o += TR_THREADS) {
            if (A.obs[o].outlier) continue;
            double e[3], Xb[3], Xc[3], J1[18], Jp[9];
            CamD cd;
            const int dim = residual(A, S, o, buf, e, Xb, Xc, cd);
            const double* R = S.sR[si];
            if (dim == 3) obs_j1<3>(R, cd, Xb, Xc, S.ks[buf][1][14], J1, Jp);
            else obs_j1<2>(R, cd, Xb, Xc, S.ks[buf][1][14], J1, Jp);
            double c = 0.0;
            for (int d = 0; d < dim; ++d) c += e[d] * (A.obs[o].w * e[d]);
            A.chi2[o] = c;
            double r0 = c, r1 = 1.0;
            if (robust) huber(c, dim == 3 ? A.huber_stereo : A.huber_mono, &r0, &r1);
            const double sw = r1 * A.obs[o].w;   // robustInformation (base_edge.h:96-102)
            v[27] += r0;
            for (int d = 0; d < dim; ++d) {
                const double* j = J1 + 6 * d;
                int q = 0;
                for (int a = 0; a < 6; ++a)
                    for (int b = a; b < 6; ++b) v[q++] += sw * j[a] * j[b];
                for (int a = 0; a < 6; ++a) v[21 + a] += sw * j[a] * e[d];
            }
        }
        block_sum_vec<28>(v, S.red);
        chi += v[27];
        if (tid < 28) S.Msh[tid] = v[tid];
        __syncthreads();
        // MN = M N (6 x 24); H += N^T MN (upper); bv -= N^T g
        if (tid < 144) {
            const int a = tid / 24, c = tid % 24;
            double sacc = 0.0;
            for (int l = 0; l < 6; ++l) {
                const int lo = a < l ? a : l, hi = a < l ? l : a;
                const int qi = lo * 6 - lo * (lo - 1) / 2 + (hi - lo);   // upper-triangle index of (lo, hi)
                sacc += S.Msh[qi] * S.sN[si][c * 6 + l];
            }
            S.MN[a * 24 + c] = sacc;
        }
        __syncthreads();
        for (int e = tid; e < 300; e += TR_THREADS) {
            int i = 0, rem = e;
            while (rem >= 24 - i) { rem -= 24 - i; ++i; }
            const int j = i + rem;
            double h = 0.0;
            for (int a = 0; a < 6; ++a) h += S.sN[si][i * 6 + a] * S.MN[a * 24 + j];
            S.H[i * 24 + j] += h;
        }
        if (tid < 24) {
            double g = 0.0;
            for (int a = 0; a < 6; ++a) g += S.sN[si][tid * 6 + a] * S.Msh[21 + a];
            S.bv[tid] -= g;
        }
        __syncthreads();
    }
    chi += prior_terms(A, S, buf, true, d0);
    for (int e = tid; e < 576; e += TR_THREADS) {   // mirror the upper triangle
        const int i = e / 24, j = e % 24;
        if (j < i) S.H[e] = S.H[j * 24 + i];
    }
    __syncthreads();
    return chi;
}

// (H + lambda I) x = bv over the active dofs [d0, 24): Cholesky on one thread (n <= 24); 1 if positive
__device__ int solve(TrackShared& S, double lambda, int d0) {
    if (threadIdx.x == 0) {
        const int n = 24 - d0;
        double L[576];
        int ok = 1;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j <= i; ++j) L[i * 24 + j] = S.H[(d0 + i) * 24 + d0 + j] + (i == j ? lambda : 0.0);
        for (int k = 0; k < n && ok; ++k) {
            double d = L[k * 24 + k];
            for (int p = 0; p < k; ++p) d -= L[k * 24 + p] * L[k * 24 + p];
            if (!(d > 0.0)) { ok = 0; break; }
            const double r = sqrt(d);
            L[k * 24 + k] = r;
            for (int i = k + 1; i < n; ++i) {
                double s = L[i * 24 + k];
                for (int p = 0; p < k; ++p) s -= L[i * 24 + p] * L[k * 24 + p];
                L[i * 24 + k] = s / r;
            }
        }
        double y[24];
        for (int i = 0; ok && i < n; ++i) {
            double s = S.bv[d0 + i];
            for (int p = 0; p < i; ++p) s -= L[i * 24 + p] * y[p];
            y[i] = s / L[i * 24 + i];
        }
        for (int i = n - 1; ok && i >= 0; --i) {
            double s = y[i];
            for (int p = i + 1; p < n; ++p) s -= L[p * 24 + i] * S.x[p];
            S.x[i] = s / L[i * 24 + i];
        }
        S.flag[0] = ok;
    }
    __syncthreads();
    return S.flag[0];
}

// trial state: buffer `to` = `from` (+) x on the free frames (T <- T exp(dxi), v += dv, src/G2oTypes.cc:41-46)
__device__ void update(TrackShared& S, int from, int to, int d0, bool ok) {
    if (threadIdx.x < 2) {
        const int k = threadIdx.x;
        const double* kc = S.ks[from][k];
        double* kn = S.ks[to][k];
        if (ok && 12 * k >= d0) {
            const double* d = S.x + 12 * k - d0;
            const SE3 T = se3_mul(kf_se3(kc), se3_exp(d));
            kn[0] = T.q.x; kn[1] = T.q.y; kn[2] = T.q.z; kn[3] = T.q.w;
            kn[4] = T.t[0]; kn[5] = T.t[1]; kn[6] = T.t[2];
            for (int j = 0; j < 6; ++j) kn[7 + j] = kc[7 + j] + d[6 + j];
            for (int j = 13; j < 16; ++j) kn[j] = kc[j];
        } else {
            for (int j = 0; j < 16; ++j) kn[j] = kc[j];
        }
    }
    __syncthreads();
}

__device__ __forceinline__ bool depth_at(const double* k, const CamD& cd, const double* Xw) {
    double R[9];
    qmat(kf_se3(k).q, R);
    const double d[3] = {Xw[0] - k[4], Xw[1] - k[5], Xw[2] - k[6]};
    double Xb[3];
    mul33tv(R, d, Xb);
    const double zc = cd.Rcb[6] * Xb[0] + cd.Rcb[7] * Xb[1] + cd.Rcb[8] * Xb[2] + cd.tcb[2];
    return zc > 0;
}

__global__ __launch_bounds__(TR_THREADS) void k_track(TrackArgs A) {
    __shared__ TrackShared S;
    const int f = blockIdx.x, tid = threadIdx.x;
    lba_track_frame& F = A.frames[f];
    const int s0 = A.smp0[f], ns = A.smp0[f + 1] - s0;
    if (tid < 16) {
        const lba_kf* src[2] = {&F.prev, &F.cur};
        for (int k = 0; k < 2; ++k) {
            const lba_kf& q = *src[k];
            double* d = S.ks[0][k];
            const double v[16] = {q.q[0], q.q[1], q.q[2], q.q[3], q.t[0], q.t[1], q.t[2], q.vel[0], q.vel[1], q.vel[2],
                                  q.vel[3], q.vel[4], q.vel[5], q.time, q.bf, 0.0};
            d[tid] = v[tid];
        }
    }
    __syncthreads();
    if (tid == 0) {   // Sophus cast<double>(): normalised quaternions
        for (int k = 0; k < 2; ++k) {
            const Quat n = qnormalize(Quat{S.ks[0][k][0], S.ks[0][k][1], S.ks[0][k][2], S.ks[0][k][3]});
            S.ks[0][k][0] = n.x; S.ks[0][k][1] = n.y; S.ks[0][k][2] = n.z; S.ks[0][k][3] = n.w;
        }
    }
    __syncthreads();
    const int d0 = F.prev.fixed ? 12 : 0;
    const float chi2Mono[4] = {5.991f, 5.991f, 5.991f, 5.991f};
    const float chi2Stereo[4] = {15.6f, 9.8f, 7.815f, 7.815f};
    int cur = 0, iters = 0, nBad = 0;
    bool robust = true;
    for (int it = 0; it < 4; ++it) {
        // ---- initializeOptimization(0) + optimize(10): g2o Levenberg (lambda from computeLambdaInit)
        double lambda = 0.0, ni = 2.0;
        int nbad_lm = 0;
        for (int k = 0; k < 10; ++k) {
            double currentChi = linearize(A, S, f, cur, robust, d0, s0, ns);
            const double iniChi = currentChi;
            if (k == 0) {
                double m = 0.0;
                for (int i = d0; i < 24; ++i) m = fmax(m, fabs(S.H[i * 24 + i]));
                lambda = A.lambda_init > 0 ? A.lambda_init : A.tau * m;
                ni = 2.0;
                nbad_lm = 0;
            }
            double rho = 0.0;
            int qmax = 0;
            do {
                const int ok = solve(S, lambda, d0);
                update(S, cur, cur ^ 1, d0, ok);
                double tempChi = evaluate(A, S, f, cur ^ 1, robust, d0, s0, ns);
                if (!ok) tempChi = DBL_MAX;
                double scale = 1e-3;
                if (ok)
                    for (int i = 0; i < 24 - d0; ++i) scale += S.x[i] * (lambda * S.x[i] + S.bv[d0 + i]);
                rho = (currentChi - tempChi) / scale;
                if (rho > 0 && isfinite(tempChi)) {
                    const double t = 2 * rho - 1;
                    double alpha = 1. - t * t * t;
                    alpha = fmin(alpha, 2. / 3.);
                    lambda *= fmax(1. / 3., alpha);
                    ni = 2;
                    currentChi = tempChi;
                    cur ^= 1;   // discardTop: the trial state becomes current
                } else {
                    lambda *= ni;
                    ni *= 2;
                }
                qmax++;
                __syncthreads();
            } while (rho < 0 && qmax < A.max_trials);
            ++iters;
            bool stop = qmax == A.max_trials || rho == 0;
            if (!stop) {
                if ((iniChi - currentChi) * 1e3 < iniChi) nbad_lm++;
                else nbad_lm = 0;
                stop = nbad_lm >= 3;
            }
            if (stop && A.early_stop) break;
        }
        // ---- re-classification (Optimizer.cc:575-672) at the current estimate
        prep(A, S, cur, false, s0, ns);
        double cnt[1] = {0.0};
        const float chi2close = (float)(1.5 * chi2Mono[it]);
        for (int o = F.obs0 + tid; o < F.obs0 + F.n_obs; o += TR_THREADS) {
            lba_track_obs& ob = A.obs[o];
            double e[3], Xb[3], Xc[3];
            CamD cd;
            const int dim = residual(A, S, o, cur, e, Xb, Xc, cd);
            if (ob.outlier) {   // e->computeError() for the level-1 edges
                double c = 0.0;
                for (int d = 0; d < dim; ++d) c += e[d] * (ob.w * e[d]);
                A.chi2[o] = c;
            }
            const float c2 = (float)A.chi2[o];
            int out;
            if (ob.kind == LBA_STEREO) {
                out = c2 > chi2Stereo[it];
            } else {
                const bool bclose = ob.close != 0;
                bool depth = depth_at(S.ks[cur][1], cd, ob.Xw);
                if (ob.kind == LBA_MONO_GP) depth = depth && depth_at(S.ks[cur][0], cd, ob.Xw);
                out = (c2 > chi2Mono[it] && !bclose) || (bclose && c2 > chi2close) || !depth;
            }
            ob.outlier = out;
            cnt[0] += out;
        }
        block_sum_vec<1>(cnt, S.red);
        nBad = (int)cnt[0];
        if (it == 2) robust = false;   // e->setRobustKernel(0)
        if (F.n_obs + 3 < 10) break;   // optimizer.edges().size() < 10
    }
    if (tid == 0) {
        const double* k = S.ks[cur][1];
        for (int i = 0; i < 4; ++i) F.cur.q[i] = k[i];
        for (int i = 0; i < 3; ++i) F.cur.t[i] = k[4 + i];
        for (int i = 0; i < 6; ++i) F.cur.vel[i] = k[7 + i];
        F.n_good = F.n_obs - nBad;
        F.iterations = iters;
    }
}

struct HipErr {
    hipError_t e;
};
#define TCHK(x)                                    \
    do {                                           \
        hipError_t _e = (x);                       \
        if (_e != hipSuccess) throw HipErr{_e};    \
    } while (0)

}  // namespace

struct lba_tracker {
    lba_config cfg{};
    hipStream_t stream = nullptr;
    lba_track_frame* d_frames = nullptr;
    lba_track_obs* d_obs = nullptr;
    int *d_obs_smp = nullptr, *d_smp0 = nullptr, *d_smp_obs0 = nullptr, *d_smp_kf = nullptr;
    double *d_smp_t = nullptr, *d_camd = nullptr, *d_chi2 = nullptr;
    size_t cap[9] = {};   // capacities of the buffers above, in elements
    std::string err;
};

namespace {
template <typename T>
void grow(T*& p, size_t& cap, size_t n) {
    if (n <= cap && p) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = std::max<size_t>(n, 1) * 2;
    TCHK(hipMalloc(reinterpret_cast<void**>(&p), cap * sizeof(T)));
}
}  // namespace

extern "C" {

int lba_tracker_create(lba_tracker** out, const lba_config* cfg) {
    if (!out || !cfg) return LBA_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || cfg->device < 0 || cfg->device >= ndev) return LBA_E_ARG;
    lba_tracker* t = new lba_tracker();
    t->cfg = *cfg;
    if (t->cfg.max_trials <= 0) t->cfg.max_trials = 10;
    if (t->cfg.tau <= 0) t->cfg.tau = 1e-5;
    if (hipSetDevice(cfg->device) != hipSuccess || hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess) {
        delete t;
        return LBA_E_HIP;
    }
    *out = t;
    return LBA_OK;
}

void lba_tracker_destroy(lba_tracker* t) {
    if (!t) return;
    (void)hipSetDevice(t->cfg.device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    void* bufs[] = {t->d_frames, t->d_obs, t->d_obs_smp, t->d_smp0, t->d_smp_obs0, t->d_smp_kf, t->d_smp_t, t->d_camd, t->d_chi2};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (t->stream) (void)hipStreamDestroy(t->stream);
    delete t;
}

int lba_track(lba_tracker* t, lba_track_frame* frames, int32_t n_frames, lba_track_obs* obs, int32_t n_obs,
              const lba_cam* cams, int32_t n_cam) {
    if (!t || n_frames < 0 || n_obs < 0 || (n_frames && !frames) || (n_obs && !obs) || n_cam < 1 || !cams)
        return LBA_E_ARG;
    if (n_frames == 0) return LBA_OK;
    // ---- per frame: pose samples (distinct time stamps of the GP observations, then the frame's own
    //      pose for the reference camera) and the observations ordered by sample
    std::vector<int> perm, obs_smp, smp0(1, 0), smp_obs0, smp_kf;
    std::vector<double> smp_t;
    perm.reserve(n_obs);
    for (int f = 0; f < n_frames; ++f) {
        const lba_track_frame& F = frames[f];
        if (F.obs0 < 0 || F.n_obs < 0 || (int64_t)F.obs0 + F.n_obs > n_obs) return LBA_E_ARG;
        if (!(std::fabs(F.cur.time - F.prev.time) > 1e-6)) return LBA_E_ARG;   // QiInv (GaussianProcess.h:32)
        std::vector<double> ts;
        bool has_kf = false;
        for (int i = F.obs0; i < F.obs0 + F.n_obs; ++i) {
            const lba_track_obs& o = obs[i];
            if (o.cam < 0 || o.cam >= n_cam) return LBA_E_ARG;
            if (o.kind == LBA_MONO_GP) ts.push_back(o.t);
            else if (o.kind == LBA_MONO || o.kind == LBA_STEREO) has_kf = true;
            else return LBA_E_ARG;
        }
        std::sort(ts.begin(), ts.end());
        ts.erase(std::unique(ts.begin(), ts.end()), ts.end());
        const int ns = (int)ts.size() + (has_kf ? 1 : 0);
        if (ns > TR_MAXS) {
            t->err = "more than 16 distinct observation times in a frame";
            return LBA_E_LIMIT;
        }
        std::vector<std::vector<int>> by(ns);
        for (int i = F.obs0; i < F.obs0 + F.n_obs; ++i) {
            const lba_track_obs& o = obs[i];
            const int s = o.kind == LBA_MONO_GP ? (int)(std::lower_bound(ts.begin(), ts.end(), o.t) - ts.begin())
                                               : (int)ts.size();
            by[s].push_back(i);
        }
        for (int s = 0; s < ns; ++s) {
            smp_obs0.push_back((int)perm.size());
            smp_t.push_back(s < (int)ts.size() ? ts[s] : F.cur.time);
            smp_kf.push_back(s < (int)ts.size() ? 0 : 1);
            for (int i : by[s]) {
                perm.push_back(i);
                obs_smp.push_back(s);
            }
        }
        smp0.push_back((int)smp_t.size());
    }
    smp_obs0.push_back((int)perm.size());
    std::vector<lba_track_obs> sob(perm.size());
    std::vector<lba_track_frame> sfr(frames, frames + n_frames);
    {
        size_t q = 0;
        for (int f = 0; f < n_frames; ++f) {
            sfr[f].obs0 = (int)q;
            for (int i = 0; i < frames[f].n_obs; ++i, ++q) sob[q] = obs[perm[q]];
        }
    }
    std::vector<double> camd((size_t)n_cam * CAMD_N);
    for (int c = 0; c < n_cam; ++c) {
        Cam cm;
        for (int i = 0; i < 4; ++i) cm.q[i] = cams[c].q[i];
        for (int i = 0; i < 3; ++i) cm.t[i] = cams[c].t[i];
        cm.fx = cams[c].fx; cm.fy = cams[c].fy; cm.cx = cams[c].cx; cm.cy = cams[c].cy;
        CamD d;
        cam_derive(cm, &d);
        double* o = camd.data() + (size_t)c * CAMD_N;
        for (int i = 0; i < 9; ++i) o[i] = d.Rcb[i];
        for (int i = 0; i < 3; ++i) o[9 + i] = d.tcb[i];
        o[12] = d.fx; o[13] = d.fy; o[14] = d.cx; o[15] = d.cy;
    }
    try {
        TCHK(hipSetDevice(t->cfg.device));
        grow(t->d_frames, t->cap[0], (size_t)n_frames);
        grow(t->d_obs, t->cap[1], perm.size());
        grow(t->d_obs_smp, t->cap[2], perm.size());
        grow(t->d_chi2, t->cap[3], perm.size());
        grow(t->d_smp0, t->cap[4], smp0.size());
        grow(t->d_smp_obs0, t->cap[5], smp_obs0.size());
        grow(t->d_smp_kf, t->cap[6], smp_kf.size());
        grow(t->d_smp_t, t->cap[7], smp_t.size());
        grow(t->d_camd, t->cap[8], camd.size());
        hipStream_t s = t->stream;
        TCHK(hipMemcpyAsync(t->d_frames, sfr.data(), sizeof(lba_track_frame) * n_frames, hipMemcpyHostToDevice, s));
        if (!sob.empty()) {
            TCHK(hipMemcpyAsync(t->d_obs, sob.data(), sizeof(lba_track_obs) * sob.size(), hipMemcpyHostToDevice, s));
            TCHK(hipMemcpyAsync(t->d_obs_smp, obs_smp.data(), sizeof(int) * obs_smp.size(), hipMemcpyHostToDevice, s));
        }
        TCHK(hipMemcpyAsync(t->d_smp0, smp0.data(), sizeof(int) * smp0.size(), hipMemcpyHostToDevice, s));
        TCHK(hipMemcpyAsync(t->d_smp_obs0, smp_obs0.data(), sizeof(int) * smp_obs0.size(), hipMemcpyHostToDevice, s));
        if (!smp_kf.empty()) {
            TCHK(hipMemcpyAsync(t->d_smp_kf, smp_kf.data(), sizeof(int) * smp_kf.size(), hipMemcpyHostToDevice, s));
            TCHK(hipMemcpyAsync(t->d_smp_t, smp_t.data(), sizeof(double) * smp_t.size(), hipMemcpyHostToDevice, s));
        }
        TCHK(hipMemcpyAsync(t->d_camd, camd.data(), sizeof(double) * camd.size(), hipMemcpyHostToDevice, s));
        TrackArgs a;
        a.frames = t->d_frames; a.obs = t->d_obs; a.obs_smp = t->d_obs_smp; a.smp0 = t->d_smp0;
        a.smp_obs0 = t->d_smp_obs0; a.smp_t = t->d_smp_t; a.smp_kf = t->d_smp_kf; a.camd = t->d_camd; a.chi2 = t->d_chi2;
        double qcinv[36];
        {   // GaussianProcess::mQcInv = Qc.inverse() (Gauss-Jordan, partial pivoting)
            double M[6][12];
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j < 12; ++j) M[i][j] = j < 6 ? t->cfg.qc[i * 6 + j] : (j - 6 == i ? 1.0 : 0.0);
            for (int c = 0; c < 6; ++c) {
                int piv = c;
                for (int r = c + 1; r < 6; ++r)
                    if (std::fabs(M[r][c]) > std::fabs(M[piv][c])) piv = r;
                if (M[piv][c] == 0.0) return LBA_E_ARG;
                if (piv != c)
                    for (int j = 0; j < 12; ++j) std::swap(M[c][j], M[piv][j]);
                const double d = M[c][c];
                for (int j = 0; j < 12; ++j) M[c][j] /= d;
                for (int r = 0; r < 6; ++r)
                    if (r != c) {
                        const double fct = M[r][c];
                        if (fct != 0.0)
                            for (int j = 0; j < 12; ++j) M[r][j] -= fct * M[c][j];
                    }
            }
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j < 6; ++j) qcinv[i * 6 + j] = M[i][6 + j];
        }
        std::memcpy(a.qcinv, qcinv, sizeof(qcinv));
        a.huber_mono = t->cfg.huber_mono; a.huber_stereo = t->cfg.huber_stereo;
        a.tau = t->cfg.tau; a.lambda_init = t->cfg.lambda_init;
        a.max_trials = t->cfg.max_trials; a.early_stop = t->cfg.early_stop;
        hipLaunchKernelGGL(k_track, dim3(n_frames), dim3(TR_THREADS), 0, s, a);
        TCHK(hipGetLastError());
        TCHK(hipMemcpyAsync(sfr.data(), t->d_frames, sizeof(lba_track_frame) * n_frames, hipMemcpyDeviceToHost, s));
        if (!sob.empty())
            TCHK(hipMemcpyAsync(sob.data(), t->d_obs, sizeof(lba_track_obs) * sob.size(), hipMemcpyDeviceToHost, s));
        TCHK(hipStreamSynchronize(s));
    } catch (const HipErr&) {
        t->err = "HIP error";
        return LBA_E_HIP;
    }
    for (size_t q = 0; q < perm.size(); ++q) obs[perm[q]].outlier = sob[q].outlier;
    for (int f = 0; f < n_frames; ++f) {
        std::memcpy(frames[f].cur.q, sfr[f].cur.q, sizeof(frames[f].cur.q));
        std::memcpy(frames[f].cur.t, sfr[f].cur.t, sizeof(frames[f].cur.t));
        std::memcpy(frames[f].cur.vel, sfr[f].cur.vel, sizeof(frames[f].cur.vel));
        frames[f].n_good = sfr[f].n_good;
        frames[f].iterations = sfr[f].iterations;
    }
    return LBA_OK;
}

}  // extern "C"
