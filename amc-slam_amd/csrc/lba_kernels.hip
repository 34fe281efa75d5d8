// lba_kernels.hip — gfx950 kernels of the GP local bundle adjustment (fp64 throughout).
//
// One LM trial (OptimizationAlgorithmLevenberg::solve, optimization_algorithm_levenberg.cpp:61-169)
// maps to:
//   k_gp_prep        per GP pair and observation time: interpolated pose + Jacobian factor, per-KF
//                    poses                                                  (GaussianProcess.cc:23-42)
//   k_lin_schur      per tile of landmarks: residual, Huber, analytic J straight into an LDS row
//                    buffer, deterministic on-chip reductions into pose-sample partials, Hpl blocks and
//                    Hll/bl (BlockSolver::buildSystem, block_solver.hpp:502-560; edge quadratic forms
//                    base_multi_edge.hpp:170-222), then in the same workgroup the landmark elimination:
//                    Dinv = (Hll + lambda I)^-1, S partials sum Hpl Dinv Hpl^T (fp64 VALU) and rhs
//                    partials (block_solver.hpp:381-430); EdgeGaussianPrior / EdgeVelocity /
//                    EdgeExtrinsicPrior quadratic forms as extra workgroups (src/G2oTypes.cc:100-118)
//   k_expand         per pose sample N^T M N into Hpp / b_p pieces; heavy landmarks (merge + elimination)
//   k_assemble       S = sum Hpp partials + lambda I - sum Schur partials, b_p, bS = b_p - sum g
//                    (block_solver.hpp:432-445)
//   k_chol_*         blocked Cholesky + forward/back substitution of S     (linear_solver_dense.h:65-113)
//   k_update         landmark back-substitution + oplus into the trial state (block_solver.hpp:461-482,
//                    sparse_optimizer.cpp:422-435) + computeScale partials
//   k_eval           residuals / robust chi2 of the trial state           (sparse_optimizer.cpp:61-114)
// All cross-workgroup sums are written as per-workgroup partials and reduced in a fixed order, so
// results are bitwise reproducible run to run (no floating-point atomics).
#include <algorithm>
#include <cfloat>
#include <utility>

#include <hip/hip_ext.h>

#include "lba_device.hpp"
#include "lba_math.hpp"
#include "../../include/amc_lba.h"

namespace lba {

static_assert(sizeof(GPSample) == GPS_STRIDE * sizeof(double), "GPSample layout drifted");
static_assert(CAMD_STRIDE == CAMREC_DOUBLES, "camera record layout drifted");

// phase stamps for diagnostics only (buffer allocated when LBA_PHASE_TIMING is set; the uniform
// null test costs one scalar branch otherwise)
#define LBA_TMARKI(buf, idx, k)                                                \
    do {                                                                        \
        if (buf) {                                                              \
            __syncthreads();                                                    \
            if (threadIdx.x == 0) (buf)[(size_t)(idx) * 16 + (k)] = clock64();  \
        }                                                                       \
    } while (0)
#define LBA_TMARK(buf, k) LBA_TMARKI(buf, blockIdx.x, k)

// LBA_DEBUG_BOUNDS builds (scripts/exp_build.sh dbg -DLBA_DEBUG_BOUNDS, loaded with AMC_LBA_LIB): every
// indexed slab / table write of the sweep, the edge items and the expansion is checked against the
// extent set-up allocated; an out-of-range index is printed and its write skipped (no trap: a fault can
// take the whole node down), and the launch's factorisation status gets LBA_DBG_INFO so the run fails.
// Release builds compile the checks away.
#ifdef LBA_DEBUG_BOUNDS
constexpr int LBA_DBG_INFO = 0x7ffe0000;
#define LBA_INB(P, i, n, what)                                                                            \
    ((unsigned)(i) < (unsigned)(n) ? true                                                                 \
                                   : (printf("lba bounds: %s index %d of %d (block %d thread %d)\n", what, \
                                             (int)(i), (int)(n), (int)blockIdx.x, (int)threadIdx.x),      \
                                      (P).info ? (void)atomicExch((P).info, LBA_DBG_INFO) : (void)0, false))
#else
#define LBA_INB(P, i, n, what) true
#endif

typedef double d4 __attribute__((ext_vector_type(4)));   // v_mfma_f64_16x16x4 accumulator

// Hand-offs between workgroups of one launch (MI355X_MICROARCH.md, inter-workgroup visibility): the payload
// stored write-through (sc1) and drained by every storing wave before the flag / counter, every load of it
// an sc1 load.  stv<WT> / ldv<WT>: plain or sc1 by a template switch (the fused flow's expand and assembly
// tasks publish; the standalone kernels do not need to).
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) int gi32_t;
typedef __attribute__((address_space(1))) unsigned long long gu64_t;

__device__ __forceinline__ double ld_sc1(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store((gu64_t*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
template <bool WT>
__device__ __forceinline__ void stv(double* p, double v) {
    if constexpr (WT) st_sc1(p, v);
    else *p = v;
}
template <bool WT>
__device__ __forceinline__ double ldv(const double* p) {
    if constexpr (WT) return ld_sc1(p);
    else return *p;
}

// queued optimisation (LMCtl): the state buffer a launch works on, whether it runs, its damping
__device__ __forceinline__ int state_idx(const DevProblem& P, int sel) {
    return sel < SEL_CUR ? sel : (P.ctl->cur ^ (sel - SEL_CUR));
}
__device__ __forceinline__ bool gated_off(const LMCtl* c, int gate) {
    return gate != GATE_NONE && (c->done || (gate == GATE_LIN && !c->need_lin));
}
__device__ __forceinline__ double damping(const DevProblem& P, double lambda) {
    return __builtin_isnan(lambda) ? P.ctl->lambda : lambda;   // (LAMBDA_CTL)
}

// element (r, c), r >= c, of the reduced system in factorisation order inside its tile of L (a structural
// non-zero of S always has one: binary search of the row's tile columns)
__device__ __forceinline__ size_t s_elem(const DevProblem& P, int r, int c) {
    const int ti = r / CHOL_NB, tj = c / CHOL_NB;
    int lo = P.cf_rowptr[ti], hi = P.cf_rowptr[ti + 1] - 1;
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (P.cf_cols[m] < tj) lo = m + 1;
        else hi = m;
    }
    return (size_t)lo * (CHOL_NB * CHOL_NB) + (r % CHOL_NB) * CHOL_NB + (c % CHOL_NB);
}

// Storage order of a Schur partial block (sslab slot, 144 doubles = 9 cache lines).  The sweep's S-partial phase
// computes a 12 x 12 block as 8 tasks on 8 consecutive lanes, task L holding rows 3 (L >> 1) .. + 2 and columns
// 6 (L & 1) .. + 5 (element u = 6 i + j of its 18); slot position f = 16 (u >> 1) + 2 L + (u & 1) puts the k-th pair
// of every task into line k, so each of the task's 16-byte stores k = 0..8 writes, with its 7 neighbours, one whole
// line (write-through stores of such lines, or 8-byte ones in the row-major layout, made the sweep 3 and 32 us slower:
// profiles/r7_fold_rejected.txt).  The reductions sum position by position, so only the element a position holds
// changes.
__device__ __forceinline__ int spos_rc(int f) {   // (row << 4 | col) of slot position f
    const int L = (f & 15) >> 1, u = 2 * (f >> 4) + (f & 1);
    const int i = u / 6, j = u - 6 * i;
    return ((3 * (L >> 1) + i) << 4) | (6 * (L & 1) + j);
}
__device__ __forceinline__ int spos_of(int r, int c) {   // slot position of element (r, c)
    const int L = 2 * (r / 3) + c / 6, u = 6 * (r % 3) + c % 6;
    return 16 * (u >> 1) + 2 * L + (u & 1);
}
typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
constexpr int BUF_SC1 = 16;   // buffer instruction cache policy: sc1
// two doubles at p (16-byte aligned), one vector store (plain: the slabs are read by the next launch)
__device__ __forceinline__ void st16(double* p, double a, double b) {
    const dbl2 v = {a, b};
    *reinterpret_cast<dbl2*>(p) = v;
}

__device__ __forceinline__ SE3 load_se3(const double* k) {
    SE3 T;
    T.q = Quat{k[0], k[1], k[2], k[3]};
    T.t[0] = k[4]; T.t[1] = k[5]; T.t[2] = k[6];
    return T;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    return v;
}

// deterministic block sum (blockDim multiple of 64, <= 1024); valid in thread 0
template <int NT>
__device__ __forceinline__ double block_sum(double v, double* red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < NT / 64; ++w) s += red[w];
    return s;
}

__device__ __forceinline__ void load_cam(const double* c, CamD* d) {
    for (int i = 0; i < 9; ++i) d->Rcb[i] = c[i];
    d->tcb[0] = c[9]; d->tcb[1] = c[10]; d->tcb[2] = c[11];
    d->fx = c[12]; d->fy = c[13]; d->cx = c[14]; d->cy = c[15];
}

// Pose of the body at the observation time (Rwb, twb): the observation's pose sample (a GP sample for
// GP edges, the KF pose record for EdgeMono / EdgeStereo).  Returns the stereo bf of the edge's first
// KF vertex.
// ObsIn: an observation's per-observation inputs, loaded together with its ob_meta by the caller (before the
// branch on its kind, so they are one memory round trip, not one after the meta load and one more after that).
struct ObsIn {
    int kfa, kfb, smp, lm;
    double z[3], w;
};
__device__ __forceinline__ ObsIn obs_in(const DevProblem& P, int o) {
    ObsIn in;
    in.kfa = P.ob_kfa[o];
    in.kfb = P.ob_kfb[o];
    in.smp = P.ob_smp[o];
    in.lm = P.ob_lm[o];
#pragma unroll
    for (int d = 0; d < 3; ++d) in.z[d] = P.ob_z[3 * (size_t)o + d];
    in.w = P.ob_w[o];
    return in;
}
__device__ __forceinline__ double obs_pose(const double* gps, const double* kst, const ObsIn& in, bool gp,
                                           double* Rwb, double* twb) {
    const int ka = gp ? in.kfa : in.kfb;
    const double* S = gps + (size_t)in.smp * GPS_STRIDE;
#pragma unroll
    for (int i = 0; i < 9; ++i) Rwb[i] = S[i];
    twb[0] = S[9]; twb[1] = S[10]; twb[2] = S[11];
    return kst[(size_t)ka * KF_STRIDE + 14];
}

// One observation of the linearisation (DIM compile-time so every per-row array stays in
// registers): residual, Huber weight, the rows [J1 e Jp] into the LDS row buffer (J1 w.r.t. the
// pose sample: the pose / velocity Jacobian J1 N is never formed, see k_linearize); returns rho(chi2).
template <int DIM, bool F32 = false>
__device__ __forceinline__ double lin_obs(const DevProblem& P, const double* gps, const double* kst, const double* lst,
                                          const double* camd, int o, const ObsIn& in, int cam, bool gp, double* rows,
                                          double* rw, int write_res) {
    CamD cd;
    load_cam(camd + (size_t)cam * CAMD_STRIDE, &cd);
    double Rwb[9], twb[3];
    const double bf = obs_pose(gps, kst, in, gp, Rwb, twb);
    const double* Xw = lst + (size_t)in.lm * 3;
    double z[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) z[d] = in.z[d];
    const double w = in.w;
    double Xb[3], Xc[3], e[DIM];
    project_residual_p<DIM, F32>(Rwb, twb, cd, Xw, z, bf, Xb, Xc, e);
    double chi = 0.0;
#pragma unroll
    for (int d = 0; d < DIM; ++d) chi += e[d] * (w * e[d]);
    double r0, r1;
    huber(chi, DIM == 3 ? P.huber_stereo : P.huber_mono, &r0, &r1);
    double J1[6 * DIM], Jp[3 * DIM];
    obs_j1_p<DIM, F32>(Rwb, cd, Xb, Xc, bf, J1, Jp);
    const double s = r1 * w;   // robustInformation = rho' * Omega (base_edge.h:96-102), Omega = w I
    const int row = P.ob_row[o] & 0xffff;
#pragma unroll
    for (int d = 0; d < DIM; ++d) {
        double* R = rows + (row + d) * ROW_STRIDE;
#pragma unroll
        for (int j = 0; j < 6; ++j) R[j] = J1[d * 6 + j];
        R[6] = e[d];
#pragma unroll
        for (int j = 0; j < 3; ++j) R[7 + j] = Jp[d * 3 + j];
        rw[row + d] = s;
    }
    P.ob_chi2[o] = chi;
    if (write_res)
#pragma unroll
        for (int d = 0; d < 3; ++d) P.ob_res[3 * (size_t)o + d] = d < DIM ? e[d] : 0.0;
    return r0;
}

// Residual-only evaluation of one observation (computeError + robust chi2) at the body pose (Rwb, twb) and
// landmark Xw; returns rho(chi2).
template <int DIM, bool F32 = false>
__device__ __forceinline__ double eval_obs_at(const DevProblem& P, const double* Rwb, const double* twb, double bf,
                                              const double* Xw, const double* camd, int o, const ObsIn& in, int cam) {
    CamD cd;
    load_cam(camd + (size_t)cam * CAMD_STRIDE, &cd);
    double z[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) z[d] = in.z[d];
    const double w = in.w;
    double Xb[3], Xc[3], e[DIM];
    project_residual_p<DIM, F32>(Rwb, twb, cd, Xw, z, bf, Xb, Xc, e);
    double chi = 0.0;
#pragma unroll
    for (int d = 0; d < DIM; ++d) chi += e[d] * (w * e[d]);
    double r0, r1;
    huber(chi, DIM == 3 ? P.huber_stereo : P.huber_mono, &r0, &r1);
    P.ob_chi2[o] = chi;
    return r0;
}
template <int DIM, bool F32 = false>
__device__ __forceinline__ double eval_obs(const DevProblem& P, const double* gps, const double* kst,
                                           const double* lst, const double* camd, int o, const ObsIn& in, int cam,
                                           bool gp) {
    double Rwb[9], twb[3];
    const double bf = obs_pose(gps, kst, in, gp, Rwb, twb);
    return eval_obs_at<DIM, F32>(P, Rwb, twb, bf, lst + (size_t)in.lm * 3, camd, o, in, cam);
}

// ------------------------------------------------------------------------------------------------
// GP pose samples: one workgroup (one wave) per GP pair.  The pair quantities (gp_pair_build) and the
// per-sample factor N (gp_sample_build) follow those serial functions' per-output operation order.  A
// wave runs divergent branches one after the other, so every transcendental step is ONE code path for
// every lane that takes it: lane 0 the pair chain (log(T1^-1 T2), Ad(T12^-1), Jr^-1(xi12)), then one
// lane per sample its exp(xi) (pose, and Ad(exp(-xi)) = Ad(exp(xi)^-1)) followed by Jr(xi), then one lane
// per (sample, row, column) of N.  ka / kb: the two KF states (16 doubles each, global or LDS); gps: the
// sample buffer of that state.
constexpr int PREP_THREADS = 64;
constexpr int PREP_SCHUNK = 32;   // samples per pass (one lane each; LDS staging of their Jr / Ad blocks)
// (inlined into k_gp_prep and k_update: a noinline body, one copy for both, measured 4.5 % slower LM
// iterations, profiles/r3e_ab_update_inline_wait.txt; the two copies may round differently in the last bit)
// shm: PREP_SHM doubles of LDS (the caller's, so k_update's roles share one allocation)
constexpr int PREP_PR = (sizeof(GPPair) / sizeof(double) + 1) & ~1;
constexpr int PREP_SHM = PREP_PR + 36 + 36 + 8 + PREP_SCHUNK * (18 + 9 + 9 + 3);
// WT: the sample poses (Rwb, twb) are stored write-through (sc1), for readers in other workgroups of the same
// launch (k_update's fused evaluation)
// pub (optional): called by every thread once the last chunk's sample poses are stored (before their Jacobian
// factors: k_update's fused evaluation reads only the poses), to publish them
struct NoPub {
    __device__ void operator()() const {}
};
template <bool WT = false, typename Pub = NoPub>
__device__ __forceinline__ void gp_pair_prep(const DevProblem& P, double* gps, int i, const double* ka,
                                             const double* kb, int jac, double* shm,
                                             unsigned long long* pst = nullptr, Pub pub = Pub()) {
    GPPair& pr = *reinterpret_cast<GPPair*>(shm);
    double* AdI = shm + PREP_PR;
    double* ad2 = AdI + 36;
    double* vbs = ad2 + 36;
    double(*sJr)[18] = reinterpret_cast<double(*)[18]>(vbs + 8);
    double(*sRm)[9] = reinterpret_cast<double(*)[9]>(sJr + PREP_SCHUNK);
    double(*stR)[9] = sRm + PREP_SCHUNK;
    double(*sg)[3] = reinterpret_cast<double(*)[3]>(stR + PREP_SCHUNK);
    const int tid = threadIdx.x;
    // (diagnostics: pst = s_memrealtime stamps after each phase, thread 0)
#define PREP_STAMP(k) do { if (pst && tid == 0) pst[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
    // the pair's sample range and the first chunk's sample times, loaded before the pair chain (after it they
    // would cost the chain one more memory round trip behind its barriers)
    const int s0 = P.gp_s0[i], s1 = P.gp_s0[i + 1];
    const double t_first = tid < min(PREP_SCHUNK, s1 - s0) ? P.gps_t[s0 + tid] : 0.0;
    if (tid < 6) vbs[tid] = kb[7 + tid];
    if (tid == 0) {
        const SE3 Ta = load_se3(ka), Tb = load_se3(kb);
        pr.T1q[0] = Ta.q.x; pr.T1q[1] = Ta.q.y; pr.T1q[2] = Ta.q.z; pr.T1q[3] = Ta.q.w;
        for (int j = 0; j < 3; ++j) pr.T1t[j] = Ta.t[j];
        for (int j = 0; j < 6; ++j) pr.v1[j] = ka[7 + j];
        pr.t1 = ka[13];
        pr.t2 = kb[13];
        const SE3 T12 = se3_mul(se3_inv(Ta), Tb);
        se3_log(T12, pr.xi12);
        if (jac) se3_adj(se3_inv(T12), AdI);         // Ad(exp(xi12))^-1 = Ad(T12^-1)
        PREP_STAMP(0);
        right_jac_inv(pr.xi12, pr.G2a);                 // C = Jr^-1(xi12)
        if (jac) se3_ad(kb + 7, ad2);
    }
    __syncthreads();
    PREP_STAMP(1);
    if (tid < 6) {                                      // w2 = Jr^-1(xi12) v2
        double w = 0.0;
        for (int l = 0; l < 6; ++l) w += pr.G2a[tid * 6 + l] * vbs[l];
        pr.w2[tid] = w;
    }
    if (jac && tid < 36) {                              // A1 = -C Ad^-1
        const int r = tid / 6, c = tid % 6;
        double v = 0.0;
        for (int l = 0; l < 6; ++l) v += pr.G2a[r * 6 + l] * AdI[l * 6 + c];
        pr.G1a[tid] = -v;
    }
    __syncthreads();
    PREP_STAMP(2);
    if (jac)
        for (int t = tid; t < 72; t += PREP_THREADS) {   // B1 = -1/2 ad(v2) A1, D = -1/2 ad(v2) C
            const int e = t % 36, r = e / 6, c = e % 6;
            const double* src = t < 36 ? pr.G1a : pr.G2a;
            double v = 0.0;
            for (int l = 0; l < 6; ++l) v += ad2[r * 6 + l] * src[l * 6 + c];
            (t < 36 ? pr.G1b : pr.G2b)[e] = v * -0.5;
        }
    __syncthreads();
    PREP_STAMP(3);
    for (int c0 = s0; c0 < s1; c0 += PREP_SCHUNK) {
        const int ns = min(PREP_SCHUNK, s1 - c0);
        // one lane per sample: the interpolated pose T1 exp(xi) (gp_sample_pose), Ad(exp(xi)^-1), Jr(xi)
        double xi[6];
        GPScalars g;
        SE3 E;
        if (tid < ns) {
            GPSample* S = reinterpret_cast<GPSample*>(gps + (size_t)(c0 + tid) * GPS_STRIDE);
            double Rl[9], tl[3];
            gp_sample_pose(pr, c0 == s0 ? t_first : P.gps_t[c0 + tid], Rl, tl, xi, &g, &E);
#pragma unroll
            for (int j = 0; j < 9; ++j) stv<WT>(S->Rwb + j, Rl[j]);
#pragma unroll
            for (int j = 0; j < 3; ++j) stv<WT>(S->twb + j, tl[j]);
        }
        if (c0 + PREP_SCHUNK >= s1) pub();   // (uniform: the last chunk)
        if (tid < ns) {
            if (jac) {
                const SE3 Em = se3_inv(E);                  // Ad(exp(-xi)) = [R', t'^ R'; 0, R']
                double Ht[9];
                qmat(Em.q, sRm[tid]);
                hat3(Em.t, Ht);
                mul33(Ht, sRm[tid], stR[tid]);
                right_jac_blocks(xi, sJr[tid], sJr[tid] + 9);   // Jr(xi) = [Jl, Q; 0, Jl]
                sg[tid][0] = g.l1; sg[tid][1] = g.l2; sg[tid][2] = g.p2;
            }
        }
        __syncthreads();
        PREP_STAMP(4);
        if (jac)
            for (int t = tid; t < ns * 36; t += PREP_THREADS) {   // one (row, column) of each N block
                const int sl = t / 36, r = (t % 36) / 6, c = t % 6;
                const double l1 = sg[sl][0], l2 = sg[sl][1], p2 = sg[sl][2];
                const double* Jl = sJr[sl];
                const double* Qb = sJr[sl] + 9;
                // row r of Jr(xi): [Jl(r), Q(r); 0, Jl(r - 3)]
                auto jr = [&](int l) {
                    if (r < 3) return l < 3 ? Jl[r * 3 + l] : Qb[r * 3 + l - 3];
                    return l < 3 ? 0.0 : Jl[(r - 3) * 3 + l - 3];
                };
                double na = 0.0, nb = 0.0, nc = 0.0;
                for (int l = 0; l < 6; ++l) {
                    const double ma = l1 * pr.G1a[l * 6 + c] + l2 * pr.G1b[l * 6 + c];
                    const double mc = l1 * pr.G2a[l * 6 + c] + l2 * pr.G2b[l * 6 + c];
                    const double j = jr(l);
                    na += j * ma;
                    nb += j * mc;
                    nc += j * pr.G2a[l * 6 + c];
                }
                double ad = 0.0;
                if (r < 3) ad = (c < 3) ? sRm[sl][r * 3 + c] : stR[sl][r * 3 + c - 3];
                else if (c >= 3) ad = sRm[sl][(r - 3) * 3 + c - 3];
                double* N = gps + (size_t)(c0 + sl) * GPS_STRIDE + 12;
                N[c * 6 + r] = na + ad;
                N[(6 + c) * 6 + r] = p2 * jr(c);
                N[(12 + c) * 6 + r] = nb;
                N[(18 + c) * 6 + r] = l2 * nc;
            }
        __syncthreads();
    PREP_STAMP(5);
    }
#undef PREP_STAMP
}

// KF k's pose record (k_depth) and the KF's pose sample (its constant N was uploaded once); WT: the sample
// stored write-through (see gp_pair_prep)
template <bool WT = false>
__device__ __forceinline__ void kf_pose_record(const DevProblem& P, double* gps, int k, const double* kk) {
    double R[9];
    qmat(Quat{kk[0], kk[1], kk[2], kk[3]}, R);
    double* o = P.kfp_pose + (size_t)k * KFP_STRIDE;
    double* so = gps + (size_t)(P.n_gps + k) * GPS_STRIDE;
    for (int j = 0; j < 9; ++j) {
        o[j] = R[j];
        stv<WT>(so + j, R[j]);
    }
    for (int j = 0; j < 3; ++j) {
        o[9 + j] = kk[4 + j];
        stv<WT>(so + 9 + j, kk[4 + j]);
    }
}

// Pose samples of the state `sel`: one workgroup per GP pair, then KF pose records.
__global__ __launch_bounds__(PREP_THREADS) void k_gp_prep(DevProblem P, int sel, int jac, int gate) {
    if (gated_off(P.ctl, gate)) return;
    const int si = state_idx(P, sel);
    const double* __restrict__ kst = P.kbuf[si];
    double* gps = P.gpsb[si];
    if ((int)blockIdx.x < P.n_gp) {
        __shared__ double shm[PREP_SHM];
        const int i = blockIdx.x;
        gp_pair_prep(P, gps, i, kst + (size_t)P.gp_kfa[i] * KF_STRIDE, kst + (size_t)P.gp_kfb[i] * KF_STRIDE, jac, shm);
        return;
    }
    const int k = (blockIdx.x - P.n_gp) * PREP_THREADS + threadIdx.x;
    if (k < P.n_kf) kf_pose_record(P, gps, k, kst + (size_t)k * KF_STRIDE);
}

// One (tile sample, 9-output chunk) task: outputs 9 CH .. 9 CH + 8 of the sample's partial, i.e. the
// upper triangle of M = sum_rows s J1^T J1 (outputs 0..20, row-major) and g = sum_rows s J1^T e
// (21..26), over the sample's contiguous rows.
template <int CH>
__device__ __forceinline__ void smp_task(const DevProblem& P, const double* rows, const double* rw, int r0, int nr,
                                         int mslot) {
    constexpr unsigned char ui[21] = {0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4, 4, 5};
    constexpr unsigned char uj[21] = {0, 1, 2, 3, 4, 5, 1, 2, 3, 4, 5, 2, 3, 4, 5, 3, 4, 5, 4, 5, 5};
    double acc[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) acc[q] = 0.0;
    // (unrolled: the next rows' LDS reads are issued ahead of this row's FMAs; the same order of additions)
#pragma unroll 4
    for (int r = r0; r < r0 + nr; ++r) {
        const double* R = rows + r * ROW_STRIDE;
        const double sw = rw[r];
        double j[7];
#pragma unroll
        for (int c = 0; c < 7; ++c) j[c] = R[c];   // J1 (6), e
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            constexpr int base = 9 * CH;
            const int idx = base + q;
            const double x = idx < 21 ? j[ui[idx < 21 ? idx : 0]] : j[idx - 21];
            const double y = idx < 21 ? j[uj[idx < 21 ? idx : 0]] : j[6];
            acc[q] += (sw * x) * y;
        }
    }
    if (!LBA_INB(P, mslot, P.n_mslots, "mslab")) return;
    double* m = P.mslab + (size_t)mslot * MS_PITCH + 9 * CH;
#pragma unroll
    for (int q = 0; q < 9; ++q) m[q] = acc[q];
}

template <int NT>
__device__ void edge_item(const DevProblem& P, int sel, int idx, const int tid, double* shm);

// ------------------------------------------------------------------------------------------------
// Pose sample s: reduce its M / g partials (fixed slot order) and expand them through the sample's
// Jacobian factor N (6 x 24, columns [KF a pose vel | KF b pose vel]) into Hpp blocks and b_p pieces:
// aa = Na^T M Na, ab = Na^T M Nb, bb = Nb^T M Nb, b_a = -Na^T g, b_b = -Nb^T g, written to the sample's
// slab slots (the same slots / transposition rule as the prior edges).  Equal to summing J^T W J
// per observation row with J = J1 N (base_multi_edge.hpp:170-222) up to rounding.
constexpr int PRI_THREADS = 256;
// partial sums per output of the M / g reduction: k_exp_asm's 576 threads take one (group, output) each; k_expand's
// 256 threads loop over the same (group, output) tasks, so both paths sum in the same order (bitwise the same)
constexpr int EXP_GROUPS = 21;

// A sample of a camera whose extrinsic is free also couples that extrinsic's block e: N is extended by the
// camera's factor [Ad(Tbc) 0] (columns 24..35) and ae, be, ee, b_e follow the same way.
template <bool WT, int NT>
__device__ void sample_expand(const DevProblem& P, const double* gps, const double* camd, int smp, double* Msh,
                              double* Nsh, double* MN, double* part, const int tid) {
    const int* sl = P.seg_slot + SEG_STRIDE * (size_t)smp;
    const int* gl = P.seg_gslot + GSEG_STRIDE * (size_t)smp;
    // N(l, c) at Nsh[6 c + l]: the sample's part loaded with the slot tables (one memory round trip)
    const double* Ng = gps + (size_t)smp * GPS_STRIDE + 12;
    double nv = tid < 144 ? Ng[tid] : 0.0;
    if (sl[0] < 0 && sl[1] < 0 && sl[2] < 0 && sl[6] < 0) return;   // no optimisable vertex (uniform per workgroup)
    const int ncol = sl[6] >= 0 ? 36 : 24;
    if (tid >= 144 && tid < 6 * ncol) nv = camd[(size_t)sl[7] * CAMD_STRIDE + 16 + (tid - 144)];
    // M / g: group q of the EXP_GROUPS sums every EXP_GROUPS-th slot of its output (4 loads in flight), then a
    // fixed combination order over the groups
    const int k1 = P.ms0[smp + 1];
    for (int t = tid; t < EXP_GROUPS * SM_STRIDE; t += NT) {
        const int q = t / SM_STRIDE, o = t - q * SM_STRIDE;
        const double* m = P.mslab + o;
        double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
        int k = P.ms0[smp] + q;
        for (; k + 3 * EXP_GROUPS < k1; k += 4 * EXP_GROUPS) {
            v0 += m[(size_t)k * MS_PITCH];
            v1 += m[(size_t)(k + EXP_GROUPS) * MS_PITCH];
            v2 += m[(size_t)(k + 2 * EXP_GROUPS) * MS_PITCH];
            v3 += m[(size_t)(k + 3 * EXP_GROUPS) * MS_PITCH];
        }
        for (; k < k1; k += EXP_GROUPS) v0 += m[(size_t)k * MS_PITCH];
        part[t] = (v0 + v1) + (v2 + v3);
    }
    if (tid < 6 * ncol) Nsh[tid] = nv;
    __syncthreads();
    if (tid < SM_STRIDE) {
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < EXP_GROUPS; ++q) v += part[q * SM_STRIDE + tid];
        Msh[tid] = v;
    }
    __syncthreads();
    // M (symmetric) from its upper triangle: index of (i, j), i <= j, in row-major upper order
    auto mref = [&](int i, int j) {
        const int a = i < j ? i : j, b = i < j ? j : i;
        return Msh[a * 6 - a * (a - 1) / 2 + (b - a)];
    };
    if (tid < 6 * ncol) {   // MN(l, c) = sum_m M(l, m) N(m, c), stored MN[6 c + l]
        const int t = tid, c = t / 6, l = t % 6;
        double v = 0.0;
#pragma unroll
        for (int m = 0; m < 6; ++m) v += mref(l, m) * Nsh[6 * c + m];
        MN[t] = v;
    }
    __syncthreads();
    // blocks aa, ab, bb, ae, be, ee: column offsets of their row / column vertex in N
    constexpr unsigned char boff_i[6] = {0, 0, 12, 0, 12, 24}, boff_j[6] = {0, 12, 12, 24, 24, 24};
    constexpr unsigned char bslot[6] = {0, 1, 2, 4, 5, 6};
    for (int t = tid; t < (ncol == 36 ? 6 : 3) * 144; t += NT) {
        const int bk = t / 144, ij = t % 144, i = ij / 12, j = ij % 12;
        const int slot = sl[bslot[bk]];
        if (slot < 0) continue;
        const int ci = boff_i[bk] + i, cj = boff_j[bk] + j;
        double v = 0.0;
#pragma unroll
        for (int l = 0; l < 6; ++l) v += Nsh[6 * ci + l] * MN[6 * cj + l];
        double* H = P.hslab + (size_t)slot * 144;
        stv<WT>(H + ((bk == 1 && sl[3]) ? j * 12 + i : i * 12 + j), v);
    }
    if (tid < ncol) {
        const int side = tid / 12, i = tid % 12;
        if (gl[side] >= 0) {
            double v = 0.0;
#pragma unroll
            for (int l = 0; l < 6; ++l) v += Nsh[6 * (12 * side + i) + l] * Msh[21 + l];
            stv<WT>(P.gslab + (size_t)gl[side] * GS_PITCH + i, -v);
        }
    }
}

// Work items of the prior / sample reduction: 0 .. n_prior + n_vel + n_eprior - 1 the EdgeGaussianPrior /
// EdgeVelocity / EdgeExtrinsicPrior quadratic forms (edge_item, NT threads), then one per pose sample
// (sample_expand over the workgroup's threads).  In
// the queued loop the edge items run as extra workgroups of k_linearize and the samples as extra
// workgroups of k_schur (they fill the slots the last tiles leave idle); k_prior_lin runs them all for
// the host-driven paths.  shm: PRI_SHM doubles of LDS.
constexpr int PRI_SHM = 144 + 216 + 216 + 144 + 144 + 12 + 12 + 1 + EXP_GROUPS * SM_STRIDE;
constexpr int EDGE_SHM = 144 * 5 + 12 + 12 + 1;
template <int NT>
__device__ void edge_item(const DevProblem& P, int sel, int idx, const int tid, double* shm) {
    double *Ji = shm, *Jj = Ji + 144, *WJi = Jj + 144, *WJj = WJi + 144, *Om = WJj + 144, *e = Om + 144,
           *We = e + 12, *wshp = We + 12;
    double& wsh = *wshp;
    if (!LBA_INB(P, idx, P.n_prior + P.n_vel + P.n_eprior, "edge item")) return;   // (uniform per workgroup)
    const int si = state_idx(P, sel);
    const double* __restrict__ kst = P.kbuf[si];
    const int ent = P.pri_entry0 + idx;
    const int* sl = P.seg_slot + SEG_STRIDE * (size_t)ent;
    const int* gl = P.seg_gslot + GSEG_STRIDE * (size_t)ent;
    if (idx >= P.n_prior + P.n_vel) {
        // EdgeExtrinsicPrior (unary, 3-d, no robust kernel; include/G2oTypes.h:470-494): J = [0 | Jrot], so
        // H_ee = J^T Om J and b_e = -J^T Om e live in the rotation rows / columns 3..5 of the block
        const int q = idx - P.n_prior - P.n_vel;
        const double* ed = P.ep_data + 16 * (size_t)q;
        if (tid == 0) {
            const double* kx = kst + (size_t)P.ep_kf[q] * KF_STRIDE;
            ext_prior_error_jac(Quat{kx[0], kx[1], kx[2], kx[3]}, Quat{ed[0], ed[1], ed[2], ed[3]}, e, Ji);
            double chi = 0.0;
            for (int i = 0; i < 3; ++i) {
                double s = 0.0;
                for (int k = 0; k < 3; ++k) s += ed[4 + 3 * i + k] * e[k];
                We[i] = s;
                chi += e[i] * s;
            }
            if (LBA_INB(P, P.n_tiles + idx, P.n_chi, "chi_lin")) P.chi_lin[P.n_tiles + idx] = chi;
        }
        __syncthreads();
        if (!LBA_INB(P, sl[2], P.n_hslots, "hslab (extrinsic prior)") ||
            !LBA_INB(P, gl[1], P.n_gslots, "gslab (extrinsic prior)"))
            return;
        double* H = P.hslab + (size_t)sl[2] * 144;
        for (int t = tid; t < 144; t += NT) {
            const int i = t / 12 - 3, j = t % 12 - 3;
            double v = 0.0;
            if (i >= 0 && i < 3 && j >= 0 && j < 3)   // (Jrot^T Om Jrot)(i, j)
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) v += Ji[a * 3 + i] * ed[4 + 3 * a + b] * Ji[b * 3 + j];
            H[t] = v;
        }
        if (tid < 12) {
            double v = 0.0;
            if (tid >= 3 && tid < 6)
                for (int a = 0; a < 3; ++a) v += Ji[a * 3 + tid - 3] * We[a];
            P.gslab[(size_t)gl[1] * GS_PITCH + tid] = -v;
        }
        return;
    }
    if (idx < P.n_prior) {
        if (tid == 0) {
            const double* ka = kst + (size_t)P.pri_a[idx] * KF_STRIDE;
            const double* kb = kst + (size_t)P.pri_b[idx] * KF_STRIDE;
            prior_error_jac(load_se3(ka), ka + 7, ka[13], load_se3(kb), kb + 7, kb[13], e, Ji, Jj);
            qi_inv(P.qcinv, kb[13] - ka[13], Om);
            double chi = 0.0;
            for (int i = 0; i < 12; ++i) {
                double s = 0.0;
                for (int k = 0; k < 12; ++k) s += Om[i * 12 + k] * e[k];
                chi += e[i] * s;
            }
            double r0 = chi, r1 = 1.0;
            if (P.huber_prior > 0) huber(chi, P.huber_prior, &r0, &r1);
            if (LBA_INB(P, P.n_tiles + idx, P.n_chi, "chi_lin")) P.chi_lin[P.n_tiles + idx] = r0;
            wsh = r1;
        }
        __syncthreads();
        const double w1 = wsh;
        for (int t = tid; t < 288; t += NT) {
            const int which = t / 144, ij = t % 144, i = ij / 12, j = ij % 12;
            const double* J = which ? Jj : Ji;
            double s = 0.0;
            for (int k = 0; k < 12; ++k) s += Om[i * 12 + k] * J[k * 12 + j];
            (which ? WJj : WJi)[ij] = w1 * s;
        }
        if (tid < 12) {
            double s = 0.0;
            for (int k = 0; k < 12; ++k) s += Om[tid * 12 + k] * e[k];
            We[tid] = w1 * s;
        }
        __syncthreads();
        // aa = Ji^T W Ji, ab = Ji^T W Jj, bb = Jj^T W Jj, ga/gb = -J^T W e (base_binary_edge.hpp:54-120)
        for (int t = tid; t < 456; t += NT) {
            if (t < 432) {
                const int bk = t / 144, ij = t % 144, i = ij / 12, j = ij % 12;
                const int slot = sl[bk == 0 ? 0 : (bk == 1 ? 1 : 2)];
                if (slot < 0 || !LBA_INB(P, slot, P.n_hslots, "hslab (prior)")) continue;
                const double* A = (bk == 2) ? Jj : Ji;
                const double* B = (bk == 0) ? WJi : WJj;
                double s = 0.0;
                for (int k = 0; k < 12; ++k) s += A[k * 12 + i] * B[k * 12 + j];
                double* H = P.hslab + (size_t)slot * 144;
                if (bk == 1 && sl[3]) H[j * 12 + i] = s;
                else H[i * 12 + j] = s;
            } else {
                const int side = (t - 432) / 12, i = (t - 432) % 12;
                if (gl[side] < 0 || !LBA_INB(P, gl[side], P.n_gslots, "gslab (prior)")) continue;
                const double* A = side ? Jj : Ji;
                double s = 0.0;
                for (int k = 0; k < 12; ++k) s += A[k * 12 + i] * We[k];
                P.gslab[(size_t)gl[side] * GS_PITCH + i] = -s;
            }
        }
    } else {
        // EdgeVelocity: e = Vel(2), J = [0_6, e_2^T], info QcInv(2,2) (include/G2oTypes.h:496-519)
        const int v = idx - P.n_prior;
        const double ev = kst[(size_t)P.vel_kf[v] * KF_STRIDE + 7 + 2];
        const double q22 = P.qcinv[2 * 6 + 2];
        if (!LBA_INB(P, sl[2], P.n_hslots, "hslab (velocity)") || !LBA_INB(P, gl[1], P.n_gslots, "gslab (velocity)") ||
            !LBA_INB(P, P.n_tiles + idx, P.n_chi, "chi_lin"))
            return;
        double* H = P.hslab + (size_t)sl[2] * 144;
        for (int t = tid; t < 144; t += NT) H[t] = (t == 8 * 12 + 8) ? q22 : 0.0;
        if (tid < 12) P.gslab[(size_t)gl[1] * GS_PITCH + tid] = (tid == 8) ? -q22 * ev : 0.0;
        if (tid == 0) P.chi_lin[P.n_tiles + idx] = ev * (q22 * ev);
    }
}

// ------------------------------------------------------------------------------------------------
// Linearisation and landmark elimination of one tile, fused: one workgroup of LS_THREADS threads per
// tile, so the tile's Hpl goes from the linearisation straight into the elimination in LDS (no second
// launch reads it back):
//   1. one observation per lane: residual, Huber weight, rows [J1 e Jp] -> LDS, robust chi2 partial
//   2. per (tile sample, 9-output chunk): the sample's M / g partial -> mslab (J = J1 N, so
//      sum J^T W J = N^T M N per sample, formed by k_expand)
//   3. per (pair, 6-row half): Hpl(k, lm) = sum over its (observation, side) entries of N_side^T G,
//      G = rho' w sum_rows J1^T Jp -> HBM (k_update's back-substitution) and registers
//   4. per landmark: Hll / bl -> HBM; eliminating: Hll + lambda I = L D L^T -> LDS (k_update forms
//      Dinv = (Hll + lambda I)^-1, Eigen's adjugate inverse, block_solver.hpp:389, from Hll)
//   (eliminating regular tiles only; from here on the LDS of the rows holds Hpl)
//   5. W = Hpl L^-T in place
//   6. S partials: per Schur entry (KF pair k1 <= k2 of the tile) C = sum_m W(m,k1) D_m^-1 W(m,k2)^T =
//      sum_m Hpl(m,k1) Dinv_m Hpl(m,k2)^T over the landmarks that see both (fp64 FMAs, 3 x 6 blocks)
//   7. rhs partials per tile KF: sum_m W(m, k) u_m, u = D^-1 L^-1 bl (= sum_m Hpl Dinv bl)
// (1-4: BlockSolver::buildSystem, block_solver.hpp:502-560, with the edges' quadratic forms,
// base_multi_edge.hpp:170-222; 4-7: BlockSolver::solve's Schur loop, block_solver.hpp:381-432.)
// Workgroups after the tiles (LS_EDGES): the motion-prior / velocity / extrinsic-prior quadratic forms
// (edge_item).  Segment tiles of heavy landmarks (tile >= n_stiles) stop after 4; k_expand merges and
// eliminates those landmarks.  With LS_SCHUR the launch also clears the envelope of S for this trial's
// assembly and the factorisation status.
constexpr int LS_THREADS = 256;
constexpr int LS_U = (TILE_PAIRS + 2) * 36;   // doubles: rows + weights while linearising, then Hpl / W
                                              // (+ two zero pairs after the tile's last: what phase 7
                                              // reads for absent (landmark, KF) pairs)
// pidx rows padded by two shorts: a wave's lanes read entry m of up to ~6 different KF rows at once (phase 6's
// tasks, phase 7's), which unpadded all fall on one LDS bank (-30 % bank-conflict cycles, profiles/r5k_*)
constexpr int PIDX_STRIDE = TILE_LMS + 2;
constexpr int DL_STRIDE = 12;   // per landmark in LDS: l10 l21 (l10 l21 - l20) 0 | D^-1 (3) 0 | u (3) 0
static_assert(TILE_ROWS * (ROW_STRIDE + 1) <= LS_U, "the LDS rows alias the Hpl staging");
static_assert(EDGE_SHM <= LS_U, "edge items run in the tile LDS");
static_assert(2 * TILE_PAIRS <= LS_THREADS && TILE_KF * TILE_KF <= LS_THREADS && TILE_SENT <= LS_THREADS &&
                  TILE_LMS <= LS_THREADS && 2 * TILE_SMP <= LS_THREADS && TILE_PROWS <= LS_THREADS,
              "one staging element / Hpl half / KF-pair slot per thread");

// F32: the fp32-residual option (LBA_FLAG_F32_RESIDUAL): phase 1's projection, residuals and Jacobian rows in fp32
template <bool F32>
__global__ __launch_bounds__(LS_THREADS, 3) void k_lin_schur(DevProblem P, int sel, int gate, double lambda_arg,
                                                             int mode) {
    __shared__ double U[LS_U];
    __shared__ double Dl[TILE_LMS * DL_STRIDE];  // per landmark: L^-T terms, D^-1, u = D^-1 L^-1 bl (DL_STRIDE)
    __shared__ int tsm[2 * TILE_SMP];
    __shared__ int osm[TILE_OBS];
    __shared__ int ocam[TILE_OBS];
    __shared__ int orow[TILE_OBS];               // per observation: first LDS row | rows << 16
    __shared__ int prow[TILE_PROWS];
    __shared__ int pr0[TILE_PAIRS + 1];
    __shared__ int lrow[TILE_ROWS];
    __shared__ int lr0[TILE_LMS + 1];
    __shared__ int scode[TILE_SENT];             // Schur entry: tile-local KF l1 | l2 << 8 (l1 <= l2)
    __shared__ int sslt[TILE_SENT];              // its sslab slot
    __shared__ __attribute__((aligned(16))) short pidx[TILE_KF * PIDX_STRIDE];   // [tile KF][landmark]: tile-local pair, npair (a zero pair): none
    __shared__ unsigned char pm[TILE_PAIRS];     // tile-local landmark of a pair
    __shared__ double red[LS_THREADS / 64];
    if (gated_off(P.ctl, gate)) return;
    const int tid = threadIdx.x;
    if (mode & LS_SCHUR) {
        // this trial's assembly starts from a cleared envelope of S (the previous factorisation left its
        // fill-in there) and a cleared factorisation status; k_assemble runs after this launch
        if (blockIdx.x == 0 && tid == 0) {
            *P.info = 0;
            if (P.cf_head) {   // ticket counters of this trial's k_chol_flow (two launches when split)
                P.cf_head[0] = 0;
                P.cf_head[1] = 0;
            }
        }
        const size_t nz = (size_t)P.n_ztiles * CHOL_NB * CHOL_NB;   // (S: the tiles of L)
        for (size_t z = (size_t)blockIdx.x * LS_THREADS + tid; z < nz; z += (size_t)gridDim.x * LS_THREADS) P.S[z] = 0.0;
    }
    if ((int)blockIdx.x >= P.n_tiles) {   // motion-prior / velocity / extrinsic-prior edge items
        edge_item<LS_THREADS>(P, sel, blockIdx.x - P.n_tiles, tid, U);
        return;
    }
    const int tile = P.tile_perm[blockIdx.x];
    const int obs0 = P.tile_obs0[tile], nobs = P.tile_nobs[tile];
    const int ts0 = P.tile_smp0[tile], nts = P.tile_nsmp[tile];
    const int pair0 = P.tile_pair0[tile], npair = P.tile_npair[tile];
    const int lm0 = P.tile_lm0[tile], nlm = P.tile_nlm[tile];
    const bool elim = (mode & LS_SCHUR) && tile < P.n_stiles;
    const int si = state_idx(P, sel);
    const double* __restrict__ kst = P.kbuf[si];
    const double* __restrict__ lst = P.lbuf[si];
    const double* __restrict__ gps = P.gpsb[si];
    const double* __restrict__ camd = P.camdb[si];
    double* rows = U;
    double* rw = U + TILE_ROWS * ROW_STRIDE;
    if (P.tdbg_lin && tid == 0) P.tdbg_lin[(size_t)tile * 16 + 12] = __builtin_amdgcn_s_memrealtime();
    LBA_TMARKI(P.tdbg_lin, tile, 0);

    // ---- stage the tile's index lists in LDS
    {
        const int q0 = P.pair_r0[pair0], nq = P.pair_r0[pair0 + npair] - q0;
        const int m0 = P.lm_r0[lm0], nm = P.lm_r0[lm0 + nlm] - m0;
        if (tid < 2 * nts) tsm[tid] = P.tsm_meta[2 * (size_t)ts0 + tid];
        if (tid < nq) prow[tid] = P.pair_rows[q0 + tid];
#pragma unroll
        for (int k = 0; k < (TILE_ROWS + LS_THREADS - 1) / LS_THREADS; ++k) {
            const int t = tid + k * LS_THREADS;
            if (t < nm) lrow[t] = P.lm_rows[m0 + t];
        }
        if (tid <= npair) pr0[tid] = P.pair_r0[pair0 + tid] - q0;
        if (tid <= nlm) lr0[tid] = P.lm_r0[lm0 + tid] - m0;
        if (elim)
            for (int t = tid; t < PIDX_STRIDE * TILE_KF; t += LS_THREADS) pidx[t] = (short)npair;
    }

    // ---- phase 1: one observation per lane: residual, robust weight, rows [J1 e Jp] -> LDS
    double rho0 = 0.0;
    if (tid < nobs) {
        const int o = obs0 + tid;
        const int meta = P.ob_meta[o], orw = P.ob_row[o];
        const ObsIn in = obs_in(P, o);
        const int kind = meta & 15, cam = meta >> 4;
        const bool gp = kind <= LBA_STEREO_GP;
        osm[tid] = in.smp;
        ocam[tid] = cam;
        const bool st = kind == LBA_STEREO_GP || kind == LBA_STEREO;
        orow[tid] = (orw & 0xffff) | ((st ? 3 : 2) << 16);
        const int wr = (mode & LS_RES) ? 1 : 0;
        rho0 = st ? lin_obs<3, F32>(P, gps, kst, lst, camd, o, in, cam, gp, rows, rw, wr)
                  : lin_obs<2, F32>(P, gps, kst, lst, camd, o, in, cam, gp, rows, rw, wr);
    }
    const double tchi = block_sum<LS_THREADS>(rho0, red);   // (its barrier also publishes rows / lists)
    if (tid == 0) P.chi_lin[tile] = tchi;
    const int nsent = elim ? P.tile_nsent[tile] : 0;
    if (elim) {   // the elimination's tables (the clearing of pidx was ordered by that barrier)
        const int sent0 = P.tile_sent0[tile];
        if (tid < nsent) {
            scode[tid] = P.sent_l1[sent0 + tid] | (P.sent_l2[sent0 + tid] << 8);
            sslt[tid] = P.sslot[sent0 + tid];
        }
        if (tid < npair) {
            const int c = P.pair_lk[pair0 + tid];
            pidx[(c & 255) * PIDX_STRIDE + (c >> 8)] = (short)tid;
            pm[tid] = (unsigned char)(c >> 8);
        }
    }
    LBA_TMARKI(P.tdbg_lin, tile, 1);

    // ---- phase 2: the tile's partial of every pose sample it observes, in the sample's 6-dim space
    for (int task = tid; task < nts * 3; task += LS_THREADS) {
        const int ts = task / 3, ch = task - 3 * ts;
        const int meta = tsm[2 * ts], mslot = tsm[2 * ts + 1];
        const int r0 = meta & 0xffff, nr = meta >> 16;
        if (ch == 0) smp_task<0>(P, rows, rw, r0, nr, mslot);
        else if (ch == 1) smp_task<1>(P, rows, rw, r0, nr, mslot);
        else smp_task<2>(P, rows, rw, r0, nr, mslot);
    }
    LBA_TMARKI(P.tdbg_lin, tile, 2);

    // ---- phase 4: Hll / bl per landmark (threads from the top; before phase 3, so no
    //      register state of phase 3 lives across it); eliminating: Hll + lambda I = L D L^T
    {
        const int t = LS_THREADS - 1 - tid;
        if (t < nlm) {
            const int l = lm0 + t;
            double H[9], b[3];
#pragma unroll
            for (int q = 0; q < 9; ++q) H[q] = 0.0;
            b[0] = b[1] = b[2] = 0.0;
            for (int q = lr0[t]; q < lr0[t + 1]; ++q) {
                const int r = lrow[q];
                const double* Rr = rows + r * ROW_STRIDE;
                const double s = rw[r];
                const double e = Rr[6];
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const double sa = s * Rr[7 + a];
#pragma unroll
                    for (int c = 0; c < 3; ++c) H[a * 3 + c] += sa * Rr[7 + c];
                    b[a] -= sa * e;
                }
            }
            if (LBA_INB(P, l, P.n_lm_all, "Hll / bl")) {
                for (int q = 0; q < 9; ++q) P.Hll[(size_t)l * 9 + q] = H[q];
                for (int q = 0; q < 3; ++q) P.bl[(size_t)l * 3 + q] = b[q];
            }
            if (elim) {
                const double lambda = damping(P, lambda_arg);
                H[0] += lambda; H[4] += lambda; H[8] += lambda;   // setLambda on Hll (block_solver.hpp:580-587)
                // (Dinv = (Hll + lambda I)^-1 for the back-substitution is formed by k_update from Hll: not stored)
                // H = L D L^T (unit lower L)
                const double d0 = H[0], l10 = H[3] / d0, l20 = H[6] / d0;
                const double d1 = H[4] - l10 * l10 * d0;
                const double l21 = (H[7] - l20 * l10 * d0) / d1;
                const double d2 = H[8] - l20 * l20 * d0 - l21 * l21 * d1;
                const double y1 = b[1] - l10 * b[0], y2 = b[2] - l20 * b[0] - l21 * y1;   // L^-1 bl
                double* o = Dl + t * DL_STRIDE;
                o[0] = l10; o[1] = l21; o[2] = l10 * l21 - l20; o[3] = 0.0;
                o[4] = 1.0 / d0; o[5] = 1.0 / d1; o[6] = 1.0 / d2; o[7] = 0.0;
                o[8] = b[0] / d0; o[9] = y1 / d1; o[10] = y2 / d2; o[11] = 0.0;
            }
        }
    }
    LBA_TMARKI(P.tdbg_lin, tile, 3);

    // ---- phase 3: Hpl per (KF, landmark) pair, six rows per thread: the sum over the pair's (observation,
    //      side) entries of N_side^T G (N_side: the 6 x 12 block of the sample's factor for that KF, or for
    //      side 2 the camera's extrinsic factor [Ad(Tbc) 0]); kept in registers until the rows are dead
    double hacc[18];
#pragma unroll
    for (int q = 0; q < 18; ++q) hacc[q] = 0.0;
    const int pl = tid >> 1, half = tid & 1;
    if (pl < npair) {
        for (int q = pr0[pl]; q < pr0[pl + 1]; ++q) {
            const int code = prow[q];
            const int ol = code & 0xffff, side = code >> 16;
            // N stored transposed: column c of N (6 values) at 12 + 6 c
            const double* Nc = side < 2 ? gps + (size_t)osm[ol] * GPS_STRIDE + 12 + 6 * (12 * side + 6 * half)
                                        : camd + (size_t)ocam[ol] * CAMD_STRIDE + 16 + 6 * (6 * half);
            const int r0 = orow[ol] & 0xffff, nrw = orow[ol] >> 16;
            double g[18];   // G = rho' w sum_rows J1^T Jp of the observation, from its LDS rows
#pragma unroll
            for (int u = 0; u < 18; ++u) g[u] = 0.0;
            for (int d = 0; d < nrw; ++d) {
                const double* Rr = rows + (r0 + d) * ROW_STRIDE;
                double jr[9];
#pragma unroll
                for (int u = 0; u < 6; ++u) jr[u] = Rr[u];
#pragma unroll
                for (int u = 0; u < 3; ++u) jr[6 + u] = Rr[7 + u];
#pragma unroll
                for (int l = 0; l < 6; ++l)
#pragma unroll
                    for (int a = 0; a < 3; ++a) g[l * 3 + a] += jr[l] * jr[6 + a];
            }
            const double sw = rw[r0];
#pragma unroll
            for (int u = 0; u < 18; ++u) g[u] *= sw;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double n[6];
#pragma unroll
                for (int l = 0; l < 6; ++l) n[l] = Nc[6 * i + l];
#pragma unroll
                for (int a = 0; a < 3; ++a)
                    hacc[i * 3 + a] = fma(n[5], g[15 + a], fma(n[4], g[12 + a], fma(n[3], g[9 + a],
                                      fma(n[2], g[6 + a], fma(n[1], g[3 + a], fma(n[0], g[a], hacc[i * 3 + a]))))));
            }
        }
        // only the segment tiles of heavy landmarks store their Hpl (k_expand merges them); a regular tile's
        // Hpl lives in LDS until its elimination, and k_update back-substitutes its landmarks in the sample
        // space without it
        if (tile >= P.n_stiles && LBA_INB(P, pair0 + pl - P.hpl_base, P.n_hpl, "Hpl")) {
            double* Hg = P.Hpl + (size_t)(pair0 + pl - P.hpl_base) * 36 + 18 * half;
#pragma unroll
            for (int q = 0; q < 18; ++q) Hg[q] = hacc[q];
        }
    }
    LBA_TMARKI(P.tdbg_lin, tile, 4);

    if (!elim) {
        if (P.tdbg_lin && tid == 0) P.tdbg_lin[(size_t)tile * 16 + 13] = __builtin_amdgcn_s_memrealtime();
        return;
    }
    __syncthreads();   // every read of the rows is done: their LDS takes Hpl
    if (pl < npair) {
        double* h = U + pl * 36 + 18 * half;
#pragma unroll
        for (int q = 0; q < 18; ++q) h[q] = hacc[q];
    }
    if (tid < 72) U[npair * 36 + tid] = 0.0;   // the zero pairs
    __syncthreads();
    LBA_TMARKI(P.tdbg_schur, tile, 0);
    // ---- phase 5: W = Hpl L^-T in place, one (pair, row) per task:
    //      L^-1 = [1 0 0; -l10 1 0; l10 l21 - l20, -l21, 1], w_a = sum_b h_b (L^-1)(a, b)
    for (int task = tid; task < npair * 12; task += LS_THREADS) {
        const int t = task / 12, r = task - 12 * t;
        const double* D = Dl + pm[t] * DL_STRIDE;
        double* h = U + t * 36 + r * 3;
        const double h0 = h[0], h1 = h[1], h2 = h[2];
        h[1] = h1 - D[0] * h0;
        h[2] = h2 - D[1] * h1 + D[2] * h0;
    }
    __syncthreads();
    LBA_TMARKI(P.tdbg_schur, tile, 1);
    // ---- phase 6: S partials, C(k1, k2) = sum over the tile's landmarks m of W(m,k1) D_m^-1 W(m,k2)^T
    //      (Hpl(m,k1) Dinv_m Hpl(m,k2)^T; W(m,k) the zero pair where m does not see k), on the VALU: gfx950
    //      retires fp64 FMAs at ~1.35x its fp64 MFMA rate (scripts/micro/f64_rates.hip) and the VALU form
    //      needs no K padding, zero blocks or padded rows.  One task per (Schur entry, 3-row group,
    //      6-column half) keeps its 3 x 6 block of C in registers; every lane walks the tile's landmarks in
    //      the same order, so a wave's LDS reads of one step hit one landmark's pairs (broadcasts, few
    //      bank conflicts) and D_m^-1 is one broadcast read.  Every entry takes 8 consecutive lanes (a diagonal
    //      entry's rows 6..11 x columns 0..5 too, though never assembled), which store its slot line by line (spos_of)
    const int nkf = P.tile_nkf[tile];
    for (int task = tid; task < nsent * 8; task += LS_THREADS) {
        const int q = task >> 3, rg = (task >> 1) & 3, ch = task & 1;
        const short* p1 = pidx + (scode[q] & 255) * PIDX_STRIDE;
        const short* p2 = pidx + (scode[q] >> 8) * PIDX_STRIDE;
        double acc[18];
#pragma unroll
        for (int u = 0; u < 18; ++u) acc[u] = 0.0;
        for (int m = 0; m < nlm; ++m) {
            const double* A = U + p1[m] * 36 + rg * 9;   // rows 3 rg .. 3 rg + 2 of W(m, k1)
            const double* B = U + p2[m] * 36 + ch * 18;  // rows 6 ch .. 6 ch + 5 of W(m, k2)
            const double* dd = Dl + m * DL_STRIDE + 4;
            double a[9], b[18];
#pragma unroll
            for (int u = 0; u < 9; ++u) a[u] = A[u] * dd[u % 3];
#pragma unroll
            for (int u = 0; u < 18; ++u) b[u] = B[u];
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 6; ++j)
                    acc[i * 6 + j] = fma(a[i * 3 + 2], b[j * 3 + 2],
                                         fma(a[i * 3 + 1], b[j * 3 + 1], fma(a[i * 3], b[j * 3], acc[i * 6 + j])));
        }
        if (!LBA_INB(P, sslt[q], P.n_sslots, "sslab")) continue;
        double* o = P.sslab + (size_t)sslt[q] * 144 + 2 * (task & 7);
#pragma unroll
        for (int k = 0; k < 9; ++k) st16(o + 16 * k, acc[2 * k], acc[2 * k + 1]);
    }
    LBA_TMARKI(P.tdbg_schur, tile, 2);
    // ---- phase 7: rhs partials: sum over the KF's landmarks of V(m,k) bl_m = W(m,k) u_m
    //      (block_solver.hpp:395-401); absent pairs read the zero pair
    {
        const int kf0 = P.tile_kf0[tile];
        for (int task = tid; task < nkf * 12; task += LS_THREADS) {
            const int l = task / 12, r = task - 12 * l;
            const short* pr = pidx + l * PIDX_STRIDE;
            double v0 = 0.0, v1 = 0.0;
            int m = 0;
            for (; m + 2 <= nlm; m += 2) {
                const double* w0 = U + pr[m] * 36 + r * 3;
                const double* w1 = U + pr[m + 1] * 36 + r * 3;
                const double* u0 = Dl + m * DL_STRIDE + 8;
                const double* u1 = u0 + DL_STRIDE;
                v0 = fma(w0[2], u0[2], fma(w0[1], u0[1], fma(w0[0], u0[0], v0)));
                v1 = fma(w1[2], u1[2], fma(w1[1], u1[1], fma(w1[0], u1[0], v1)));
            }
            if (m < nlm) {
                const double* w0 = U + pr[m] * 36 + r * 3;
                const double* u0 = Dl + m * DL_STRIDE + 8;
                v0 = fma(w0[2], u0[2], fma(w0[1], u0[1], fma(w0[0], u0[0], v0)));
            }
            if (LBA_INB(P, P.tkf_gslot[kf0 + l], P.n_gpslots, "gpslab")) P.gpslab[(size_t)P.tkf_gslot[kf0 + l] * GS_PITCH + r] = v0 + v1;
        }
    }
    LBA_TMARKI(P.tdbg_schur, tile, 3);
    if (P.tdbg_lin && tid == 0) P.tdbg_lin[(size_t)tile * 16 + 13] = __builtin_amdgcn_s_memrealtime();
}

// One heavy landmark (k_expand work item, PRI_THREADS threads): its segments' partials summed in a fixed
// order into the landmark's Hll, bl and canonical Hpl blocks (what k_update and the host paths read);
// eliminating, Dinv = (Hll + lambda I)^-1, V = Hpl Dinv, the rhs partial V bl of each of its KFs and the
// S partial V(a) Hpl(b)^T of each pair of its KFs (block_solver.hpp:381-432: any number of KFs, like
// g2o's Hpl columns).  shm: 21 doubles.
template <bool WT>
__device__ void heavy_item(const DevProblem& P, int h, double lambda, int schur, double* shm) {
    const int tid = threadIdx.x;
    const int l = P.hv_lm[h], s0 = P.hv_seg0[h], s1 = P.hv_seg0[h + 1];
    const int hp0 = P.hv_hp0[h], nhp = P.hv_hp0[h + 1] - hp0, cp0 = P.lm_pair0[l];
    double* HB = shm;   // Hll (9), bl (3), Dinv (9)
    if (tid < 12) {
        double v = 0.0;
        for (int s = s0; s < s1; ++s)
            v += tid < 9 ? P.Hll[(size_t)(P.n_lm + s) * 9 + tid] : P.bl[(size_t)(P.n_lm + s) * 3 + tid - 9];
        HB[tid] = v;
        if (tid < 9) P.Hll[(size_t)l * 9 + tid] = v;
        else P.bl[(size_t)l * 3 + tid - 9] = v;
    }
    double* const Hpl = P.Hpl - (size_t)P.hpl_base * 36;   // (pair index -> Hpl slot: only heavy pairs are stored)
    for (int t = tid; t < nhp * 36; t += PRI_THREADS) {
        const int j = t / 36, e = t - 36 * j;
        double v = 0.0;
        for (int q = P.hp_src0[hp0 + j]; q < P.hp_src0[hp0 + j + 1]; ++q) v += Hpl[(size_t)P.hp_src[q] * 36 + e];
        Hpl[(size_t)(cp0 + j) * 36 + e] = v;
    }
    if (!schur) return;
    __syncthreads();
    if (tid == 0) {
        double Hd[9];
        for (int q = 0; q < 9; ++q) Hd[q] = HB[q];
        Hd[0] += lambda; Hd[4] += lambda; Hd[8] += lambda;   // setLambda (block_solver.hpp:580-587)
        inv3(Hd, HB + 12);
        for (int q = 0; q < 9; ++q) P.Dinv[(size_t)l * 9 + q] = HB[12 + q];
    }
    __syncthreads();
    const double* Di = HB + 12;
    for (int t = tid; t < nhp * 12; t += PRI_THREADS) {   // V = Hpl Dinv and the rhs partial V bl
        const int j = t / 12, r = t - 12 * j;
        const double* hr = Hpl + (size_t)(cp0 + j) * 36 + r * 3;
        double* vr = P.Vh + (size_t)(hp0 + j) * 36 + r * 3;
        double g = 0.0;
        for (int a = 0; a < 3; ++a) {
            const double v = hr[0] * Di[a] + hr[1] * Di[3 + a] + hr[2] * Di[6 + a];
            vr[a] = v;
            g += v * HB[9 + a];
        }
        stv<WT>(P.gpslab + (size_t)P.hp_gslot[hp0 + j] * GS_PITCH + r, g);
    }
    __syncthreads();
    const int np2 = nhp * (nhp + 1) / 2, ss0 = P.hv_ss0[h];
    for (int t = tid; t < np2 * 144; t += PRI_THREADS) {   // the S partial of KF pair (a <= b): V(a) Hpl(b)^T
        const int pp = t / 144, e = t - 144 * pp, i = e / 12, jj = e - 12 * i;
        int a = 0, rem = pp;
        while (rem >= nhp - a) { rem -= nhp - a; ++a; }
        const double* v = P.Vh + (size_t)(hp0 + a) * 36 + i * 3;
        const double* hb = Hpl + (size_t)(cp0 + a + rem) * 36 + jj * 3;
        stv<WT>(P.sslab + (size_t)P.hv_sslot[ss0 + pp] * 144 + spos_of(i, jj), v[0] * hb[0] + v[1] * hb[1] + v[2] * hb[2]);
    }
}

// After k_lin_schur: workgroups [0, n_smp) expand the pose samples' M / g partials through their factors
// N into Hpp blocks and b_p pieces (sample_expand); [n_smp, n_smp + n_heavy) the heavy landmarks
// (heavy_item: the merge of their segments, and with schur their elimination)
__global__ __launch_bounds__(PRI_THREADS) void k_expand(DevProblem P, int sel, int gate, double lambda_arg, int schur) {
    __shared__ double shm[PRI_SHM];
    if (gated_off(P.ctl, gate)) return;
    if ((int)blockIdx.x < P.n_smp) {
        const int si = state_idx(P, sel);
        double *Msh = shm, *Nsh = Msh + 144, *MN = Nsh + 216, *part = MN + 216;
        sample_expand<false, PRI_THREADS>(P, P.gpsb[si], P.camdb[si], blockIdx.x, Msh, Nsh, MN, part, threadIdx.x);
        return;
    }
    heavy_item<false>(P, blockIdx.x - P.n_smp, schur ? damping(P, lambda_arg) : 0.0, schur, shm);
}

// Reduced camera system of one trial, straight from the target-sorted partial slabs (each
// output block sums one contiguous range, so the reads are coalesced and the order is fixed):
//   S(bi, bj) = sum Hpp partials + lambda I (diagonal) - sum Schur partials   (block_solver.hpp:432-445,
//   setLambda :573-579), only for the blocks inside the structural pattern (the rest of S is zero
//   from the upload and never written);  b_p = sum b partials;  bS = b_p - sum Schur rhs partials.
// sum of x[(s0 + G q) * W + e] over the slots s0, s0 + G, ... < s1: four loads in flight, combined in
// a fixed order
// whether this rank adds the once-per-system terms of natural row r (damping, padding identity, computeScale):
// its owner in the distributed factorisation, rank 0 for a row every rank holds
__device__ __forceinline__ bool row_adds(const DevProblem& P, int r) {
    const int o = P.row_own ? P.row_own[r] : -1;
    return o == P.part_rank || (o < 0 && P.part_rank == 0);
}

template <int G, int W, bool SC = false>
__device__ __forceinline__ double slot_sum(const double* __restrict__ x, int s0, int s1, int e) {
    double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
    int s = s0;
    for (; s + 3 * G < s1; s += 4 * G) {
        v0 += ldv<SC>(x + (size_t)s * W + e);
        v1 += ldv<SC>(x + (size_t)(s + G) * W + e);
        v2 += ldv<SC>(x + (size_t)(s + 2 * G) * W + e);
        v3 += ldv<SC>(x + (size_t)(s + 3 * G) * W + e);
    }
    for (; s < s1; s += G) v0 += ldv<SC>(x + (size_t)s * W + e);
    return (v0 + v1) + (v2 + v3);
}

// (fused expansion + assembly) wait until the pose samples that write the slots [s0, s1) of a target (prod_of: the
// sample of each slot, < 0: written by an earlier launch) have published this launch's epoch; bounded, as
// k_chol_flow's waits
__device__ __forceinline__ void exp_wait(const DevProblem& P, const int* prod_of, int s0, int s1, unsigned epoch) {
    for (int s = s0 + (int)threadIdx.x; s < s1; s += (int)blockDim.x) {
        const int q = prod_of[s];
        if (q < 0) continue;
        unsigned spins = 0;
        while ((unsigned)__hip_atomic_load((gi32_t*)(P.exp_flag + (size_t)FLAG_STRIDE * q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1u << 20)) {   // (~0.5 s: never expected) the slots may be stale: the call fails
                __hip_atomic_fetch_or((gi32_t*)P.fault, FAULT_EXP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
}

// One output of the assembly: S block asm_list[item] (item < n_asm) or the rhs of pose block item - n_asm.
// FUSED (k_exp_asm): the Hpp / b_p partials come from expansion workgroups of the same launch, so the Schur
// partials (an earlier launch's) are summed first, then the block waits for its samples (wait: the launch is not
// gated off) and sums theirs -- the same operations in the same order as k_assemble, so S / bS are bitwise its.
// The hand-off is MI355X_MICROARCH.md's sc1 form: the expansions store every Hpp / b_p piece write-through, drain
// and set their flag; the blocks poll the flags and load every piece with sc1 loads (hslab and gslab slots fill
// whole cache lines of their own).  An agent-scope acquire after the wait instead of the sc1 loads (here and in
// k_update's upd_wait) cost 1.5-11 us per LM iteration (profiles/r7j_ab_acquire_rejected.txt).
template <bool FUSED>
__device__ __forceinline__ void assemble_item(const DevProblem& P, int item, double lambda, int flags, double* red, bool wait,
                                              unsigned epoch, unsigned long long* xs = nullptr) {
    const int tid = threadIdx.x;
    const int n = P.npad;   // leading dimension of S
    if (item < P.n_asm) {
        const int ub = P.asm_list[item];
        const int bi = P.ub_i[ub], bj = P.ub_j[ub];
        // lane (e, g): slot position e of the Schur partials, the same element's row-major position eh of the Hpp ones
        const int e = tid % 144, g = tid / 144, rc = spos_rc(e), eh = 12 * (rc >> 4) + (rc & 15);
        double v;
        if constexpr (FUSED) {
            const double sv = slot_sum<RED_GROUPS, 144>(P.sslab, P.ss0[ub] + g, P.ss0[ub + 1], e);
            if (xs) xs[1] = __builtin_amdgcn_s_memrealtime() + (sv != sv);   // (diagnostics: the partials are in)
            if (wait) exp_wait(P, P.hs_prod, P.hs0[ub], P.hs0[ub + 1], epoch);
            if (xs) xs[2] = __builtin_amdgcn_s_memrealtime();
            v = slot_sum<RED_GROUPS, 144, true>(P.hslab, P.hs0[ub] + g, P.hs0[ub + 1], eh);
            v -= sv;
        } else {
            v = slot_sum<RED_GROUPS, 144>(P.hslab, P.hs0[ub] + g, P.hs0[ub + 1], eh);
            if (flags & ASM_SCHUR) v -= slot_sum<RED_GROUPS, 144>(P.sslab, P.ss0[ub] + g, P.ss0[ub + 1], e);
        }
        red[tid] = v;
        __syncthreads();
        if (g == 0) {
            double t = red[e];
#pragma unroll
            for (int q = 1; q < RED_GROUPS; ++q) t += red[144 * q + e];   // (4 groups: ((a + b) + c) + d)
            const int i = rc >> 4, j = rc & 15;
            const int r = 12 * bj + j, c = 12 * bi + i;   // element (row r, col c) of S, r >= c in blocks
            if (bi == bj && i == j && row_adds(P, r)) t += lambda;   // damping: added once over the ranks
            if (flags & ASM_FULL) {                       // natural order, both triangles (dense np x np)
                P.Sfull[(size_t)r * P.np + c] = t;
                P.Sfull[(size_t)c * P.np + r] = t;
            } else if (flags & ASM_DIAG) {                // the natural diagonal only (computeLambdaInit)
                if (bi == bj && i == j) P.Sdiag[r] = t;
            } else if (bi != bj || j >= i) {               // factorisation order, lower triangle: one
                // write per unordered pair (the natural-lower entry; a diagonal block's partial sums
                // are not bitwise symmetric, so writing both would race)
                const int rh = P.rpos[r], ch = P.rpos[c];
                P.S[s_elem(P, max(rh, ch), min(rh, ch))] = t;
            }
        }
        if ((flags & ASM_SCHUR) && item == 0)   // padding rows: identity (their owner)
            for (int r = P.np + tid; r < n; r += 144 * RED_GROUPS) {
                if (!row_adds(P, r)) continue;
                const int rh = P.rpos[r];
                P.S[s_elem(P, rh, rh)] = 1.0;
                P.bS[rh] = 0.0;
            }
    } else {
        const int k = item - P.n_asm;
        constexpr int RG = 12 * RED_GROUPS;   // (48 groups of 12 threads)
        const int e = tid % 12, g = tid / 12;
        double v, w;
        if constexpr (FUSED) {
            w = slot_sum<RG, GS_PITCH>(P.gpslab, P.gps0[k] + g, P.gps0[k + 1], e);
            if (wait) exp_wait(P, P.gs_prod, P.gs0[k], P.gs0[k + 1], epoch);
            v = slot_sum<RG, GS_PITCH, true>(P.gslab, P.gs0[k] + g, P.gs0[k + 1], e);
        } else {
            v = slot_sum<RG, GS_PITCH>(P.gslab, P.gs0[k] + g, P.gs0[k + 1], e);
            w = (flags & ASM_SCHUR) ? slot_sum<RG, GS_PITCH>(P.gpslab, P.gps0[k] + g, P.gps0[k + 1], e) : 0.0;
        }
        red[tid] = v;
        __syncthreads();
        double bpv = 0.0;
        if (tid < 12) {
            for (int q = 0; q < RG; ++q) bpv += red[q * 12 + tid];
            P.bp[12 * k + tid] = bpv;
        }
        __syncthreads();
        red[tid] = w;
        __syncthreads();
        if (tid < 12) {
            double t = 0.0;
            for (int q = 0; q < RG; ++q) t += red[q * 12 + tid];
            const int r = 12 * k + tid;
            const int rh = (flags & ASM_FULL) ? r : P.rpos[r];
            P.bS[rh] = bpv - t;   // bS = b_p - sum Hpl Dinv bl (factorisation order)
        }
    }
}

__global__ __launch_bounds__(144 * RED_GROUPS) void k_assemble(DevProblem P, double lambda_arg, int flags, int gate) {
    __shared__ double red[144 * RED_GROUPS];
    if (gated_off(P.ctl, gate)) return;
    assemble_item<false>(P, blockIdx.x, damping(P, lambda_arg), flags, red, false, 0);
}

// k_expand's sample expansions and k_assemble's outputs of a trial in one launch (P.fuse_asm: no heavy landmarks,
// not partitioned): workgroups [0, n_smp) expand a pose sample each (sample_expand, all 576 threads),
// store its Hpp / b_p pieces write-through and publish the launch's epoch in exp_flag; the assembly workgroups
// after them sum their Schur partials meanwhile and then wait for just the samples their slots come from.  The
// expansions are the lowest workgroup ids (dispatched first).  gate: the expansions' (k_expand's) gate -- when it
// holds the launch off, the assembly still runs (as k_assemble does, on scratch) without waiting.
__global__ __launch_bounds__(144 * RED_GROUPS) void k_exp_asm(DevProblem P, int sel, int gate, double lambda_arg, unsigned epoch) {
    constexpr int SHM = PRI_SHM > 144 * RED_GROUPS ? PRI_SHM : 144 * RED_GROUPS;
    __shared__ double shm[SHM];
    const bool off = gated_off(P.ctl, gate);
    const int tid = threadIdx.x;
    // diagnostics (LBA_PHASE_TIMING): s_memrealtime stamps in slots 8.. of the sweep's elimination stamp rows
    // (expansions: start / expanded / published; assembly blocks: start / partials in / samples in / stored)
    unsigned long long* xs = (P.tdbg_schur && tid == 0 && (int)blockIdx.x < P.n_tiles && !off)
                                 ? P.tdbg_schur + (size_t)blockIdx.x * 16 + 8 : nullptr;
    if (xs) xs[0] = __builtin_amdgcn_s_memrealtime();
    if ((int)blockIdx.x < P.n_smp) {
        if (off) return;
        const int si = state_idx(P, sel);
        double *Msh = shm, *Nsh = Msh + 144, *MN = Nsh + 216, *part = MN + 216;
        sample_expand<true, 144 * RED_GROUPS>(P, P.gpsb[si], P.camdb[si], blockIdx.x, Msh, Nsh, MN, part, tid);
        if (xs) xs[1] = __builtin_amdgcn_s_memrealtime();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store((gi32_t*)(P.exp_flag + (size_t)FLAG_STRIDE * blockIdx.x), (int)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (xs) xs[2] = __builtin_amdgcn_s_memrealtime();
        return;
    }
    assemble_item<true>(P, blockIdx.x - P.n_smp, damping(P, lambda_arg), ASM_SCHUR, shm, !off, epoch, xs);
    if (xs) xs[3] = __builtin_amdgcn_s_memrealtime();
}

// ------------------------------------------------------------------------------------------------
// Dense Cholesky S = L L^T of the reduced camera system in its factorisation order (panels permuted
// by the nested dissection of lba_plan.hpp), as ONE dataflow launch (k_chol_flow below).  S and L are
// stored as the tiles of L's symbolic structure (fill-in included): tile t is 32 x 32 doubles row-major at
// t * 1024, the host precomputes every tile id a task touches (memory O(nnz(L)), not npad^2).  The
// system is padded to a multiple of CNB with an identity tail, so every panel is exactly CNB wide and
// the panel code below is compile-time.  A non-positive pivot sets *info (the LDLT !isPositive failure
// of linear_solver_dense.h:108-112).
constexpr int CNB = CHOL_NB;

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, lane);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// empty asm that "modifies" v: forces an update to be materialised where it is written (stops the
// compiler from sinking a rank-1 update down to its first use, which keeps O(n^2) operands live)
__device__ __forceinline__ void pin(double& v) { asm volatile("" : "+v"(v)); }

// 1/sqrt(d): hardware estimate (5e-8 relative) + one cubically convergent step
// r' = r + r e (1/2 + 3/8 e), e = 1 - d r^2: 0.62 ulp worst case over 2^20 samples, against 1.08 ulp for
// two Newton steps, at four dependent operations instead of six (scripts/micro/rsq_accuracy.hip)
__device__ __forceinline__ double rsqrt_nr(double d) {
    const double r = __builtin_amdgcn_rsq(d);
    const double e = fma(-(d * r), r, 1.0);
    return fma(r * e, fma(0.375, e, 0.5), r);
}

// lane x <- v of lane B + (x & 15): the pivot column of one 16-row half of the diagonal block copied
// into every 16-lane row of the wave, so the rank-1 update can read entry k with the DPP64 row
// broadcast (row_newbcast: each lane of a row takes lane k & 15 of that row)
template <int B>
__device__ __forceinline__ double rep16(double v, int lane) {
    const int addr = (B + (lane & 15)) << 2;
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(addr, (int)(unsigned)u);
    const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(addr, (int)(unsigned)(u >> 32));
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}
// acc = fma(-rep[lane of this row with index K & 15], l, acc): one v_fmac_f64 with a DPP64 operand, the same
// rounding as fma(-l, cb[K], acc) from a readlane broadcast (two v_readlane_b32 fewer per entry)
template <int K>
__device__ __forceinline__ void fmac_bcast(double& acc, double rep, double l) {
    asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(rep), "v"(l), "i"(K & 15));
}

// Panel pivot sequence over the columns [J, E) of one 16-column half, generated at compile time so every row[]
// index is a constant: pivot J: l = row[J] r (r = 1/sqrt of the pivot); column J by broadcast; the rank-1 update
// row[k] -= l L(k, J) (J < k < E).  The panel is factored as two halves (piv_pipe<0, 16>, cross_update on the
// matrix cores, piv_pipe<16, 32>), so the broadcasts cover 2 x 120 entries instead of 496.  The sequence is
// software-pipelined across pivots (round 2's unpipelined reference form gave bitwise these results): the chain of
// pivot J (the next pivot's diagonal, its reciprocal square root, the broadcast) is issued first, and the
// rank-1 updates of pivot J - 1 on columns J + 1 .. E - 1 are interleaved into it, so the chain no longer waits
// behind the DPP updates (which wait for their ds_bpermute broadcast, ~80 cycles) nor they behind the chain.
// Column J + 1, the next pivot's, takes pivot J's update through a readlane broadcast right away.  The
// diagonal the chain needs is tracked per lane (dg: the same fma sequence the lane's own diagonal entry
// receives), so it never waits for a deferred update.  Every column still receives its updates one fma at a
// time in pivot order.  Non-positive pivots show as a non-positive (or NaN) diagonal of L (see factor).
template <int J, int E, int S>
__device__ __forceinline__ void pipe_defer(double (&row)[CNB], double rp, double lp) {
    // deferred update slot S of pivot J - 1: columns J + 1 + S*ND/5 .. J + 1 + (S+1)*ND/5 - 1
    constexpr int B = E - 16;
    constexpr int ND = J > B ? E - 1 - J : 0;
#pragma unroll
    for (int t = (S * ND) / 5; t < ((S + 1) * ND) / 5; ++t) {
        switch (J + 1 + t) {   // (constant after unrolling: the DPP lane select is an immediate)
#define LBA_PD(K) case K: fmac_bcast<K>(row[K], rp, lp); break;
            LBA_PD(1) LBA_PD(2) LBA_PD(3) LBA_PD(4) LBA_PD(5) LBA_PD(6) LBA_PD(7) LBA_PD(8) LBA_PD(9) LBA_PD(10)
            LBA_PD(11) LBA_PD(12) LBA_PD(13) LBA_PD(14) LBA_PD(15) LBA_PD(16) LBA_PD(17) LBA_PD(18) LBA_PD(19)
            LBA_PD(20) LBA_PD(21) LBA_PD(22) LBA_PD(23) LBA_PD(24) LBA_PD(25) LBA_PD(26) LBA_PD(27) LBA_PD(28)
            LBA_PD(29) LBA_PD(30) LBA_PD(31)
#undef LBA_PD
            default: break;
        }
    }
}
template <int J, int E>
__device__ __forceinline__ void piv_pipe(double (&row)[CNB], double rn, double dg, double lp, double rp, int lane) {
    constexpr int B = E - 16;
    if constexpr (J < E) {
        const double lij = row[J] * rn;   // lane J: sqrt(d); lanes > J: L(l, J)
        row[J] = lij;
        if constexpr (J + 1 < E) {
            const double own = dg - lij * lij;       // lane J + 1: the next pivot
            const double dgn = fma(-lij, lij, dg);   // the lane's own diagonal entry after this pivot's update
            double rep = 0.0;
            if constexpr (J + 2 < E) rep = rep16<B>(lij, lane);
            // (the scheduler would sink the ds_bpermute down to its first use, the deferred updates of the
            // next window, and stall the chain there on its ~80-cycle return: keep it here)
            __builtin_amdgcn_sched_barrier(0);
            const double sL = readlane_d(lij, J + 1);
            double c = __builtin_amdgcn_rsq(own);
            pin(c);
            pipe_defer<J, E, 0>(row, rp, lp);
            double t = own * c;
            pin(t);
            pipe_defer<J, E, 1>(row, rp, lp);
            double e = fma(-t, c, 1.0);
            pin(e);
            pipe_defer<J, E, 2>(row, rp, lp);
            t = fma(0.375, e, 0.5);
            const double m = c * e;
            pin(t);
            pipe_defer<J, E, 3>(row, rp, lp);
            c = fma(m, t, c);
            pin(c);
            pipe_defer<J, E, 4>(row, rp, lp);
            row[J + 1] = fma(-lij, sL, row[J + 1]);   // = fmac(-L(J+1, J), lij): the first update of column J + 1
            const double rnn = readlane_d(c, J + 1);
            piv_pipe<J + 1, E>(row, rnn, dgn, lij, rep, lane);
        }
    }
}

// Between the halves: every stacked row's columns 16..31 -= (its columns 0..15) (rows 16..31's
// columns 0..15)^T, i.e. A22 -= L21 L21^T and the tile rows' share, as 3 row tiles (rows 16..63) x 4 k-steps of
// v_mfma_f64_16x16x4 on the wave's LDS staging buffer (columns 0..15 in, the product out through
// columns 16..31).  Rows 0..15 get no product: their columns 16..31 lie above the diagonal of L_jj, which no
// reader takes (L_jj is stored masked), and the second half's pivots never read lanes 0..15.  An fp64 MFMA holds
// its wave ≈75 cycles, so the fourth row tile cost ≈340 of the factor's ≈6.9k cycles (scripts/micro/factor_stages.hip;
// issuing the k-steps inside the first half's pivots, or on a helper wave, gained nothing more:
// profiles/r6b_factor_stages.txt).
__device__ __forceinline__ void cross_update(double (&row)[CNB], double (*st)[CNB + 1], int lane, double dg0 = 0.0,
                                             double* dg2 = nullptr) {
#pragma unroll
    for (int c = 0; c < 16; ++c) st[lane][c] = row[c];
    wave_sync();
    const int lr = lane & 15, kq = lane >> 4;
    d4 acc[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        const double bv = st[16 + lr][4 * ks + kq];
#pragma unroll
        for (int t = 0; t < 3; ++t)
            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(st[16 * (t + 1) + lr][4 * ks + kq], bv, acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) st[16 * (t + 1) + kq + 4 * q][16 + lr] = acc[t][q];
    wave_sync();
    // (lanes 16..31: the diagonal entry after the update, for piv_pipe's tracking; the first half did not
    // touch columns 16..31, so it is the original entry minus the product, as row[lane] below)
    if (dg2) *dg2 = dg0 - st[lane][lane & 31];
#pragma unroll
    for (int c = 0; c < 16; ++c) row[16 + c] -= st[lane][16 + c];
}

// The stacked panel in `st` (rows 0..31 the diagonal block) factored by ONE wave: piv_pipe over the two
// halves with the matrix-core cross update between them.  bad: a non-positive (or NaN) pivot, seen as a diagonal entry of L that is not > 0 (a pivot
// d <= 0 or NaN gives rsq(d) = NaN / inf, so L(J, J) = NaN; d > 0 gives L(J, J) = d rsq(d) > 0).
__device__ __forceinline__ void factor_pipe(double (*st)[CNB + 1], int lane, bool& bad) {
    double row[CNB];
#pragma unroll
    for (int c = 0; c < CNB; ++c) row[c] = st[lane][c];
    const double dg0 = st[lane][lane & 31];
    piv_pipe<0, 16>(row, readlane_d(rsqrt_nr(row[0]), 0), dg0, 0.0, 0.0, lane);
    double dg2 = 0.0;
    cross_update(row, st, lane, dg0, &dg2);
    piv_pipe<16, CNB>(row, readlane_d(rsqrt_nr(row[16]), 16), dg2, 0.0, 0.0, lane);
#pragma unroll
    for (int c = 0; c < CNB; ++c) st[lane][c] = row[c];
    wave_sync();
    bad = lane < CNB && !(st[lane][lane & 31] > 0.0);
}

// ------------------------------------------------------------------------------------------------
// Dataflow factorisation of the permuted system in ONE launch.
// One task per tile of the envelope, in a topological order (column by column) pulled from a ticket
// counter, so progress never depends on which workgroups are resident or in what order they start:
//   tile (i, j), i > j: keeps A(i, j) and its own copy of A(j, j) in registers (the
//     v_mfma_f64_16x16x4 output layout, one 16 x 16 quadrant per wave); for every envelope panel
//     p < j it waits for L(j, p) (and L(i, p) where row i reaches p) and applies
//     A(i,j) -= L(i,p) L(j,p)^T, A(j,j) -= L(j,p) L(j,p)^T; then one wave factors the stacked
//     [A(j,j); A(i,j)] (the two-level pivot sequence above) and L(i, j) is published.  The
//     copies of A(j, j) see the same updates in the same order, so they are bitwise identical;
//   panel j (i = j): the same updates of A(j, j) and b_j -= L(j,p) y_p, then [A_jj; b_j^T] -> L_jj,
//     y_j and [A_jj; I] -> L_jj^-T on two waves, published for the diagonal tasks below it.
// The chain from one panel to the next is one hand-off, the last update and one factorisation.
constexpr unsigned CF_SPIN_LIMIT = 1u << 22;   // ~0.5 s of polling before giving up (never expected)
constexpr int CF_TIMEOUT = 0x7fff0000;          // *info value of a timed-out launch

struct CholFlow {
    int n, NP, ntasks;
    unsigned epoch;
    const int* task_i;   // per task: i
    const int* tasks;    // j | kind << 24 | lookahead << 28 (0: factor tile (i, j) (i = j: panel j), 1: L^-1 tile (i, j),
                         // 2: solution block x_j, 3: forward block y_i, 4 / 5: band forward / back substitution,
                         // 6 / 7: a subtree's contribution to a top tile / top rhs block (distributed factorisation))
    const int* task_t;   // per task: 5 tile ids (factor tasks: (j,j), (i,j), (k,k), (j,k), (i,k); -1 none)
    const int* plist_t;  // per list entry: 3 tile ids (factor: (j,p), (i,p), (k,p); L^-1 / forward: (i,k); back: (i,j))
    const int* pl0;      // per task: first entry of its update list in plist ([pl0[t], pl0[t+1]))
    const int* plist;    // p | (row i takes part) << 24, in the order every task applies panel updates
                         // (the order panels finish: left k and right k side by side, then the separator)
    const double* S;     // assembled system (factorisation order, lower)
    double* Lm;
    double* LinvT;
    const double* b;     // right-hand side (factorisation order)
    double* yv;
    int* info;
    int* lready;         // per tile: epoch once L(i, j) is published
    int* fready;         // per panel: epoch once L_jj^-T is published
    int* dready;         // per panel: epoch once y_i is published (after every Linv(i, .))
    int* zready;         // per panel: epoch once z(i, i) = L_ii^-1 b_i is published
    double* zv;          // [NP][NP][CNB] z(i, k) = Linv(i, k) b_k, the shares of y_i
    unsigned long long* head;   // ticket counter (zeroed by k_schur ahead of every trial)
    int* abort_flag;
    int* fault;                 // DevProblem::fault: a timed-out wait also fails the call (FAULT_FLOW)
    unsigned long long* tdbg;   // diagnostics: per panel, s_memrealtime stamps of its task
    unsigned long long* tdbg2;  // diagnostics: stamps of the L^-1 tasks of the last two panel rows
    unsigned long long* tdbg3;  // diagnostics: per factor task (ticket < 4096): stamps, i, j
    // the solve x = L^-T y without a back-substitution chain: L^-1 tiles (computed alongside the
    // factorisation) and per output panel one GEMV
    double* Linv;        // [npad][npad] tiles (i, j), i > j, of L^-1 (factorisation order)
    int* ivready;        // per lower tile (tri_id): epoch once Linv(i, j) is published
    double* xout;        // the solution, natural order
    const int* rnat;     // natural row of a factorisation row
    // band mode (kinds 4, 5): forward / back substitution tasks instead of L^-1 tiles
    unsigned long long* xg;   // [2 npad] x in factorisation order, handed off between back tasks as 8-byte granules
                              // {epoch << 32 | one half of a double}: the data is its own flag
};

// lanes 0..2 of wave 0 poll up to three flags (null = none) for `epoch` side by side (relaxed, agent
// scope: one round trip when they are already set, not one per flag); the workgroup learns the result
__device__ __forceinline__ bool cf_wait(const CholFlow& a, const int* f1, const int* f2, int* s_ok,
                                        const int* f3 = nullptr) {
    if (threadIdx.x < 64) {
        const int l = threadIdx.x;
        const int* f = l == 0 ? f1 : (l == 1 ? f2 : (l == 2 ? f3 : nullptr));
        bool done = f == nullptr;
        bool ok = true;
        for (unsigned spins = 0;; ++spins) {
            if (!done) done = (unsigned)__hip_atomic_load((gi32_t*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.epoch;
            if (__all(done)) break;
            if (spins > CF_SPIN_LIMIT ||
                ((spins & 255) == 255 &&
                 (unsigned)__hip_atomic_load((gi32_t*)a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.epoch)) {
                if (l == 0) {
                    __hip_atomic_store((gi32_t*)a.abort_flag, (int)a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    *a.info = CF_TIMEOUT;
                    __hip_atomic_fetch_or((gi32_t*)a.fault, FAULT_FLOW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (l == 0) *s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    return *s_ok != 0;
}

// non-blocking: are all flags (null = none) at `epoch`?  (lanes 0..2 read, the workgroup learns it)
__device__ __forceinline__ bool cf_test(const CholFlow& a, const int* f1, const int* f2, int* s_ok,
                                        const int* f3 = nullptr) {
    if (threadIdx.x < 64) {
        const int l = threadIdx.x;
        const int* f = l == 0 ? f1 : (l == 1 ? f2 : (l == 2 ? f3 : nullptr));
        const bool done = f == nullptr ||
                          (unsigned)__hip_atomic_load((gi32_t*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.epoch;
        const bool all = __all(done);
        if (l == 0) *s_ok = all ? 1 : 0;
    }
    __syncthreads();
    return *s_ok != 0;
}

// every flag of a list at `epoch`?  (flag q polled by thread q mod 256: the waits overlap)
template <class F>
__device__ __forceinline__ bool cf_wait_list(const CholFlow& a, int cnt, F flag, int* s_ok) {
    if (threadIdx.x == 0) *s_ok = 1;
    __syncthreads();
    for (int q = threadIdx.x; q < cnt; q += blockDim.x) {
        const int* f = flag(q);
        unsigned spins = 0;
        while ((unsigned)__hip_atomic_load((gi32_t*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != a.epoch) {
            if (++spins > CF_SPIN_LIMIT ||
                ((spins & 255) == 0 &&
                 (unsigned)__hip_atomic_load((gi32_t*)a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.epoch)) {
                __hip_atomic_store((gi32_t*)a.abort_flag, (int)a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                *a.info = CF_TIMEOUT;
                __hip_atomic_fetch_or((gi32_t*)a.fault, FAULT_FLOW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                *s_ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    return *s_ok != 0;
}

// Hand-offs of 32 x 32 tiles move 16 bytes per access (write-through sc1 buffer stores, sc1 buffer loads, all of a
// thread's loads in flight together): thread t covers the element pairs e = 2 t + 512 m (m = 0, 1), row e >> 5,
// columns e & 31 and the next.  An 8 KB tile handed from one workgroup to another (store, drain, flag, poll, load)
// took 1.0-1.2 us this way against 1.7-1.8 us with 8-byte sc1 accesses (scripts/micro/handoff_lat.hip,
// profiles/r4w_handoff_latency.txt).  tile_rsrc: a buffer over the tile (row stride ld doubles).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const double* p, int ld) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(8 * (31 * (long long)ld + CNB)), 0x00020000);
}
__device__ __forceinline__ double lo_dbl(v4u q) { return __longlong_as_double(((long long)q.y << 32) | q.x); }
__device__ __forceinline__ double hi_dbl(v4u q) { return __longlong_as_double(((long long)q.w << 32) | q.z); }
// a 32 x 32 tile of handed-off data into registers (two 16-byte sc1 loads per thread), and from there to LDS
__device__ __forceinline__ void cf_fetch(const double* src, int ld, double (&r)[4]) {
    const __amdgpu_buffer_rsrc_t rs = tile_rsrc(src, ld);
    v4u q[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int e = 2 * (int)threadIdx.x + 512 * m;
        q[m] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((e >> 5) * ld + (e & 31)) * 8, 0, BUF_SC1);
    }
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        r[2 * m] = lo_dbl(q[m]);
        r[2 * m + 1] = hi_dbl(q[m]);
    }
}
__device__ __forceinline__ void cf_put(double (*T)[CNB + 1], const double (&r)[4]) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int e = 2 * (int)threadIdx.x + 512 * m;
        T[e >> 5][e & 31] = r[2 * m];
        T[e >> 5][(e & 31) + 1] = r[2 * m + 1];
    }
}
// rows r0 .. r0 + 31 of a staged panel (LDS) out as a handed-off 32 x 32 tile (two 16-byte sc1 stores per thread)
__device__ __forceinline__ void cf_store_tile(double* dst, int ld, const double (*T)[CNB + 1]) {
    const __amdgpu_buffer_rsrc_t rs = tile_rsrc(dst, ld);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int e = 2 * (int)threadIdx.x + 512 * m, r = e >> 5, c = e & 31;
        const long long a0 = __double_as_longlong(T[r][c]), a1 = __double_as_longlong(T[r][c + 1]);
        const v4u q = {(unsigned)a0, (unsigned)(a0 >> 32), (unsigned)a1, (unsigned)(a1 >> 32)};
        __builtin_amdgcn_raw_buffer_store_b128(q, rs, (r * ld + c) * 8, 0, BUF_SC1);
    }
}

// every storing wave drains its sc1 stores, then one lane publishes the flag
__device__ __forceinline__ void cf_publish(const CholFlow& a, int* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store((gi32_t*)flag, (int)a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 32 x 32 tile of a row-major matrix (leading dimension n) -> LDS, sc1 loads (handed-off data)
__device__ __forceinline__ void cf_load_tile(const double* src, int n, double (*T)[CNB + 1]) {
    double r[4];
    cf_fetch(src, n, r);
    cf_put(T, r);
}

// acc (this wave's quadrant) += X[rows of rb] Y[rows of cb]^T, K = 32
__device__ __forceinline__ d4 cf_mma_nt(const double (*X)[CNB + 1], const double (*Y)[CNB + 1], int rb, int cb,
                                        int lr, int kq, d4 acc) {
#pragma unroll
    for (int k0 = 0; k0 < CNB; k0 += 4)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(X[rb * 16 + lr][k0 + kq], Y[cb * 16 + lr][k0 + kq], acc, 0, 0, 0);
    return acc;
}
// acc += X[rows of rb] Y[:, columns of cb], K = 32
__device__ __forceinline__ d4 cf_mma_nn(const double (*X)[CNB + 1], const double (*Y)[CNB + 1], int rb, int cb,
                                        int lr, int kq, d4 acc) {
#pragma unroll
    for (int k0 = 0; k0 < CNB; k0 += 4)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(X[rb * 16 + lr][k0 + kq], Y[k0 + kq][cb * 16 + lr], acc, 0, 0, 0);
    return acc;
}

#ifndef LBA_CF_BAND_WAVES   // waves per SIMD the band kernel is compiled for (A/B builds only; 3 spills and is
#define LBA_CF_BAND_WAVES 2   // slower, profiles/r8t_ab_chol_waves.txt)
#endif
// BAND: the substitution solve's kernel (kinds 0, 4, 5, 6, 7, no lookahead: the host gives none in band mode); the
// L^-1 solve's kernel (kinds 0 with or without lookahead, 1, 2, 3, 4) otherwise
template <bool BAND>
__device__ __forceinline__ void chol_flow_body(const CholFlow& a, const DevProblem& P) {
    (void)P;
    __shared__ double Lt[3][CNB][CNB + 1];       // update operands L(j, p), L(i, p), L(k, p)
    __shared__ double stg[BAND ? 1 : 2][2 * CNB][CNB + 1];  // stacked panels of the factoring waves
    __shared__ long long s_ticket;
    __shared__ int s_ok;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rb = wave >> 1, cb = wave & 1, lr = lane & 15, kq = lane >> 4;
    const int n = a.n;
    // (the tile ids a task touches come precomputed with it, read into registers at the task's start or
    // with its list entry, so no address on the chain waits for a table search)
    auto tile_at = [&](auto* base, int tid_) { return base + ((size_t)tid_ << 10); };
    auto tri_id = [&](int i, int j) { return i * (i + 1) / 2 + j; };
    auto load_quad = [&](int tl, double (&q)[4]) {   // tile tl of S (assembled by an earlier launch)
#pragma unroll
        for (int m = 0; m < 4; ++m) q[m] = tile_at(a.S, tl)[(rb * 16 + kq + 4 * m) * CNB + cb * 16 + lr];
    };
    auto stage_quad = [&](double (*T)[CNB + 1], int r0, const double (&q)[4]) {
#pragma unroll
        for (int m = 0; m < 4; ++m) T[r0 + rb * 16 + kq + 4 * m][cb * 16 + lr] = q[m];
    };
    auto sub_mma = [&](double (&q)[4], d4 p) {
#pragma unroll
        for (int m = 0; m < 4; ++m) q[m] -= p[m];
    };
    // one wave: two-level pivot sequence of its stacked panel in `st` (row r of lane r)
    auto factor = [&](double (*st)[CNB + 1], bool& bad) { factor_pipe(st, lane, bad); };
    const d4 z4 = {0.0, 0.0, 0.0, 0.0};
    while (true) {
        if (tid == 0) s_ticket = (long long)atomicAdd(a.head, 1ull);
        __syncthreads();
        const long long t = s_ticket;
        __syncthreads();
        if (t >= a.ntasks) break;
        const int code = a.tasks[t];
        const int j = code & 0xffffff, i = a.task_i[t];
        const int kind = (code >> 24) & 15;
        const bool la = !BAND && ((code >> 28) & 1);   // factor task with lookahead over column k = j - 1
        if (!BAND && kind == 1) {
            // ---------------------------------------------------- L^-1 tile (i, j), i > j:
            // Linv(i,j) = -L_ii^-1 sum_k L(i,k) Linv(k,j) over the list's k (Linv(j,j) = LinvT_j^T)
            const d4 z = {0.0, 0.0, 0.0, 0.0};
            d4 acc = z;
            bool ok = true;
            unsigned long long* tv = (a.tdbg2 && tid == 0 && i >= a.NP - 2) ? a.tdbg2 + 16 * j + 4 * (i - (a.NP - 2)) : nullptr;
            if (tv) tv[0] = __builtin_amdgcn_s_memrealtime();
            const int zr = tid >> 3, zc = (tid & 7) * 4;   // z(i, j): row zr, columns zc .. zc + 3
            double bj[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) bj[u] = ld_sc1(a.b + j * CNB + zc + u);
            for (int q = a.pl0[t]; q < a.pl0[t + 1]; ++q) {
                const int k = a.plist[q] & 0xffffff, tik = a.plist_t[3 * q];
                if (!cf_wait(a, a.lready + tik, k == j ? a.fready + j : a.ivready + tri_id(k, j), &s_ok)) {
                    ok = false;
                    break;
                }
                cf_load_tile(tile_at(a.Lm, tik), CNB, Lt[0]);
                if (k == j) {
#pragma unroll
                    for (int m = 0; m < 4; ++m) {   // Linv(j,j)[r][c] = LinvT_j[c][r]
                        const int e = tid + 256 * m;
                        Lt[1][e & 31][e >> 5] = ld_sc1(a.LinvT + (size_t)j * CNB * CNB + e);
                    }
                } else {
                    cf_load_tile(a.Linv + (size_t)(k * CNB) * n + j * CNB, n, Lt[1]);
                }
                __syncthreads();
                acc = cf_mma_nn(Lt[0], Lt[1], rb, cb, lr, kq, acc);
                __syncthreads();
            }
            if (tv) tv[1] = __builtin_amdgcn_s_memrealtime();
            if (!ok || !cf_wait(a, a.fready + i, nullptr, &s_ok)) return;
            if (tv) tv[2] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
            for (int m = 0; m < 4; ++m) {   // L_ii^-1 = LinvT_i^T
                const int e = tid + 256 * m;
                Lt[0][e & 31][e >> 5] = ld_sc1(a.LinvT + (size_t)i * CNB * CNB + e);
                Lt[1][rb * 16 + kq + 4 * m][cb * 16 + lr] = acc[m];
            }
            __syncthreads();
            const d4 v = cf_mma_nn(Lt[0], Lt[1], rb, cb, lr, kq, z);
            __syncthreads();   // (Lt[1] was an operand of the product)
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int rr = rb * 16 + kq + 4 * m, cc = cb * 16 + lr;
                st_sc1(a.Linv + (size_t)(i * CNB + rr) * n + j * CNB + cc, -v[m]);
                Lt[1][rr][cc] = -v[m];
            }
            __syncthreads();
            double zs = 0.0;
#pragma unroll
            for (int u = 0; u < 4; ++u) zs += Lt[1][zr][zc + u] * bj[u];
            zs += __shfl_xor(zs, 1);
            zs += __shfl_xor(zs, 2);
            zs += __shfl_xor(zs, 4);
            if ((tid & 7) == 0) st_sc1(a.zv + ((size_t)i * a.NP + j) * CNB + zr, zs);
            cf_publish(a, a.ivready + tri_id(i, j));
            if (tv) tv[3] = __builtin_amdgcn_s_memrealtime();
            continue;
        }
        if (!BAND && kind == 2) {
            // ---------------------------------------------------- x_j = sum_r Linv(r,j)^T y_r over the list's
            // r (Linv(j,j)^T = LinvT_j), into xsol in natural panel order.  Each term's tile is fetched as
            // soon as it is published, ahead of y_r.
            const int c = tid & 31, rq = tid >> 5;   // output c, rows 4 rq .. 4 rq + 3 of each term
            double part = 0.0;
            bool ok = true;
            for (int q = a.pl0[t]; q < a.pl0[t + 1]; ++q) {
                const int r = a.plist[q] & 0xffffff;
                if (!cf_wait(a, r == j ? a.fready + j : a.ivready + tri_id(r, j), nullptr, &s_ok)) {
                    ok = false;
                    break;
                }
                double lv[4], yr[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int rr = 4 * rq + u;
                    lv[u] = r == j ? ld_sc1(a.LinvT + (size_t)j * CNB * CNB + c * CNB + rr)
                                   : ld_sc1(a.Linv + (size_t)(r * CNB + rr) * n + j * CNB + c);
                }
                if (!cf_wait(a, a.dready + r, nullptr, &s_ok)) {
                    ok = false;
                    break;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) yr[u] = ld_sc1(a.yv + r * CNB + 4 * rq + u);
#pragma unroll
                for (int u = 0; u < 4; ++u) part += lv[u] * yr[u];
            }
            if (!ok) return;
            Lt[1][rq][c] = part;
            __syncthreads();
            if (tid < CNB) {
                double x = 0.0;
#pragma unroll
                for (int u = 0; u < 8; ++u) x += Lt[1][u][tid];
                a.xout[a.rnat[j * CNB + tid]] = x;
            }
            if (a.tdbg && tid == 0) a.tdbg[16 * j + 15] = __builtin_amdgcn_s_memrealtime();
            __syncthreads();
            continue;
        }
        if (BAND && kind == 6) {
            // ---------------------------------------------------- distributed factorisation, part 0: this rank's
            // contribution to top tile (i, j), S(i,j) -= sum over its subtree panels p (the list) of L(i,p) L(j,p)^T
            // (the ranks' S tiles of the top are all-reduced before part 1 factors them)
            const int t_ij = a.task_t[5 * t];
            d4 acc = z4;
            for (int q = a.pl0[t]; q < a.pl0[t + 1]; ++q) {
                const int tjp = a.plist_t[3 * q], tip = a.plist_t[3 * q + 1];
                if (!cf_wait(a, a.lready + tjp, a.lready + tip, &s_ok)) return;
                cf_load_tile(tile_at(a.Lm, tjp), CNB, Lt[0]);
                cf_load_tile(tile_at(a.Lm, tip), CNB, Lt[1]);
                __syncthreads();
                acc = cf_mma_nt(Lt[1], Lt[0], rb, cb, lr, kq, acc);
                __syncthreads();
            }
            double* Sq = const_cast<double*>(tile_at(a.S, t_ij));   // (read by the pack kernel after this launch)
#pragma unroll
            for (int m = 0; m < 4; ++m) Sq[(rb * 16 + kq + 4 * m) * CNB + cb * 16 + lr] -= acc[m];
            continue;
        }
        if (BAND && kind == 7) {
            // ---------------------------------------------------- distributed factorisation, part 0: this rank's
            // contribution to the top rhs block i, bS_i -= sum over its subtree panels p (the list) of L(i,p) y_p
            const int r = tid & 31, g = tid >> 5;
            double acc = 0.0;
            for (int q = a.pl0[t]; q < a.pl0[t + 1]; ++q) {
                const int kk = a.plist[q] & 0xffffff, tik = a.plist_t[3 * q];
                if (!cf_wait(a, a.lready + tik, a.dready + kk, &s_ok)) return;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    acc += ld_sc1(tile_at(a.Lm, tik) + r * CNB + 4 * g + u) * ld_sc1(a.yv + kk * CNB + 4 * g + u);
            }
            Lt[1][g][r] = acc;
            __syncthreads();
            if (tid < CNB) {
                double v = 0.0;
#pragma unroll
                for (int u = 0; u < 8; ++u) v += Lt[1][u][tid];
                const_cast<double*>(a.b)[i * CNB + tid] -= v;
            }
            __syncthreads();
            continue;
        }
        if (kind == 4) {
            // ---------------------------------------------------- band mode, forward substitution:
            // y_i = L_ii^-1 (b_i - sum_k L(i,k) y_k) over the list's k (update order); thread (r, g) takes
            // row r, columns 4g .. 4g + 3 of every term
            const int r = tid & 31, g = tid >> 5;
            double acc = 0.0;
            for (int q = a.pl0[t]; q < a.pl0[t + 1]; ++q) {
                const int kk = a.plist[q] & 0xffffff, tik = a.plist_t[3 * q];
                if (!cf_wait(a, a.lready + tik, a.dready + kk, &s_ok)) return;
                double lv[4], yk[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    lv[u] = ld_sc1(tile_at(a.Lm, tik) + r * CNB + 4 * g + u);
                    yk[u] = ld_sc1(a.yv + kk * CNB + 4 * g + u);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) acc += lv[u] * yk[u];
            }
            if (!cf_wait(a, a.fready + i, nullptr, &s_ok)) return;
#pragma unroll
            for (int m = 0; m < 4; ++m) {   // L_ii^-T -> Lt[2] in one round of loads
                const int e = tid + 256 * m;
                Lt[2][e >> 5][e & 31] = ld_sc1(a.LinvT + (size_t)i * CNB * CNB + e);
            }
            Lt[1][g][r] = acc;
            __syncthreads();
            if (tid < CNB) {
                double v = ld_sc1(a.b + i * CNB + tid);
#pragma unroll
                for (int u = 0; u < 8; ++u) v -= Lt[1][u][tid];
                Lt[0][0][tid] = v;
            }
            __syncthreads();
            if (tid < CNB) {   // (L_ii^-1 v)[r] = sum_c LinvT_i[c][r] v[c]
                double y = 0.0;
#pragma unroll 8
                for (int c = 0; c < CNB; ++c) y += Lt[2][c][tid] * Lt[0][0][c];
                st_sc1(a.yv + i * CNB + tid, y);
            }
            cf_publish(a, a.dready + i);
            if (a.tdbg && tid == 0) a.tdbg[16 * i + 7] = __builtin_amdgcn_s_memrealtime();
            continue;
        }
        if (BAND && kind == 5) {
            // ---------------------------------------------------- band mode, back substitution:
            // x_j = L_jj^-T (y_j - sum_i L(i,j)^T x_i) over the list's rows i > j (completion order);
            // thread (c, g) takes output c, rows 4g .. 4g + 3 of every term.  Everything that is not an
            // x_i is fetched first (L_jj^-T into LDS, y_j, the terms' L(i,j) entries into registers: the
            // factorisation published them long before), so the chain from x_i to x_j is one hand-off,
            // the dot products and the publication
            const int c = tid & 31, g = tid >> 5;
            constexpr int MT = 4;   // terms held in registers (the rest are fetched as they come, ahead of their x_i)
            const int q0 = a.pl0[t], nt = a.pl0[t + 1] - q0;
            if (!cf_wait(a, a.fready + j, a.dready + j, &s_ok)) return;
#pragma unroll
            for (int m = 0; m < 4; ++m) {   // L_jj^-T -> Lt[0] (row c of Lt[0] = column c of L_jj^-1)
                const int e = tid + 256 * m;
                Lt[0][e >> 5][e & 31] = ld_sc1(a.LinvT + (size_t)j * CNB * CNB + e);
            }
            const double yj = tid < CNB ? ld_sc1(a.yv + j * CNB + tid) : 0.0;
            // every term's tile L(i, j) published (one poll per term, side by side: one round trip for the list)
            if (!cf_wait_list(a, nt, [&](int q) { return a.lready + a.plist_t[3 * (q0 + q)]; }, &s_ok)) return;
            double lv[MT][4];
#pragma unroll
            for (int q = 0; q < MT; ++q)
                if (q < nt) {
                    const int tl = a.plist_t[3 * (q0 + q)];
#pragma unroll
                    for (int u = 0; u < 4; ++u) lv[q][u] = ld_sc1(tile_at(a.Lm, tl) + (4 * g + u) * CNB + c);
                }
            // x_i of a term: wave 0 polls its 64 granules (one per lane, one round trip: the flag is the data) and
            // hands the 32 values to the workgroup in LDS (xs[q & 1]: a buffer is rewritten two terms later, behind
            // the barrier of the term between)
            double(*xs)[CNB] = reinterpret_cast<double(*)[CNB]>(&Lt[1][8][0]);
            auto take_x = [&](int ii, double* dst) {
                if (tid < 64) {
                    const gu64_t* gp = (const gu64_t*)(a.xg + (size_t)ii * 2 * CNB + tid);
                    unsigned long long v = 0;
                    bool ok = true;
                    for (unsigned spins = 0;; ++spins) {
                        v = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (__all((unsigned)(v >> 32) == a.epoch)) break;
                        if (spins > CF_SPIN_LIMIT ||
                            ((spins & 255) == 255 &&
                             (unsigned)__hip_atomic_load((gi32_t*)a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.epoch)) {
                            if (tid == 0) {
                                __hip_atomic_store((gi32_t*)a.abort_flag, (int)a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                *a.info = CF_TIMEOUT;
                                __hip_atomic_fetch_or((gi32_t*)a.fault, FAULT_FLOW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            }
                            ok = false;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    const unsigned lo = (unsigned)v, hi = (unsigned)__shfl_xor((int)lo, 1);   // lane 2r: low half
                    if ((tid & 1) == 0) dst[tid >> 1] = __longlong_as_double(((long long)hi << 32) | lo);
                    if (tid == 0) s_ok = ok ? 1 : 0;
                }
                __syncthreads();
                return s_ok != 0;
            };
            double acc = 0.0;
#pragma unroll
            for (int q = 0; q < MT; ++q)
                if (q < nt) {
                    const int ii = a.plist[q0 + q] & 0xffffff;
                    if (!take_x(ii, xs[q & 1])) return;
                    double xi[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) xi[u] = xs[q & 1][4 * g + u];
#pragma unroll
                    for (int u = 0; u < 4; ++u) acc += lv[q][u] * xi[u];
                }
            for (int q = MT; q < nt; ++q) {
                const int ii = a.plist[q0 + q] & 0xffffff;
                const int tl = a.plist_t[3 * (q0 + q)];
                double l4[4], xi[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) l4[u] = ld_sc1(tile_at(a.Lm, tl) + (4 * g + u) * CNB + c);
                if (!take_x(ii, xs[q & 1])) return;
#pragma unroll
                for (int u = 0; u < 4; ++u) xi[u] = xs[q & 1][4 * g + u];
#pragma unroll
                for (int u = 0; u < 4; ++u) acc += l4[u] * xi[u];
            }
            Lt[1][g][c] = acc;
            __syncthreads();
            if (tid < CNB) {
                double v = yj;
#pragma unroll
                for (int u = 0; u < 8; ++u) v -= Lt[1][u][tid];
                Lt[2][0][tid] = v;
            }
            __syncthreads();
            if (tid < CNB) {   // (L_jj^-T v)[c] = sum_r LinvT_j[c][r] v[r]
                double x = 0.0;
#pragma unroll 8
                for (int rr = 0; rr < CNB; ++rr) x += Lt[0][tid][rr] * Lt[2][0][rr];
                const unsigned long long xb = (unsigned long long)__double_as_longlong(x), tag = (unsigned long long)a.epoch << 32;
                gu64_t* gp = (gu64_t*)(a.xg + (size_t)j * 2 * CNB + 2 * tid);
                __hip_atomic_store(gp, tag | (xb & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(gp + 1, tag | (xb >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                a.xout[a.rnat[j * CNB + tid]] = x;
            }
            __syncthreads();
            if (a.tdbg && tid == 0) a.tdbg[16 * j + 15] = __builtin_amdgcn_s_memrealtime();
            continue;
        }
        if (!BAND && kind == 3) {
            // ---------------------------------------------------- y_i = sum_k z(i, k) over the list's k
            // (z(i, k) = Linv(i, k) b_k, made by the tasks of Linv(i, k) and panel i): the forward solve
            // without a chain through the panels
            const int q0 = a.pl0[t], cnt = a.pl0[t + 1] - q0;
            if (!cf_wait_list(a, cnt, [&](int q) {
                    const int k = a.plist[q0 + q] & 0xffffff;
                    return k == i ? a.zready + i : a.ivready + tri_id(i, k);
                }, &s_ok)) return;
            const int r = tid & 31, g = tid >> 5;   // row r, terms g, g + 8, ...
            double acc = 0.0;
            for (int q = g; q < cnt; q += 32) {
                double zz[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int qq = q + 8 * u;
                    zz[u] = qq < cnt ? ld_sc1(a.zv + ((size_t)i * a.NP + (a.plist[q0 + qq] & 0xffffff)) * CNB + r) : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) acc += zz[u];
            }
            Lt[1][g][r] = acc;
            __syncthreads();
            if (tid < CNB) {
                double y = 0.0;
#pragma unroll
                for (int u = 0; u < 8; ++u) y += Lt[1][u][tid];
                st_sc1(a.yv + i * CNB + tid, y);
            }
            cf_publish(a, a.dready + i);
            if (a.tdbg && tid == 0) a.tdbg[16 * i + 7] = __builtin_amdgcn_s_memrealtime();
            continue;
        }
        const bool diag = i == j;
        // diagnostics: stamps of panel j's task (slots 0..6) and of tile (j + 1, j) (slots 8..14)
        unsigned long long* tm = (a.tdbg && tid == 0 && (diag || i == j + 1)) ? a.tdbg + 16 * j + (diag ? 0 : 8) : nullptr;
        if (tm) tm[0] = __builtin_amdgcn_s_memrealtime();
        unsigned long long* tf = (a.tdbg3 && tid == 0 && t < 4096) ? a.tdbg3 + (size_t)CF_TDBG_STRIDE * t : nullptr;
        if (tf) { tf[0] = __builtin_amdgcn_s_memrealtime(); tf[4] = i | (j << 12) | ((int)la << 24); }
        // the task's tiles: (j,j), (i,j), and with lookahead (k,k), (j,k), (i,k) (-1 when (i,k) is zero)
        const int t_jj = a.task_t[5 * t], t_ij = a.task_t[5 * t + 1], t_kk = a.task_t[5 * t + 2],
                  t_jk = a.task_t[5 * t + 3], t_ik = a.task_t[5 * t + 4];
        const bool ik_env = la && !diag && t_ik >= 0;   // tile (i, j - 1) structurally non-zero
        double qd[4], qa[4];
        load_quad(t_jj, qd);
        if (!diag) load_quad(t_ij, qa);
        // lookahead: the task also holds A(k,k), A(j,k), A(i,k) of the previous column k = j - 1, whose
        // update is the last one of A(j,j) and A(i,j) in update order (the host checks); it factors
        // column k's two tiles itself, so only L(., p <= k - 1) is waited for, one chain step earlier
        const bool ik = ik_env;   // tile (i, k) structurally non-zero
        double qk[4], qjk[4], qik[4];
        if (la) {
            load_quad(t_kk, qk);
            load_quad(t_jk, qjk);
            if (ik) load_quad(t_ik, qik);
        }
        // ---- updates from the envelope panels p (< j, or < k with lookahead), software-pipelined (the
        //      next panel's tiles are fetched into registers when already published, while this panel's
        //      products run).  Entry: p | row i takes part << 24 [| row j << 25 | row k << 26 (lookahead)]
        double rj[4], ri[4], rk[4];
        bool have = false;
        auto rows = [&](int e, bool& fj, bool& fi, bool& fk) {
            fi = !diag && ((e >> 24) & 1);
            fj = la ? ((e >> 25) & 1) : true;
            fk = la && ((e >> 26) & 1);
        };
        // list entry q: tiles (j,p), (i,p), (k,p) in plist_t
        auto ready = [&](int q, bool block) {
            bool fj, fi, fk;
            rows(a.plist[q], fj, fi, fk);
            const int* f1 = fj ? a.lready + a.plist_t[3 * q] : nullptr;
            const int* f2 = fi ? a.lready + a.plist_t[3 * q + 1] : nullptr;
            const int* f3 = fk ? a.lready + a.plist_t[3 * q + 2] : nullptr;
            return block ? cf_wait(a, f1, f2, &s_ok, f3) : cf_test(a, f1, f2, &s_ok, f3);
        };
        auto fetch = [&](int q) {
            bool fj, fi, fk;
            rows(a.plist[q], fj, fi, fk);
            if (fj) cf_fetch(tile_at(a.Lm, a.plist_t[3 * q]), CNB, rj);
            if (fi) cf_fetch(tile_at(a.Lm, a.plist_t[3 * q + 1]), CNB, ri);
            if (fk) cf_fetch(tile_at(a.Lm, a.plist_t[3 * q + 2]), CNB, rk);
        };
        // entries [q0, known] of the list are published: tested up to 16 entries at a time (one flag per lane, one
        // round trip); a published flag stays so, so a list of long-published tiles costs one round trip per 16
        // entries instead of one per entry ahead of its products
        const int q0 = a.pl0[t], q1 = a.pl0[t + 1];
        int known = q0 - 1;
        auto test_ahead = [&](int upto) {   // extend `known` towards `upto` (non-blocking)
            if (known >= upto) return;
            const int first = known + 1, last = min(first + 15, q1 - 1);
            if (threadIdx.x < 64) {
                const int l = threadIdx.x, q = first + l / 3, part = l % 3;
                bool done = true;
                if (l < 48 && q <= last) {
                    bool fj, fi, fk;
                    rows(a.plist[q], fj, fi, fk);
                    if (part == 0 ? fj : (part == 1 ? fi : fk))
                        done = (unsigned)__hip_atomic_load((gi32_t*)(a.lready + a.plist_t[3 * q + part]), __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT) == a.epoch;
                }
                const unsigned long long nb = __ballot(!done);   // lanes of entries not yet published
                if (l == 0) s_ok = nb ? first + (int)(__builtin_ctzll(nb) / 3) - 1 : last;
            }
            __syncthreads();
            known = s_ok;   // (the next write of s_ok comes after a barrier that follows this read)
        };
        bool ok = true;
        // lookahead: column k's two tiles are factored as soon as their own updates are in (after the list
        // entry marked with bit 27, or before the first entry when the task's bit 29 says none updates them),
        // so the rest of the list (updates of rows j / i only) waits while it factors; the update from k is
        // applied last, as before (the same order of updates on every copy of a tile)
        auto factor_k = [&]() {
            // ---- column k here: [A(k,k); A(j,k)] on wave 0 and [A(k,k); A(i,k)] on wave 1 -> L(j,k), L(i,k)
            //      (the same stacked factorisations as the tasks of column k), kept staged for the update
            stage_quad(stg[0], 0, qk);
            stage_quad(stg[0], CNB, qjk);
            if (ik) {
                stage_quad(stg[BAND ? 0 : 1], 0, qk);
                stage_quad(stg[BAND ? 0 : 1], CNB, qik);
            }
            __syncthreads();
            if (wave == 0 || (wave == 1 && ik)) {
                bool bad;
                factor(stg[BAND ? 0 : wave], bad);
                (void)bad;   // (reported by panel k's own task)
            }
            __syncthreads();
            if (tf) tf[6] = __builtin_amdgcn_s_memrealtime();
        };
        if (la && ((code >> 29) & 1)) factor_k();
        // the panels in update order (the same order in every task: the copies of a tile stay bitwise
        // identical)
        for (int q = q0; q < q1; ++q) {
            const int e = a.plist[q];
            bool fj, fi, fk;
            rows(e, fj, fi, fk);
            const bool waited = !have;
            if (!have) {
                if (!ready(q, true)) { ok = false; break; }
                known = max(known, q);
                if (tf) { tf[3] = __builtin_amdgcn_s_memrealtime(); tf[4] = (tf[4] & 0xffffffull) | ((unsigned long long)(la) << 24) | ((unsigned long long)(e & 0xffffff) << 32); }
                fetch(q);
            }
            if (fj) cf_put(Lt[0], rj);
            if (fi) cf_put(Lt[1], ri);
            if (fk) cf_put(Lt[2], rk);
            __syncthreads();
            if (q + 1 < q1) test_ahead(q + 1);
            have = q + 1 < q1 && q + 1 <= known;
            if (have) fetch(q + 1);
            if (fj) sub_mma(qd, cf_mma_nt(Lt[0], Lt[0], rb, cb, lr, kq, z4));
            if (fi && fj) sub_mma(qa, cf_mma_nt(Lt[1], Lt[0], rb, cb, lr, kq, z4));
            if (fk) {
                sub_mma(qk, cf_mma_nt(Lt[2], Lt[2], rb, cb, lr, kq, z4));
                if (fj) sub_mma(qjk, cf_mma_nt(Lt[0], Lt[2], rb, cb, lr, kq, z4));
                if (ik && fi) sub_mma(qik, cf_mma_nt(Lt[1], Lt[2], rb, cb, lr, kq, z4));
            }
            __syncthreads();
            if (tf && q - q0 < 16) {
                tf[8 + 2 * (q - q0)] = __builtin_amdgcn_s_memrealtime();
                tf[9 + 2 * (q - q0)] = (unsigned long long)((e & 0xffffff) | ((int)waited << 24));
            }
            if (la && ((e >> 27) & 1)) factor_k();
        }
        if (tf) tf[5] = __builtin_amdgcn_s_memrealtime();
        if (ok && la) {   // the update from column k (factored above)
            sub_mma(qd, cf_mma_nt(stg[0] + CNB, stg[0] + CNB, rb, cb, lr, kq, z4));
            if (ik) sub_mma(qa, cf_mma_nt(stg[BAND ? 0 : 1] + CNB, stg[0] + CNB, rb, cb, lr, kq, z4));
            __syncthreads();
            if (tm) tm[2] = __builtin_amdgcn_s_memrealtime();
        }
        if (tf) tf[1] = __builtin_amdgcn_s_memrealtime();
        if (!ok) return;
        if (tm) tm[1] = __builtin_amdgcn_s_memrealtime();
        const size_t p0 = (size_t)j * CNB;
        if (!diag) {
            // ---- [A(j,j); A(i,j)] on wave 0 -> L(i, j) (rows 32..63)
            stage_quad(stg[0], 0, qd);
            stage_quad(stg[0], CNB, qa);
            __syncthreads();
            if (tm) tm[4] = __builtin_amdgcn_s_memrealtime();
            if (wave == 0) {
                bool bad;
                const unsigned long long c0 = tf ? clock64() : 0;
                factor(stg[0], bad);
                if (tf) tf[7] = clock64() - c0;
                if (tm) tm[5] = __builtin_amdgcn_s_memrealtime();
                (void)bad;   // (a non-positive pivot of A(j,j) is reported by panel j's own task)
            }
            __syncthreads();
            // L(i, j) from the staged panel by all four waves (a quarter of the write-through bytes per
            // wave: the drain before the flag is a quarter as long as one wave storing the tile)
            cf_store_tile(tile_at(a.Lm, t_ij), CNB, stg[0] + CNB);
            cf_publish(a, a.lready + t_ij);
            if (tm) tm[6] = __builtin_amdgcn_s_memrealtime();
            if (tf) tf[2] = __builtin_amdgcn_s_memrealtime();
            continue;
        }
        // ---- panel j: [A_jj; I] -> L_jj, L_jj^-T on wave 0, published for the L^-1 tasks
        stage_quad(stg[0], 0, qd);
#pragma unroll
        for (int m = 0; m < 4; ++m) {   // rows 32..63: the identity
            const int e = tid + 256 * m, r = e >> 5, c = e & 31;
            stg[0][CNB + r][c] = (c == r) ? 1.0 : 0.0;
        }
        __syncthreads();
        if (tm) tm[4] = __builtin_amdgcn_s_memrealtime();
        if (wave == 0) {
            bool bad;
            const unsigned long long c0 = tf ? clock64() : 0;
            factor(stg[0], bad);
            if (tf) tf[7] = clock64() - c0;
            if (__ballot(bad) != 0 && lane == 0) *a.info = 1 + (int)p0;
            if (tm) tm[5] = __builtin_amdgcn_s_memrealtime();
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 4; ++m) {   // L_jj (plain: no reader in this launch), L_jj^-T, by all waves
            const int e = tid + 256 * m, r = e >> 5, c = e & 31;
            tile_at(a.Lm, t_jj)[r * CNB + c] = (c <= r) ? stg[0][r][c] : 0.0;
        }
        cf_store_tile(a.LinvT + p0 * CNB, CNB, stg[0] + CNB);
        cf_publish(a, a.fready + j);
        if (tm) tm[6] = __builtin_amdgcn_s_memrealtime();
        if (tf) tf[2] = __builtin_amdgcn_s_memrealtime();
        if (a.zv) {   // z(j, j) = L_jj^-1 b_j from L_jj^-T (rows 32..63 of the staged panel)
            const int r = tid >> 3, c0 = (tid & 7) * 4;
            double zs = 0.0;
#pragma unroll
            for (int u = 0; u < 4; ++u) zs += stg[0][CNB + c0 + u][r] * ld_sc1(a.b + j * CNB + c0 + u);
            zs += __shfl_xor(zs, 1);
            zs += __shfl_xor(zs, 2);
            zs += __shfl_xor(zs, 4);
            if ((tid & 7) == 0) st_sc1(a.zv + ((size_t)j * a.NP + j) * CNB + r, zs);
        }
        cf_publish(a, a.zready + j);
    }
}

// the L^-1 solve (dense mode: config 1's few tasks, one workgroup per CU with the lookahead's registers; compiled for
// 2 waves per SIMD it spills and config 1's solve takes 99 instead of 77 us, profiles/r8t_ab_chol_waves.txt)
__global__ __launch_bounds__(256) void k_chol_flow(CholFlow a, DevProblem P) { chol_flow_body<false>(a, P); }
// the substitution solve (band mode: thousands of tasks; no lookahead, so two workgroups fit a CU)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LBA_CF_BAND_WAVES, LBA_CF_BAND_WAVES)))
void k_chol_flow_band(CholFlow a, DevProblem P) { chol_flow_body<true>(a, P); }

// ------------------------------------------------------------------------------------------------
constexpr int UPD_THREADS = 64;     // one landmark (or KF) per thread: many small blocks for latency hiding
static_assert(UPD_THREADS == UPD_BLOCK_KFS, "k_update's KF blocks (the host numbers the fused evaluation's producers)");

// Trial state of a KF (state kc): Twb <- Twb exp(dxi), v += dv (G2oTypes.cc:41-46) with the step dx (12) =
// the solved step, or the stale x when the factorisation failed (BlockSolver leaves x untouched, g2o then
// applies and pops it); dx null: a fixed KF.  One (non-inlined) function body for every caller, so every copy
// of a state is bitwise identical.
// A KF's trial state: kc its state, dx its step (x of the solve, or BlockSolver's stale x after a failed
// factorisation; nullptr: fixed), d <- the step (dx may be d itself: every element is read before any is written),
// kn <- the trial state.  (Every input is loaded into registers before the first store: through generic pointers
// the compiler could not hoist a load above a store that might alias it, and interleaved loads and stores
// serialise into one memory round trip per element.)
__device__ __attribute__((noinline)) void kf_trial_state(const double* __restrict__ kc, const double* dx, double* d,
                                                         double* __restrict__ kn) {
    double c[KF_STRIDE];
#pragma unroll
    for (int j = 0; j < KF_STRIDE; ++j) c[j] = kc[j];
    if (dx) {
        double dl[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) dl[j] = dx[j];
        const SE3 T = se3_mul(load_se3(c), se3_exp(dl));
#pragma unroll
        for (int j = 0; j < 12; ++j) d[j] = dl[j];
        kn[0] = T.q.x; kn[1] = T.q.y; kn[2] = T.q.z; kn[3] = T.q.w;
        kn[4] = T.t[0]; kn[5] = T.t[1]; kn[6] = T.t[2];
#pragma unroll
        for (int j = 0; j < 6; ++j) kn[7 + j] = c[7 + j] + dl[6 + j];
#pragma unroll
        for (int j = 13; j < KF_STRIDE; ++j) kn[j] = c[j];
    } else {
#pragma unroll
        for (int j = 0; j < KF_STRIDE; ++j) kn[j] = c[j];
    }
}

// One observation's share of the back-substitution, sum_k Hpl(k, l)^T x_k = sum_{o of l} G_o^T t_s(o): with
// G_o = rho' w sum_rows J1^T Jp (the observation's part of every Hpl block it feeds, k_lin_schur phase 3) and
// t_s = N_s x (the step of the observation's pose sample), G_o^T t = rho' w sum_rows Jp^T (J1 t).  The
// linearisation is recomputed at the state the sweep linearised (the same inputs and code as lin_obs).
template <int DIM, bool F32 = false>
__device__ __forceinline__ void bs_obs(const DevProblem& P, const double* gps, const double* kst, const double* lst,
                                       const double* camd, const ObsIn& in, int cam, bool gp, const double* t,
                                       double* v) {
    CamD cd;
    load_cam(camd + (size_t)cam * CAMD_STRIDE, &cd);
    double Rwb[9], twb[3];
    const double bf = obs_pose(gps, kst, in, gp, Rwb, twb);
    double z[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) z[d] = in.z[d];
    const double w = in.w;
    double Xb[3], Xc[3], e[DIM];
    project_residual_p<DIM, F32>(Rwb, twb, cd, lst + (size_t)in.lm * 3, z, bf, Xb, Xc, e);
    double chi = 0.0;
#pragma unroll
    for (int d = 0; d < DIM; ++d) chi += e[d] * (w * e[d]);
    double r0, r1;
    huber(chi, DIM == 3 ? P.huber_stereo : P.huber_mono, &r0, &r1);
    double J1[6 * DIM], Jp[3 * DIM];
    obs_j1_p<DIM, F32>(Rwb, cd, Xb, Xc, bf, J1, Jp);
    const double s = r1 * w;
    v[0] = v[1] = v[2] = 0.0;
#pragma unroll
    for (int d = 0; d < DIM; ++d) {
        double u = 0.0;
#pragma unroll
        for (int j = 0; j < 6; ++j) u += J1[d * 6 + j] * t[j];
#pragma unroll
        for (int a = 0; a < 3; ++a) v[a] += u * Jp[d * 3 + a];
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) v[a] *= s;
}

// Rows r0, r0 + 1 (r0 even) of a pose sample's step t_s = N_s [x_a; x_b] (+ the extrinsic factor on x_e): N column c
// at 12 + 6 c, so the two rows of a column are one 16-byte load; bk: the sample's pose blocks (a, b, extrinsic) and
// camera.  Each row is summed in column order, as one row per task did.  (Formed per sample once, by k_update's
// GP-pair / KF-block workgroups, and handed to the tiles through their flags, it made the fused k_update slower: the
// producers' chains are the launch's other critical path, profiles/r4u_ab_ts_per_sample_rejected.txt.)
__device__ __forceinline__ void ts_rows2(const DevProblem& P, const double* gps, const double* camd, int smp, int4 bk, int r0,
                                         double& a0, double& a1) {
    const double* N = gps + (size_t)smp * GPS_STRIDE + 12 + r0;
    const int hs[3] = {bk.x, bk.y, bk.z};
    a0 = 0.0;
    a1 = 0.0;
#pragma unroll
    for (int side = 0; side < 3; ++side) {
        const int h = hs[side];
        if (h < 0) continue;
        const double* x = P.xsol + 12 * (size_t)h;
        const double* Nc = side < 2 ? N + 6 * 12 * side : camd + (size_t)bk.w * CAMD_STRIDE + 16 + r0;
#pragma unroll
        for (int c = 0; c < 12; ++c) {
            const double2 n2 = *reinterpret_cast<const double2*>(Nc + 6 * c);
            a0 += n2.x * x[c];
            a1 += n2.y * x[c];
        }
    }
}
// The landmarks of regular tile `tile` (one UPD_THREADS workgroup): dx_l = Dinv_l (b_l - sum_{o of l} G_o^T t_s(o))
// (block_solver.hpp:461-482), oplus, computeScale partial.  Returns this thread's scale term.
constexpr int UPD_TILE_OBS_PER_THREAD = (TILE_OBS + 63) / 64;
constexpr int UPD_TILE_TASKS_PER_THREAD = (TILE_SMP * 3 + UPD_THREADS - 1) / UPD_THREADS;   // (sample, row pair) tasks
constexpr int BS_SHM = TILE_SMP * 6 + TILE_OBS * 3;
// (Latency-bound: every load a thread needs is issued in a few batches, each stage's index loads for all of its
// tasks before their data loads, and the landmark's own inputs at entry, so a tile costs a handful of memory
// round trips instead of one chain per task.)
// (ltr, optional, LDS [TILE_LMS][3]: the tile's trial landmark positions, for the fused evaluation)
template <bool F32>
__device__ double bs_tile(const DevProblem& P, int tile, int si, bool ok, double lambda, double* lo, double* shm,
                          unsigned long long* stamp, double* ltr = nullptr) {
    double(*tsh)[6] = reinterpret_cast<double(*)[6]>(shm);                  // t_s per tile sample
    double(*vsh)[3] = reinterpret_cast<double(*)[3]>(shm + TILE_SMP * 6);   // G_o^T t per observation
    const int tid = threadIdx.x;
    const int lm0 = P.tile_lm0[tile], nlm = P.tile_nlm[tile];
    const double* __restrict__ lst = P.lbuf[si];
    // this thread's landmark: b_l, Hll, its state and the step of a failed factorisation, loaded up front
    const bool has_l = tid < nlm;
    const int l = lm0 + (has_l ? tid : 0);
    double blv[3], Hv[9], lv[3], xold[3];
    int lob0 = 0, lob1 = 0;
    if (has_l) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            blv[a] = P.bl[3 * (size_t)l + a];
            lv[a] = lst[3 * (size_t)l + a];
            xold[a] = P.x[P.np + 3 * (size_t)l + a];
        }
#pragma unroll
        for (int q = 0; q < 9; ++q) Hv[q] = P.Hll[(size_t)l * 9 + q];
        lob0 = P.lm_obs0[l];
        lob1 = P.lm_obs0[l + 1];
    }
    // (run whatever the factorisation's status, read at the launch's start: branching on it would put that load's
    // round trip ahead of every load below; after a failed factorisation the results go unused)
    {
        const int ts0 = P.tile_smp0[tile], nts = P.tile_nsmp[tile];
        const int obs0 = P.tile_obs0[tile], nobs = P.tile_nobs[tile];
        const double* __restrict__ kst = P.kbuf[si];
        const double* __restrict__ gps = P.gpsb[si];
        const double* __restrict__ camd = P.camdb[si];
        // t_s(r) = sum_c N_s(r, c) [x_a; x_b](c) (+ the extrinsic factor on x_e): one task per (sample, row pair)
        int sm[UPD_TILE_TASKS_PER_THREAD];
        int4 bk[UPD_TILE_TASKS_PER_THREAD];
#pragma unroll
        for (int q = 0; q < UPD_TILE_TASKS_PER_THREAD; ++q) {
            const int task = tid + UPD_THREADS * q;
            const bool in = task < nts * 3;
            sm[q] = in ? P.tsm_smp[ts0 + task / 3] : -1;
            bk[q] = in ? *reinterpret_cast<const int4*>(P.tsm_blk + 4 * (size_t)(ts0 + task / 3)) : make_int4(-1, -1, -1, -1);
        }
        double acc[UPD_TILE_TASKS_PER_THREAD][2];
#pragma unroll
        for (int q = 0; q < UPD_TILE_TASKS_PER_THREAD; ++q) {
            const int task = tid + UPD_THREADS * q;
            acc[q][0] = acc[q][1] = 0.0;
            if (sm[q] >= 0) ts_rows2(P, gps, camd, sm[q], bk[q], 2 * (task % 3), acc[q][0], acc[q][1]);
        }
#pragma unroll
        for (int q = 0; q < UPD_TILE_TASKS_PER_THREAD; ++q)
            if (sm[q] >= 0) {
                const int task = tid + UPD_THREADS * q;
                tsh[task / 3][2 * (task % 3)] = acc[q][0];
                tsh[task / 3][2 * (task % 3) + 1] = acc[q][1];
            }
        __syncthreads();
        if (stamp) stamp[0] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int k = 0; k < UPD_TILE_OBS_PER_THREAD; ++k) {
            const int ol = tid + UPD_THREADS * k;
            if (ol < nobs) {
                const int o = obs0 + ol;
                const int meta = P.ob_meta[o], orw = P.ob_row[o];
                const ObsIn in = obs_in(P, o);
                const int kind = meta & 15, cam = meta >> 4;
                const bool gp = kind <= LBA_STEREO_GP;
                const double* t = tsh[orw >> 16];
                if (kind == LBA_STEREO_GP || kind == LBA_STEREO) bs_obs<3, F32>(P, gps, kst, lst, camd, in, cam, gp, t, vsh[ol]);
                else bs_obs<2, F32>(P, gps, kst, lst, camd, in, cam, gp, t, vsh[ol]);
            }
        }
        __syncthreads();
        if (stamp) stamp[1] = __builtin_amdgcn_s_memrealtime();
    }
    double sc = 0.0;
    if (has_l) {
        double xl[3];
        double* xd = P.x + P.np + 3 * (size_t)l;
        if (ok) {
            double c[3] = {blv[0], blv[1], blv[2]};
            const int ob0 = P.tile_obs0[tile];
            for (int o = lob0; o < lob1; ++o) {
                const double* v = vsh[o - ob0];
                c[0] -= v[0]; c[1] -= v[1]; c[2] -= v[2];
            }
            // Dinv = (Hll + lambda I)^-1 (Eigen's adjugate inverse, block_solver.hpp:389), the sweep's Hll and damping
            double D[9];
            Hv[0] += lambda; Hv[4] += lambda; Hv[8] += lambda;
            inv3(Hv, D);
            for (int a = 0; a < 3; ++a) {
                xl[a] = D[a * 3] * c[0] + D[a * 3 + 1] * c[1] + D[a * 3 + 2] * c[2];
                xd[a] = xl[a];
            }
        } else {
            xl[0] = xold[0]; xl[1] = xold[1]; xl[2] = xold[2];
        }
        for (int a = 0; a < 3; ++a) {
            const double v = lv[a] + xl[a];
            lo[3 * (size_t)l + a] = v;
            if (ltr) ltr[3 * tid + a] = v;
            sc += xl[a] * (lambda * xl[a] + blv[a]);
        }
    }
    return sc;
}

#ifndef LBA_UPD_POLL_SLEEP
#define LBA_UPD_POLL_SLEEP 2
#endif
// Fused evaluation (k_update, eval = 1): wait until the producers `prod` (one per lane, < 0: none; the GP pairs and
// KF blocks whose pose samples / states the workgroup reads) have stored them write-through and set their flag to
// this launch's epoch (lanes poll side by side; bounded, as k_chol_flow's waits)
__device__ __forceinline__ void upd_wait(const DevProblem& P, int prod, unsigned epoch) {
    // (one poll per distinct producer: a lane whose left neighbour waits for the same one stays quiet)
    const int left = __shfl_up(prod, 1, 64);
    if ((threadIdx.x & 63) > 0 && left == prod) prod = -1;
    bool done = prod < 0;
    unsigned spins = 0;
    while (!__all(done)) {
        if (!done) {
            const unsigned f = (unsigned)__hip_atomic_load((gi32_t*)(P.upd_flag + (size_t)FLAG_STRIDE * prod), __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
            done = f == epoch;
        }
        if (__all(done)) break;
        __builtin_amdgcn_s_sleep(LBA_UPD_POLL_SLEEP);
        if (++spins > (1u << 20)) {   // (~0.5 s: never expected) the samples may be stale: the call fails
            if (!done) __hip_atomic_fetch_or((gi32_t*)P.fault, FAULT_UPD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
    }
    __syncthreads();
}
// ... and a producer (workgroup role `self`) reports its (write-through) stores done
__device__ __forceinline__ void upd_publish(const DevProblem& P, int self, unsigned epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store((gi32_t*)(P.upd_flag + (size_t)FLAG_STRIDE * self), (int)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The tile's observations at the trial state (k_eval's tile item: the same per-observation arithmetic and the same
// reduction tree, so chi_eval / ob_chi2 are bitwise k_eval's): poses from the trial samples, landmarks from ltr
// (this workgroup's back-substitution).  The samples are written in this launch, write-through, by other
// workgroups; they are read with plain loads, which is safe without an acquire because no line holding a trial
// pose is read in this launch before its producer's flag: the caches start the launch invalidated, a tile reads only
// the first 96 bytes (Rwb, twb) of the records it waited for, and the bytes a pose's line shares with the previous
// record are that record's Jacobian factor, which nothing reads in this launch.  The acquire fence the consumer
// form would otherwise need cost 1.5-11 us per LM iteration (profiles/r7j_ab_acquire_rejected.txt), and sc1 loads
// of these few hundred hot records from every tile more than the whole k_eval launch (+12 us).  Everything but
// the poses is loaded before the wait for the samples (upd_wait_samples), so after it the tile is one round of
// loads from done.
struct TrialObs {
    ObsIn in;
    int o, meta;
    double bf;
};
__device__ __forceinline__ void eval_tile_prefetch(const DevProblem& P, int tile, int si, TrialObs (&to)[UPD_TILE_OBS_PER_THREAD]) {
    const int tid = threadIdx.x;
    const double* __restrict__ kst = P.kbuf[si];      // (bf: the same in both state buffers)
    const int obs0 = P.tile_obs0[tile], nobs = P.tile_nobs[tile];
#pragma unroll
    for (int k = 0; k < UPD_TILE_OBS_PER_THREAD; ++k) {
        const int ol = tid + UPD_THREADS * k;
        to[k].o = ol < nobs ? obs0 + ol : -1;
        if (ol < nobs) {
            to[k].meta = P.ob_meta[obs0 + ol];
            to[k].in = obs_in(P, obs0 + ol);
        }
    }
#pragma unroll
    for (int k = 0; k < UPD_TILE_OBS_PER_THREAD; ++k)
        if (to[k].o >= 0) {
            const bool gp = (to[k].meta & 15) <= LBA_STEREO_GP;
            to[k].bf = kst[(size_t)(gp ? to[k].in.kfa : to[k].in.kfb) * KF_STRIDE + 14];
        }
}
template <bool F32>
__device__ __forceinline__ void eval_tile_trial(const DevProblem& P, int tile, int si, const double* ltr,
                                                const TrialObs (&to)[UPD_TILE_OBS_PER_THREAD]) {
    const int tid = threadIdx.x;
    const double* __restrict__ gpn = P.gpsb[si ^ 1];
    const double* __restrict__ camd = P.camdb[si];    // (no free extrinsic: the same in both)
    const int lm0 = P.tile_lm0[tile];
    double Rwb[UPD_TILE_OBS_PER_THREAD][9], twb[UPD_TILE_OBS_PER_THREAD][3];
#pragma unroll
    for (int k = 0; k < UPD_TILE_OBS_PER_THREAD; ++k)
        if (to[k].o >= 0) {
            const double* S = gpn + (size_t)to[k].in.smp * GPS_STRIDE;
#pragma unroll
            for (int i = 0; i < 9; ++i) Rwb[k][i] = S[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) twb[k][i] = S[9 + i];
        }
    double rho[UPD_TILE_OBS_PER_THREAD];
#pragma unroll
    for (int k = 0; k < UPD_TILE_OBS_PER_THREAD; ++k) {
        rho[k] = 0.0;
        if (to[k].o >= 0) {
            const int kind = to[k].meta & 15, cam = to[k].meta >> 4;
            const double* Xw = ltr + 3 * (to[k].in.lm - lm0);
            rho[k] = (kind == LBA_STEREO_GP || kind == LBA_STEREO)
                         ? eval_obs_at<3, F32>(P, Rwb[k], twb[k], to[k].bf, Xw, camd, to[k].o, to[k].in, cam)
                         : eval_obs_at<2, F32>(P, Rwb[k], twb[k], to[k].bf, Xw, camd, to[k].o, to[k].in, cam);
        }
    }
    // k_eval: one observation per thread of TILE_OBS = 2 x 64; block_sum = wave sums, then 0 + wave 0 + wave 1
    static_assert(UPD_TILE_OBS_PER_THREAD == 2 && TILE_OBS == 2 * UPD_THREADS, "k_eval's reduction tree");
    const double s0 = wave_sum(rho[0]), s1 = wave_sum(rho[1]);
    if (tid == 0) {
        double s = 0.0;
        s += s0;
        s += s1;
        P.chi_eval[tile] = s;
    }
}

// The step and the trial state (block_solver.hpp:461-482 back-substitution, sparse_optimizer.cpp:422-435
// oplus, computeScale partials), fused with the pose samples of the trial state:
//   workgroups [0, n_gp): one per GP pair: its two KFs' trial states (kf_trial_state), then the pair's
//     samples with their Jacobian factors (gp_pair_prep, jac) into the trial state's sample buffer, so
//     an accepted trial's next linearisation needs no preparation launch;
//   then one KF per thread (trial state, KF pose sample, x, scale); then one workgroup per regular tile
//   (bs_tile: its landmarks back-substituted in the sample space, oplus, scale); then one heavy landmark
//   per thread (dx_l = Dinv (bl - sum Hpl^T dx_p), oplus, scale).
// k_update's LDS, one allocation for its three roles: a GP pair (its KFs' trial-state slots, then
// gp_pair_prep's buffers), a KF block (kf_trial_state's output slots: the function stays one compiled body
// for both callers, their trial states must agree bitwise, without its output arrays living in scratch), a
// tile (bs_tile).  (One allocation keeps k_update at 8 workgroups per CU, so every tile is resident at once.)
constexpr int UPD_GP_SHM = 2 * 12 + 2 * KF_STRIDE + 2 * (KF_STRIDE + 12) + PREP_SHM;
constexpr int UPD_KF_SHM = UPD_THREADS * (12 + KF_STRIDE);
constexpr int UPD_SHM = UPD_GP_SHM > UPD_KF_SHM ? (UPD_GP_SHM > BS_SHM ? UPD_GP_SHM : BS_SHM)
                                                : (UPD_KF_SHM > BS_SHM ? UPD_KF_SHM : BS_SHM);
template <bool WT>
__device__ void prior_eval_t(const DevProblem& P, const double* __restrict__ kst, int idx);
// eval (with P.fuse_eval): the trial state's errors too.  The producers of the pose samples (the GP pairs and KF
// blocks) store the samples / KF states write-through and report once they are stored; the regular tiles, after
// their back-substitution, and the motion-prior / velocity items (workgroups after the update's) wait for all
// producers and evaluate: k_eval's work in the same launch.  The host fuses only when the whole grid is resident
// at once (P.fuse_eval, set from the occupancy), so a waiting workgroup never holds a slot a producer needs,
// whatever the dispatch order.  (Roles from an atomic ticket instead, for any grid size, cost one same-address
// atomic per workgroup: +10 us per trial at config 1, +700 us at config 2, profiles/r4i_ab_fused_eval_ticket_rejected.txt.)
template <bool F32>
__global__ __launch_bounds__(UPD_THREADS) void k_update(DevProblem P, double lambda_arg, int sel, int gate, int jac,
                                                        int eval, unsigned epoch) {
    __shared__ double red[UPD_THREADS / 64];
    __shared__ double ushm[UPD_SHM];
    __shared__ double ltr[TILE_LMS * 3];
    if (gated_off(P.ctl, gate)) return;
    const bool fused = eval && P.fuse_eval;
    const int role = blockIdx.x;
    // diagnostics (LBA_PHASE_TIMING): s_memrealtime start / end of each workgroup in slots 14 / 15 of the
    // sweep's stamp rows (k_update runs after the sweep; n_upd_blocks <= n_tiles is checked)
    unsigned long long* ustamp = (P.tdbg_lin && threadIdx.x == 0 && (int)blockIdx.x < P.n_tiles)
                                     ? P.tdbg_lin + (size_t)blockIdx.x * 16 + 14 : nullptr;
    if (ustamp) ustamp[0] = __builtin_amdgcn_s_memrealtime();
    const double lambda = damping(P, lambda_arg);
    const int si = state_idx(P, sel);
    const double* __restrict__ kst = P.kbuf[si];
    const double* __restrict__ lst = P.lbuf[si];
    double* __restrict__ ko = P.kbuf[si ^ 1];
    double* __restrict__ lo = P.lbuf[si ^ 1];
    double* gps = P.gpsb[si ^ 1];
    const bool ok = (*P.info == 0);
    const int nkb = (P.n_kf + UPD_THREADS - 1) / UPD_THREADS;
    if (role >= P.n_upd_blocks) {   // (fused) motion-prior / velocity edges of the trial state: the KF blocks
        const int nkb_ = (P.n_kf + UPD_THREADS - 1) / UPD_THREADS;
        // (every KF block, UPD_THREADS of them per round: a prior may touch any keyframe)
        for (int b0 = 0; b0 < nkb_; b0 += UPD_THREADS)
            upd_wait(P, b0 + (int)threadIdx.x < nkb_ ? P.n_gp + b0 + (int)threadIdx.x : -1, epoch);
        prior_eval_t<false>(P, ko, (role - P.n_upd_blocks) * UPD_THREADS + threadIdx.x);   // (plain loads: see eval_tile_trial)
        return;
    }
    if (role < P.n_gp) {
        const int i = role;
        double* kdl = ushm;                    // [2][12]
        double* kab = ushm + 2 * 12;           // [2][KF_STRIDE]
        double* kin = ushm + 2 * 12 + 2 * KF_STRIDE;   // [2][KF_STRIDE + 12]: the two KFs' states and steps,
                                                       // staged by 56 lanes in one round of loads
        {
            const int t = threadIdx.x, side = t >= KF_STRIDE + 12 ? 1 : 0, e = t - side * (KF_STRIDE + 12);
            if (t < 2 * (KF_STRIDE + 12)) {
                const int k = P.gp_hab[4 * i + side], h = P.gp_hab[4 * i + 2 + side];
                if (e < KF_STRIDE) {
                    kin[t] = kst[(size_t)k * KF_STRIDE + e];
                } else if (h >= 0) {   // the step, both candidates loaded ahead of the status (no round trip on it)
                    const double xs = P.xsol[12 * (size_t)h + e - KF_STRIDE], xo = P.x[12 * (size_t)h + e - KF_STRIDE];
                    kin[t] = ok ? xs : xo;
                }
            }
        }
        __syncthreads();
        if (threadIdx.x < 2) {
            double* in = kin + (KF_STRIDE + 12) * threadIdx.x;
            kf_trial_state(in, P.gp_hab[4 * i + 2 + threadIdx.x] >= 0 ? in + KF_STRIDE : nullptr, kdl + 12 * threadIdx.x,
                           kab + KF_STRIDE * threadIdx.x);
        }
        __syncthreads();
#ifndef LBA_EXP_NO_GPPREP
        // (the poses published as soon as they are stored, ahead of their Jacobian factors)
        auto pub = [&]() {
            if (fused) upd_publish(P, role, epoch);
            if (ustamp) ustamp[-3] = __builtin_amdgcn_s_memrealtime();   // (slot 11: published)
        };
        gp_pair_prep<true>(P, gps, i, kab, kab + KF_STRIDE, jac, ushm + 2 * 12 + 2 * KF_STRIDE + 2 * (KF_STRIDE + 12),
                           ustamp ? P.tdbg_lin + (size_t)blockIdx.x * 16 + 5 : nullptr, pub);
#endif
        if (threadIdx.x == 0) P.scale_part[role] = 0.0;
        if (ustamp) ustamp[1] = __builtin_amdgcn_s_memrealtime();
        return;
    }
    double sc = 0.0;
    bool tile_eval = false;
    if (role < P.n_gp + nkb) {
        const int k = (role - P.n_gp) * UPD_THREADS + threadIdx.x;
        // (diagnostics: stamps in slots 5 .. 8 of its row: start, trial states formed, stored, published)
        unsigned long long* kst_stamp = ustamp ? P.tdbg_lin + (size_t)blockIdx.x * 16 + 5 : nullptr;
        if (kst_stamp) kst_stamp[0] = __builtin_amdgcn_s_memrealtime();
        if (k < P.n_kf) {
            const int h = P.kf_hidx[k], xc = P.kf_cam[k];
            // this KF's b_p rows and their owners, loaded before the first store (see kf_trial_state)
            double bph[12];
            bool adds[12];
#pragma unroll
            for (int j = 0; j < 12; ++j) {
                bph[j] = h >= 0 ? P.bp[12 * h + j] : 0.0;
                adds[j] = h >= 0 && row_adds(P, 12 * h + j);
            }
            double* d = ushm + 12 * threadIdx.x;
            double* kn = ushm + 12 * UPD_THREADS + KF_STRIDE * threadIdx.x;
            if (h >= 0)   // the step staged in d (both candidates loaded ahead of the status; d gets them anyway)
#pragma unroll
                for (int j = 0; j < 12; ++j) {
                    const double xs = P.xsol[12 * (size_t)h + j], xo = P.x[12 * (size_t)h + j];
                    d[j] = ok ? xs : xo;
                }
            kf_trial_state(kst + (size_t)k * KF_STRIDE, h >= 0 ? d : nullptr, d, kn);
            if (kst_stamp) kst_stamp[1] = __builtin_amdgcn_s_memrealtime();
            double* kw = ko + (size_t)k * KF_STRIDE;
            for (int j = 0; j < KF_STRIDE; ++j) stv<true>(kw + j, kn[j]);   // (write-through: the fused evaluation)
            kf_pose_record<true>(P, gps, k, kn);
            if (kst_stamp) kst_stamp[2] = __builtin_amdgcn_s_memrealtime();
            if (xc >= 0) {   // a free extrinsic: the trial state's camera record (Tcb, intrinsics, Ad(Tbc))
                const double* c0 = P.camdb[si] + (size_t)xc * CAMD_STRIDE;
                SE3 T;
                T.q = Quat{kn[0], kn[1], kn[2], kn[3]};
                T.t[0] = kn[4]; T.t[1] = kn[5]; T.t[2] = kn[6];
                cam_record(T, c0[12], c0[13], c0[14], c0[15], P.camdb[si ^ 1] + (size_t)xc * CAMD_STRIDE);
            }
            if (h >= 0)
#pragma unroll
                for (int j = 0; j < 12; ++j) {
                    if (ok) P.x[12 * h + j] = d[j];
                    // (partitioned: b_p is the all-reduced one, a row's term is counted by its owner)
                    if (adds[j]) sc += d[j] * (lambda * d[j] + bph[j]);
                }
        }
        if (fused) upd_publish(P, role, epoch);
        if (kst_stamp) kst_stamp[3] = __builtin_amdgcn_s_memrealtime();
    } else if (role < P.n_gp + nkb + P.n_stiles) {
        sc = bs_tile<F32>(P, role - P.n_gp - nkb, si, ok, lambda, lo, ushm,
                     ustamp ? P.tdbg_lin + (size_t)blockIdx.x * 16 + 5 : nullptr, fused ? ltr : nullptr);
        tile_eval = fused;
    } else {
        // heavy landmarks (device indices n_lm - n_heavy ..): through their merged Hpl blocks
        const int l = P.n_lm - P.n_heavy + (role - P.n_gp - nkb - P.n_stiles) * UPD_THREADS + threadIdx.x;
        if (l < P.n_lm) {
            double xl[3];
            double* xd = P.x + P.np + 3 * (size_t)l;
            if (ok) {
                double c[3] = {P.bl[3 * (size_t)l], P.bl[3 * (size_t)l + 1], P.bl[3 * (size_t)l + 2]};
                for (int p = P.lm_pair0[l]; p < P.lm_pair0[l + 1]; ++p) {
                    const double* B = P.Hpl + (size_t)(p - P.hpl_base) * 36;
                    const double* xp = P.xsol + 12 * (size_t)P.pair_kf[p];
                    for (int r = 0; r < 12; ++r) {
                        c[0] -= B[r * 3] * xp[r];
                        c[1] -= B[r * 3 + 1] * xp[r];
                        c[2] -= B[r * 3 + 2] * xp[r];
                    }
                }
                const double* D = P.Dinv + (size_t)l * 9;
                for (int a = 0; a < 3; ++a) {
                    xl[a] = D[a * 3] * c[0] + D[a * 3 + 1] * c[1] + D[a * 3 + 2] * c[2];
                    xd[a] = xl[a];
                }
            } else {
                xl[0] = xd[0]; xl[1] = xd[1]; xl[2] = xd[2];
            }
            for (int a = 0; a < 3; ++a) {
                lo[3 * (size_t)l + a] = lst[3 * (size_t)l + a] + xl[a];
                sc += xl[a] * (lambda * xl[a] + P.bl[3 * (size_t)l + a]);
            }
        }
    }
    const double s = block_sum<UPD_THREADS>(sc, red);
    if (threadIdx.x == 0) P.scale_part[role] = s;
    if (tile_eval) {
        TrialObs to[UPD_TILE_OBS_PER_THREAD];
        eval_tile_prefetch(P, role - P.n_gp - nkb, si, to);
        // the producers of the tile's pose samples (one sample per lane: TILE_SMP = UPD_THREADS)
        const int tl = role - P.n_gp - nkb;
        static_assert(TILE_SMP <= UPD_THREADS, "one tile sample per lane");
        const int prod = (int)threadIdx.x < P.tile_nsmp[tl] ? P.smp_prod[P.tsm_smp[P.tile_smp0[tl] + threadIdx.x]] : -1;
        upd_wait(P, prod, epoch);   // (its barrier also completes ltr)
        if (ustamp) ustamp[-3] = __builtin_amdgcn_s_memrealtime();   // (slot 11: samples in; slots 12 / 13 are the
                                                                     // sweep's start / end of the same row)
        eval_tile_trial<F32>(P, role - P.n_gp - nkb, si, ltr, to);
    }
    if (ustamp) ustamp[1] = __builtin_amdgcn_s_memrealtime();
}

// ------------------------------------------------------------------------------------------------
template <bool WT>
__device__ void prior_eval_t(const DevProblem& P, const double* __restrict__ kst, int idx);
__device__ __forceinline__ void prior_eval(const DevProblem& P, const double* __restrict__ kst, int idx) {
    prior_eval_t<false>(P, kst, idx);
}

// Robust chi2 of the state: one workgroup per observation tile, then workgroups of TILE_OBS prior /
// velocity edges.  (The trial summary stays a separate k_finalize launch: having the last workgroup
// do it needs a device-scope release per workgroup, i.e. an L2 writeback each on this multi-XCD
// part, measured 3x slower than the extra launch.)
template <bool F32>
__global__ __launch_bounds__(TILE_OBS) void k_eval(DevProblem P, int sel, int gate) {
    __shared__ double red[TILE_OBS / 64];
    const int tile = blockIdx.x, tid = threadIdx.x;
    if (gated_off(P.ctl, gate)) return;
    const int si = state_idx(P, sel);
    const double* __restrict__ kst = P.kbuf[si];
    const double* __restrict__ lst = P.lbuf[si];
    const double* __restrict__ gps = P.gpsb[si];
    const double* __restrict__ camd = P.camdb[si];
    if (tile < P.n_tiles) {
        double rho0 = 0.0;
        if (tid < P.tile_nobs[tile]) {
            const int o = P.tile_obs0[tile] + tid;
            const int meta = P.ob_meta[o];
            const ObsIn in = obs_in(P, o);
            const int kind = meta & 15, cam = meta >> 4;
            const bool gp = kind <= LBA_STEREO_GP;
            rho0 = (kind == LBA_STEREO_GP || kind == LBA_STEREO) ? eval_obs<3, F32>(P, gps, kst, lst, camd, o, in, cam, gp)
                                                                 : eval_obs<2, F32>(P, gps, kst, lst, camd, o, in, cam, gp);
        }
        const double s = block_sum<TILE_OBS>(rho0, red);
        if (tid == 0) P.chi_eval[tile] = s;
    } else {
        prior_eval(P, kst, (tile - P.n_tiles) * TILE_OBS + tid);
    }
}

// motion-prior / velocity edge idx: robust chi2 of the state kst into chi_eval (WT: the state read sc1, written
// in this launch: k_update's fused evaluation)
template <bool WT>
__device__ void prior_eval_t(const DevProblem& P, const double* __restrict__ kst, int idx) {
    if (idx < P.n_prior) {
        double ka[14], kb[14];
#pragma unroll
        for (int j = 0; j < 14; ++j) {
            ka[j] = ldv<WT>(kst + (size_t)P.pri_a[idx] * KF_STRIDE + j);
            kb[j] = ldv<WT>(kst + (size_t)P.pri_b[idx] * KF_STRIDE + j);
        }
        double e[12], Om[144];
        prior_error_jac<double>(load_se3(ka), ka + 7, ka[13], load_se3(kb), kb + 7, kb[13], e, nullptr, nullptr);
        qi_inv(P.qcinv, kb[13] - ka[13], Om);
        double chi = 0.0;
        for (int i = 0; i < 12; ++i) {
            double s = 0.0;
            for (int k = 0; k < 12; ++k) s += Om[i * 12 + k] * e[k];
            chi += e[i] * s;
        }
        double r0 = chi, r1 = 1.0;
        if (P.huber_prior > 0) huber(chi, P.huber_prior, &r0, &r1);
        P.chi_eval[P.n_tiles + idx] = r0;
    } else if (idx < P.n_prior + P.n_vel) {
        const int v = idx - P.n_prior;
        const double ev = ldv<WT>(kst + (size_t)P.vel_kf[v] * KF_STRIDE + 9);
        P.chi_eval[P.n_tiles + idx] = ev * (P.qcinv[14] * ev);
    } else if (idx < P.n_prior + P.n_vel + P.n_eprior) {   // EdgeExtrinsicPrior: e^T Om e
        const int q = idx - P.n_prior - P.n_vel;
        const double* ed = P.ep_data + 16 * (size_t)q;
        const double* kx = kst + (size_t)P.ep_kf[q] * KF_STRIDE;
        double e[3];
        ext_prior_error_jac(Quat{ldv<WT>(kx), ldv<WT>(kx + 1), ldv<WT>(kx + 2), ldv<WT>(kx + 3)},
                            Quat{ed[0], ed[1], ed[2], ed[3]}, e, nullptr);
        double chi = 0.0;
        for (int i = 0; i < 3; ++i) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += ed[4 + 3 * i + k] * e[k];
            chi += e[i] * s;
        }
        P.chi_eval[P.n_tiles + idx] = chi;
    }
}

// Trial summary: chi2 of the linearisation point, chi2 of the trial state, computeScale, factor
// status.  Besides the device copy it is published straight into host-mapped coherent memory,
// followed (after a system-scope fence) by the trial's sequence number, which the host polls:
// no copy kernel and no stream synchronisation per trial.
// queued: also take the LM decision of this trial on the device controller (the host-driven loop in
// lba_host.hip: optimize, i.e. OptimizationAlgorithmLevenberg::solve,
// optimization_algorithm_levenberg.cpp:61-169, and SparseOptimizer::optimize's iteration loop,
// sparse_optimizer.cpp:360-400), log whether the trial relinearised, and publish the controller.
__device__ void lm_decide(LMCtl& c, double chi_lin, double chi_trial, double scale, bool solved, int* hlog) {
#pragma clang fp contract(off)   // round every operation like the host loop (no fused multiply-add)
    if (hlog) hlog[c.slot % HLOG_CAP] = c.done ? 0 : 1;   // whether the trial's gated kernels ran
    c.slot++;
    if (c.done) return;
    // chi2 of the starting state (g2o's activeRobustChi2 before optimize): the first trial's chi2 at its
    // linearisation point, which is that state (no evaluation launch of its own ahead of the queue)
    if (c.chi0_lin) { c.chi0 = chi_lin; c.chi0_lin = 0; }
    if (c.qmax == 0) c.cur_chi = c.ini_chi = chi_lin;
    double temp = chi_trial;
    c.last_chi = chi_trial;
    if (!solved) { temp = DBL_MAX; c.failures++; }
    const double rho = (c.cur_chi - temp) / (scale + 1e-3);
    if (rho > 0 && isfinite(temp)) {
        const double t = 2 * rho - 1;
        double alpha = 1. - t * t * t;
        alpha = fmin(alpha, 2. / 3.);
        c.lambda *= fmax(1. / 3., alpha);
        c.ni = 2;
        c.cur_chi = temp;
        c.cur ^= 1;               // discardTop: the trial state becomes current
    } else {
        c.lambda *= c.ni;         // pop: keep the current state
        c.ni *= 2;
    }
    c.qmax++;
    if (rho < 0 && c.qmax < c.max_trials) {   // another trial of the same iteration
        c.need_lin = 0;
        return;
    }
    c.trials += c.qmax;
    c.it++;
    int result = LBA_RESULT_OK;
    if (c.qmax == c.max_trials || rho == 0) {
        result = LBA_RESULT_TERMINATE;
    } else if (c.early_stop) {
        if ((c.ini_chi - c.cur_chi) * 1e3 < c.ini_chi) c.nbad++;
        else c.nbad = 0;
        if (c.nbad >= 3) result = LBA_RESULT_TERMINATE;
    }
    c.result = result;
    c.qmax = 0;
    c.need_lin = 1;
    if ((result != LBA_RESULT_OK && c.early_stop) || c.it >= c.iters) c.done = 1;
}

// chi2 of the linearisation point, chi2 of the trial state, computeScale: sums in a fixed order
template <int NT>
__device__ void trial_sums(const DevProblem& P, double* red, double& sa, double& sb, double& sc) {
    const int tid = threadIdx.x;
    const int nc = P.n_tiles + P.n_prior + P.n_vel + P.n_eprior;
    // (the loads of U strided elements are issued before their additions, out-of-range ones masked: the
    //  same per-thread order of additions as the plain strided loop, without one round trip per element)
    // (the three arrays' loads of one round are issued together: one memory round trip per U * NT elements of
    //  the longer list, not one per list)
    constexpr int U = 8;
    double a = 0.0, b = 0.0, c = 0.0;
    const int nu = P.n_upd_blocks, nmax = nc > nu ? nc : nu;
    for (int i0 = tid; i0 < nmax; i0 += U * NT) {
        double xa[U], xb[U], xc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * NT;
            xa[u] = i < nc ? P.chi_lin[i] : 0.0;
            xb[u] = i < nc ? P.chi_eval[i] : 0.0;
            xc[u] = i < nu ? P.scale_part[i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i0 + u * NT < nc) { a += xa[u]; b += xb[u]; }
            if (i0 + u * NT < nu) c += xc[u];
        }
    }
    sa = block_sum<NT>(a, red);
    __syncthreads();
    sb = block_sum<NT>(b, red);
    __syncthreads();
    sc = block_sum<NT>(c, red);
}

// partitioned mode: this rank's sums (and factorisation status) for the all-reduce ahead of k_finalize
__global__ __launch_bounds__(256) void k_partials(DevProblem P) {
    __shared__ double red[256 / 64];
    double sa, sb, sc;
    trial_sums<256>(P, red, sa, sb, sc);
    if (threadIdx.x == 0) {
        P.red4[0] = sa; P.red4[1] = sb; P.red4[2] = sc; P.red4[3] = (double)(*P.info);
        // the fault word's bits, one per slot: summed over the ranks, every rank sees every rank's fault and fails
        // the call together (one rank alone throwing would leave the others in the next collective)
        const int f = *P.fault;
        for (int b = 0; b < RED_FAULT_BITS; ++b) P.red4[4 + b] = (double)((f >> b) & 1);
    }
}

// partitioned mode: bS and b_p into (unpack = 0) or back out of (unpack = 1) the all-reduce buffer (S itself,
// the packed envelope, is all-reduced in place)
__global__ __launch_bounds__(256) void k_env_pack(DevProblem P, int unpack, int gate) {
    if (gated_off(P.ctl, gate)) return;
    const int n = P.npad;
    double* buf = P.env_buf;
    // distributed factorisation: the top tiles of S first (after part 0 of k_chol_flow subtracted this rank's
    // contributions from them)
    const long long ntop = (long long)P.n_top_tiles * CHOL_NB * CHOL_NB;
    for (long long e = blockIdx.x * 256 + threadIdx.x; e < ntop; e += 256LL * gridDim.x) {
        double* sp = P.S + ((size_t)P.top_tiles[e >> 10] << 10) + (e & 1023);
        if (unpack) *sp = buf[e];
        else buf[e] = *sp;
    }
    buf += ntop;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < n + P.np; e += 256 * gridDim.x) {
        double* sp = e < n ? P.bS + e : P.bp + (e - n);
        if (unpack) *sp = buf[e];
        else buf[e] = *sp;
    }
}

// mode (FIN_*): host-driven trial (publish the summary); queued trial (decide, and publish the
// controller mirror when it is the last trial of a batch)
template <int NT>
__device__ void finalize_body(const DevProblem& P, unsigned long long seq, int mode, double* red) {
    const int tid = threadIdx.x;
    double sa, sb, sc, sinfo;
    // the controller and the factorisation status are loaded ahead of the sums (they do not change in this
    // launch): the decision then waits for one round of loads, not three
    LMCtl ctl;
    if (tid == 0 && mode != FIN_HOST) ctl = *P.ctl;
    const int info = P.part_n > 0 ? 0 : *P.info;
    int fault = *P.fault;
    if (P.part_n > 0) {   // partitioned: the all-reduced sums of every rank's k_partials
        sa = P.red4[0]; sb = P.red4[1]; sc = P.red4[2]; sinfo = P.red4[3];
        fault = 0;
        for (int b = 0; b < RED_FAULT_BITS; ++b) fault |= (P.red4[4 + b] != 0.0) << b;
    } else {
        trial_sums<NT>(P, red, sa, sb, sc);
        sinfo = (double)info;
    }
    if (tid != 0) return;
    const double v[4] = {sa, sb, sc, sinfo};
    if (mode == FIN_HOST) {
        for (int i = 0; i < 4; ++i) P.fin[i] = v[i];
    } else {
        if (!ctl.done)
            for (int i = 0; i < 4; ++i) P.fin[i] = v[i];
        lm_decide(ctl, sa, sb, sc, sinfo == 0.0, P.hlog);
        *P.ctl = ctl;
        if (mode != FIN_QUEUED_PUBLISH) return;
        volatile double* h = P.hfin + 8;
        const double* src = reinterpret_cast<const double*>(&ctl);
        for (int i = 0; i < LMCTL_DOUBLES; ++i) h[i] = src[i];
    }
    if (P.hfin) {
        volatile double* h = P.hfin;
        for (int i = 0; i < 4; ++i) h[i] = v[i];
        h[5] = (double)fault;
        __threadfence_system();
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(P.hfin + 4), seq, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(256) void k_finalize(DevProblem P, unsigned long long seq, int mode) {
    __shared__ double red[4];
    finalize_body<256>(P, seq, mode, red);
}

// lba_set_problem's zero ranges (pairs: address, 4-byte words), grid-stride over every range: the 16-byte-aligned body
// of a range with 16-byte stores, its ragged head and tail with 4-byte ones
__global__ __launch_bounds__(256) void k_zero_ranges(const unsigned long long* __restrict__ r, int n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x, t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = 0; k < n; ++k) {
        unsigned* d = reinterpret_cast<unsigned*>(r[2 * k]);
        const size_t words = r[2 * k + 1];
        const size_t head = min((size_t)(((16 - (r[2 * k] & 15)) & 15) / 4), words);   // words before a 16-byte boundary
        const size_t nq = (words - head) / 4;
        uint4* q = reinterpret_cast<uint4*>(d + head);
        for (size_t i = t0; i < nq; i += stride) q[i] = make_uint4(0u, 0u, 0u, 0u);
        for (size_t i = t0; i < head; i += stride) d[i] = 0u;
        for (size_t i = head + 4 * nq + t0; i < words; i += stride) d[i] = 0u;
    }
}
// words: the ranges' total, which sizes the grid (one 16-byte store per thread and pass, at most 2048 workgroups)
#ifndef LBA_ZERO_MAX_BLOCKS
#define LBA_ZERO_MAX_BLOCKS 2048
#endif
void launch_zero_ranges(const unsigned long long* ranges, int n, size_t words, hipStream_t s) {
    const size_t blocks = std::min<size_t>(LBA_ZERO_MAX_BLOCKS, std::max<size_t>(1, (words / 4 + 255) / 256));
    if (n > 0) hipLaunchKernelGGL(k_zero_ranges, dim3((unsigned)blocks), dim3(256), 0, s, ranges, n);
}

__global__ void k_ctl_init(DevProblem P, LMCtl c) {
    if (threadIdx.x == 0) *P.ctl = c;
}

// computeLambdaInit (optimization_algorithm_levenberg.cpp:171-185) on the device for a queued
// optimisation: tau * max |H_ii| over the pose diagonal (Sdiag: ASM_DIAG with lambda = 0, no Schur terms:
// diag Hpp) and the landmark diagonals.  A max is exact in any order.
__global__ __launch_bounds__(1024) void k_lambda_init(DevProblem P, double tau) {
    __shared__ double red[16];
    const int tid = threadIdx.x;
    double m = 0.0;
    for (int i = tid; i < P.np; i += 1024) m = fmax(m, fabs(P.Sdiag[i]));
    for (int i = tid; i < 3 * P.n_lm; i += 1024) m = fmax(m, fabs(P.Hll[9 * (size_t)(i / 3) + 4 * (i % 3)]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_down(m, off, 64));
    if ((tid & 63) == 0) red[tid >> 6] = m;
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 16; ++w) m = fmax(m, red[w]);
        P.ctl->lambda = tau * m;
    }
}

// isDepthPositive (src/G2oTypes.cc:65-81): GP edges test both KF poses (include/G2oTypes.h:305-314)
__global__ __launch_bounds__(256) void k_depth(DevProblem P, int sel, unsigned char* ok) {
    const int o = blockIdx.x * 256 + threadIdx.x;
    if (o >= P.n_obs) return;
    const double* __restrict__ lst = P.lbuf[state_idx(P, sel)];
    const int meta = P.ob_meta[o];
    const int kind = meta & 15, cam = meta >> 4;
    CamD cd;
    load_cam(P.camdb[state_idx(P, sel)] + (size_t)cam * CAMD_STRIDE, &cd);
    const double* Xw = lst + (size_t)P.ob_lm[o] * 3;
    int good = 1;
    const int ks[2] = {P.ob_kfb[o], kind <= LBA_STEREO_GP ? P.ob_kfa[o] : -1};
    for (int s = 0; s < 2; ++s) {
        if (ks[s] < 0) continue;
        const double* kp = P.kfp_pose + (size_t)ks[s] * KFP_STRIDE;
        const double d[3] = {Xw[0] - kp[9], Xw[1] - kp[10], Xw[2] - kp[11]};
        double Xb[3];
        mul33tv(kp, d, Xb);
        const double zc = cd.Rcb[6] * Xb[0] + cd.Rcb[7] * Xb[1] + cd.Rcb[8] * Xb[2] + cd.tcb[2];
        if (!(zc > 0)) good = 0;
    }
    ok[o] = (unsigned char)good;
}

// ------------------------------------------------------------------------------------------------ launchers
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

void launch_gp_prep(const DevProblem& P, int sel, int jac, int gate, hipStream_t s) {
    const int nb = P.n_gp + cdiv(P.n_kf, PREP_THREADS);
    if (nb) hipLaunchKernelGGL(k_gp_prep, dim3(nb), dim3(PREP_THREADS), 0, s, P, sel, jac, gate);
}
void launch_lin_schur(const DevProblem& P, int sel, int gate, double lambda, int mode, hipStream_t s, hipEvent_t e0,
                      hipEvent_t e1) {
    const int ne = (mode & LS_EDGES) ? P.n_prior + P.n_vel + P.n_eprior : 0;
    const dim3 g(P.n_tiles + ne);
    if (g.x == 0) return;
    auto kern = P.f32res ? k_lin_schur<true> : k_lin_schur<false>;
    if (e0)   // the events carry the dispatch's own start / end timestamps
        hipExtLaunchKernelGGL(kern, g, dim3(LS_THREADS), 0, s, e0, e1, 0, P, sel, gate, lambda, mode);
    else
        hipLaunchKernelGGL(kern, g, dim3(LS_THREADS), 0, s, P, sel, gate, lambda, mode);
}
void launch_expand(const DevProblem& P, int sel, int gate, double lambda, int schur, hipStream_t s) {
    const int n = P.n_smp + P.n_heavy;
    if (n) hipLaunchKernelGGL(k_expand, dim3(n), dim3(PRI_THREADS), 0, s, P, sel, gate, lambda, schur);
}
void launch_exp_asm(const DevProblem& P, int sel, int gate, double lambda, unsigned epoch, hipStream_t s) {
    const int n = P.n_smp + P.n_asm + P.n_pb;
    if (n) hipLaunchKernelGGL(k_exp_asm, dim3(n), dim3(144 * RED_GROUPS), 0, s, P, sel, gate, lambda, epoch);
}
void launch_assemble(const DevProblem& P, double lambda, int flags, int gate, hipStream_t s) {
    const int n = P.n_asm + P.n_pb;
    if (n) hipLaunchKernelGGL(k_assemble, dim3(n), dim3(144 * RED_GROUPS), 0, s, P, lambda, flags, gate);
}
static CholFlow make_flow(const DevProblem& P, unsigned epoch) {
    CholFlow a;
    const int n = P.npad;   // multiple of CHOL_NB (identity tail)
    a.n = n; a.NP = n / CHOL_NB; a.ntasks = P.cf_ntasks; a.epoch = epoch;
    a.tasks = P.cf_tasks; a.task_i = P.cf_task_i; a.task_t = P.cf_task_t; a.pl0 = P.cf_pl0;
    a.plist_t = P.cf_plist_t;
    a.plist = P.cf_plist;
    a.S = P.S; a.Lm = P.Lm; a.LinvT = P.LinvT; a.b = P.bS; a.yv = P.yv; a.info = P.info;
    a.lready = P.cf_lready; a.dready = P.cf_dready; a.head = P.cf_head; a.abort_flag = P.cf_abort; a.fault = P.fault;
    a.tdbg = P.tdbg_chol;
    a.tdbg2 = P.tdbg_bs;
    a.tdbg3 = P.tdbg_cf;
    a.Linv = P.cf_linv; a.ivready = P.cf_ivready; a.xout = P.xsol; a.rnat = P.rnat; a.fready = P.cf_fready;
    a.zready = P.cf_zready; a.zv = P.cf_zv;
    a.xg = P.cf_xg;
    return a;
}
static void launch_flow(const CholFlow& a, const DevProblem& P, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    // persistent workgroups: as many as are resident at once (256 CUs; the dense kernel fits one per CU, the
    // extra ones start as the others leave and find no tickets)
    const dim3 g(min(a.ntasks, 256 * max(2, P.cf_band ? LBA_CF_BAND_WAVES : 1)));
    if (g.x == 0) return;
    auto kern = P.cf_band ? k_chol_flow_band : k_chol_flow;
    if (e0 || e1)
        hipExtLaunchKernelGGL(kern, g, dim3(256), 0, s, e0, e1, 0, a, P);
    else
        hipLaunchKernelGGL(kern, g, dim3(256), 0, s, a, P);
}
void launch_cholesky_solve(const DevProblem& P, int gate, unsigned epoch, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    (void)gate;
    if (P.npad == 0) return;
    launch_flow(make_flow(P, epoch), P, s, e0, e1);
}
void launch_cholesky_part(const DevProblem& P, int part, unsigned epoch, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    if (P.npad == 0) return;
    CholFlow a = make_flow(P, epoch);
    if (part == 1) {
        a.tasks = P.cf_tasks2; a.task_i = P.cf_task_i2; a.task_t = P.cf_task_t2; a.pl0 = P.cf_pl02;
        a.plist = P.cf_plist2; a.plist_t = P.cf_plist_t2; a.ntasks = P.cf_ntasks2;
        a.head = P.cf_head + 1;
    }
    launch_flow(a, P, s, e0, e1);
}
int update_grid(const DevProblem& P, int eval) {
    return P.n_upd_blocks + ((eval && P.fuse_eval) ? cdiv(P.n_prior + P.n_vel, UPD_THREADS) : 0);
}
int update_resident_blocks(int device) {
    int per_cu = 0, ncu = 0;
    int per_cu32 = 0;   // (the fp32-residual instantiation too: the fused evaluation needs either resident at once)
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_update<false>, UPD_THREADS, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu32, k_update<true>, UPD_THREADS, 0) != hipSuccess)
        return 0;
    per_cu = per_cu < per_cu32 ? per_cu : per_cu32;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
    return per_cu * ncu;
}
void launch_update(const DevProblem& P, double lambda, int sel, int gate, int jac, hipStream_t s, int eval,
                   unsigned epoch) {
    const int fused = eval && P.fuse_eval;
    const int nb = P.n_upd_blocks + (fused ? cdiv(P.n_prior + P.n_vel, UPD_THREADS) : 0);
    hipLaunchKernelGGL(P.f32res ? k_update<true> : k_update<false>, dim3(nb), dim3(UPD_THREADS), 0, s, P, lambda, sel,
                       gate, jac, fused, epoch);
}
void launch_eval(const DevProblem& P, int sel, int gate, unsigned long long seq, int mode, hipStream_t s) {
    const int nb = P.n_tiles + cdiv(P.n_prior + P.n_vel + P.n_eprior, TILE_OBS);
    if (nb) hipLaunchKernelGGL(P.f32res ? k_eval<true> : k_eval<false>, dim3(nb), dim3(TILE_OBS), 0, s, P, sel, gate);
    if (mode != FIN_NONE) launch_finalize(P, seq, mode, s);
}
void launch_partials(const DevProblem& P, hipStream_t s) {
    hipLaunchKernelGGL(k_partials, dim3(1), dim3(256), 0, s, P);
}
void launch_env_pack(const DevProblem& P, int unpack, int gate, hipStream_t s) {
    hipLaunchKernelGGL(k_env_pack, dim3(8), dim3(256), 0, s, P, unpack, gate);
}
void launch_finalize(const DevProblem& P, unsigned long long seq, int mode, hipStream_t s) {
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(256), 0, s, P, seq, mode);
}
void launch_ctl_init(const DevProblem& P, const LMCtl& c, hipStream_t s) {
    hipLaunchKernelGGL(k_ctl_init, dim3(1), dim3(64), 0, s, P, c);
}
void launch_lambda_init(const DevProblem& P, double tau, hipStream_t s) {
    hipLaunchKernelGGL(k_lambda_init, dim3(1), dim3(1024), 0, s, P, tau);
}
void launch_depth(const DevProblem& P, int sel, unsigned char* ok, hipStream_t s) {
    if (P.n_obs) hipLaunchKernelGGL(k_depth, dim3(cdiv(P.n_obs, 256)), dim3(256), 0, s, P, sel, ok);
}

// ---- window farm (lba_farm_exchange): device-resident pack / unpack of the shared vertex estimates.
// Pack: this rank's published keyframes (q t v: FARM_KF doubles each) and landmarks (3 each) from the
// current state buffer into its slot of the exchange buffer; unpack: every vertex another rank owns,
// from that rank's slot (src: offset in the buffer), a bit-exact copy of the owner's estimate.
__global__ __launch_bounds__(256) void k_farm_pack(const double* __restrict__ kst, const double* __restrict__ lst,
                                                   const int* __restrict__ pub_kf, int npk,
                                                   const int* __restrict__ pub_lm, int npl, int kcap,
                                                   double* __restrict__ out) {
    const int nk = npk * FARM_KF, n = nk + 3 * npl;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
        if (e < nk) {
            const int i = e / FARM_KF, c = e - FARM_KF * i;
            out[e] = kst[(size_t)pub_kf[i] * KF_STRIDE + c];
        } else {
            const int j = (e - nk) / 3, c = (e - nk) - 3 * j;
            out[(size_t)kcap * FARM_KF + 3 * j + c] = lst[(size_t)pub_lm[j] * 3 + c];
        }
    }
}
__global__ __launch_bounds__(256) void k_farm_unpack(double* __restrict__ kst, double* __restrict__ lst,
                                                     const int* __restrict__ rkf, int nrk,
                                                     const int* __restrict__ rlm, int nrl,
                                                     const double* __restrict__ buf) {
    const int nk = nrk * FARM_KF, n = nk + 3 * nrl;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
        if (e < nk) {   // rkf: (destination KF, source offset) pairs
            const int i = e / FARM_KF, c = e - FARM_KF * i;
            kst[(size_t)rkf[2 * i] * KF_STRIDE + c] = buf[(size_t)rkf[2 * i + 1] + c];
        } else {
            const int j = (e - nk) / 3, c = (e - nk) - 3 * j;
            lst[(size_t)rlm[2 * j] * 3 + c] = buf[(size_t)rlm[2 * j + 1] + c];
        }
    }
}
void launch_farm_pack(const double* kst, const double* lst, const int* pub_kf, int npk, const int* pub_lm, int npl,
                      int kcap, double* out, hipStream_t s) {
    const int n = npk * FARM_KF + 3 * npl;
    if (n) hipLaunchKernelGGL(k_farm_pack, dim3(std::min(cdiv(n, 256), 1024)), dim3(256), 0, s, kst, lst, pub_kf, npk,
                              pub_lm, npl, kcap, out);
}
void launch_farm_unpack(double* kst, double* lst, const int* rkf, int nrk, const int* rlm, int nrl, const double* buf,
                        hipStream_t s) {
    const int n = nrk * FARM_KF + 3 * nrl;
    if (n) hipLaunchKernelGGL(k_farm_unpack, dim3(std::min(cdiv(n, 256), 1024)), dim3(256), 0, s, kst, lst, rkf, nrk,
                              rlm, nrl, buf);
}

}  // namespace lba
