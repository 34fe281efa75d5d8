// The stacked 64 x 32 panel factorisation of k_chol_flow (factor_pipe) at the current build, stage by stage (first
// half, cross update, second half: clock64 of one wave), and variants of the cross update between the halves:
//   cur  lba::cross_update (4 row tiles x 4 k-steps of v_mfma_f64_16x16x4)
//   skip the same without row tile 0 (rows 0..15, columns 16..31: above the diagonal of L_jj, never read)
//   fold skip with its k-steps 0..2 issued inside the first half's pivot sequence (piv_pipe_x)
//   help skip on a second wave (another SIMD's matrix core), fed column groups through LDS flags (piv_pipe_h)
// Results of every variant are compared bitwise with factor_pipe's on the entries the kernel reads (rows 32..63 and
// the lower triangle of rows 0..31).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 factor_stages.hip -o /tmp/fs && /tmp/fs
#include "../../amc-slam_amd/csrc/lba_kernels.hip"

#include <cstdio>
#include <cstring>

namespace {
using lba::CNB;

// cross_update without row tile 0
__device__ __forceinline__ void cross_skip(double (&row)[CNB], double (*st)[CNB + 1], int lane, double dg0, double* dg2) {
#pragma unroll
    for (int c = 0; c < 16; ++c) st[lane][c] = row[c];
    lba::wave_sync();
    const int lr = lane & 15, kq = lane >> 4;
    lba::d4 acc[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[t] = lba::d4{0.0, 0.0, 0.0, 0.0};
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
    lba::wave_sync();
    *dg2 = dg0 - st[lane][lane & 31];
#pragma unroll
    for (int c = 0; c < 16; ++c) row[16 + c] -= st[lane][16 + c];
}


// piv_pipe with the cross update's k-steps folded in: columns 4 ks .. 4 ks + 3 are final once pivot 4 ks + 3 has
// scaled its column, so they go to LDS at that pivot, the MFMA operands are read one pivot later and the k-step's
// three MFMAs issue one pivot after that, on the matrix core beside the pivot chain (same operands, same order:
// bitwise the separate cross update)
template <int J, int E>
__device__ __forceinline__ void piv_pipe_x(double (&row)[CNB], double rn, double dg, double lp, double rp, int lane,
                                           double (*st)[CNB + 1], lba::d4 (&acc)[3], double (&op)[3]) {
    constexpr int B = E - 16;
    if constexpr (J < E) {
        const double lij = row[J] * rn;
        row[J] = lij;
        if constexpr (J + 1 < E) {
            const double own = dg - lij * lij;
            const double dgn = fma(-lij, lij, dg);
            double rep = 0.0;
            if constexpr (J + 2 < E) rep = lba::rep16<B>(lij, lane);
            __builtin_amdgcn_sched_barrier(0);
            const int lr = lane & 15, kq = lane >> 4;
            if constexpr (J % 4 == 3) {
#pragma unroll
                for (int c = J - 3; c <= J; ++c) st[lane][c] = row[c];
            }
            if constexpr (J >= 4 && J % 4 == 0) {
#pragma unroll
                for (int t = 0; t < 3; ++t) op[t] = st[16 * (t + 1) + lr][J - 4 + kq];
            }
            if constexpr (J >= 5 && J % 4 == 1) {
#pragma unroll
                for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(op[t], op[0], acc[t], 0, 0, 0);
            }
            const double sL = lba::readlane_d(lij, J + 1);
            double c = __builtin_amdgcn_rsq(own);
            lba::pin(c);
            lba::pipe_defer<J, E, 0>(row, rp, lp);
            double t = own * c;
            lba::pin(t);
            lba::pipe_defer<J, E, 1>(row, rp, lp);
            double e = fma(-t, c, 1.0);
            lba::pin(e);
            lba::pipe_defer<J, E, 2>(row, rp, lp);
            t = fma(0.375, e, 0.5);
            const double m = c * e;
            lba::pin(t);
            lba::pipe_defer<J, E, 3>(row, rp, lp);
            c = fma(m, t, c);
            lba::pin(c);
            lba::pipe_defer<J, E, 4>(row, rp, lp);
            row[J + 1] = fma(-lij, sL, row[J + 1]);
            const double rnn = lba::readlane_d(c, J + 1);
            piv_pipe_x<J + 1, E>(row, rnn, dgn, lij, rep, lane, st, acc, op);
        }
    }
}

// the cross update's last k-step (columns 12..15) and the product's way back to rows
__device__ __forceinline__ void cross_tail(double (&row)[CNB], double (*st)[CNB + 1], int lane, double dg0, double* dg2,
                                           lba::d4 (&acc)[3]) {
#pragma unroll
    for (int c = 12; c < 16; ++c) st[lane][c] = row[c];
    lba::wave_sync();
    const int lr = lane & 15, kq = lane >> 4;
    double op[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) op[t] = st[16 * (t + 1) + lr][12 + kq];
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(op[t], op[0], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) st[16 * (t + 1) + kq + 4 * q][16 + lr] = acc[t][q];
    lba::wave_sync();
    *dg2 = dg0 - st[lane][lane & 31];
#pragma unroll
    for (int c = 0; c < 16; ++c) row[16 + c] -= st[lane][16 + c];
}

template <int V>
__global__ __launch_bounds__(64) void k_stages(const double* A, double* out, unsigned long long* cyc, int reps) {
    __shared__ double st[2 * CNB][CNB + 1];
    const int lane = threadIdx.x;
    unsigned long long h1 = 0, cr = 0, h2 = 0, tot = 0;
    for (int rp = 0; rp < reps; ++rp) {
        for (int c = 0; c < CNB; ++c) st[lane][c] = A[lane * CNB + c];
        lba::wave_sync();
        const unsigned long long c00 = clock64();
        double row[CNB];
#pragma unroll
        for (int c = 0; c < CNB; ++c) row[c] = st[lane][c];
        const double dg0 = st[lane][lane & 31];
        lba::pin(row[0]);
        const unsigned long long c0 = clock64();
        lba::d4 acc[3];
        double op[3];
        if constexpr (V == 2) {
#pragma unroll
            for (int t = 0; t < 3; ++t) acc[t] = lba::d4{0.0, 0.0, 0.0, 0.0};
            piv_pipe_x<0, 16>(row, lba::readlane_d(lba::rsqrt_nr(row[0]), 0), dg0, 0.0, 0.0, lane, st, acc, op);
        } else {
            lba::piv_pipe<0, 16>(row, lba::readlane_d(lba::rsqrt_nr(row[0]), 0), dg0, 0.0, 0.0, lane);
        }
        lba::pin(row[15]);
        const unsigned long long c1 = clock64();
        double dg2 = 0.0;
        if constexpr (V == 0) lba::cross_update(row, st, lane, dg0, &dg2);
        else if constexpr (V == 1) cross_skip(row, st, lane, dg0, &dg2);
        else cross_tail(row, st, lane, dg0, &dg2, acc);
        lba::pin(row[16]);
        const unsigned long long c2 = clock64();
        lba::piv_pipe<16, CNB>(row, lba::readlane_d(lba::rsqrt_nr(row[16]), 16), dg2, 0.0, 0.0, lane);
        lba::pin(row[31]);
        const unsigned long long c3 = clock64();
#pragma unroll
        for (int c = 0; c < CNB; ++c) st[lane][c] = row[c];
        lba::wave_sync();
        const unsigned long long c4 = clock64();
        h1 += c1 - c0; cr += c2 - c1; h2 += c3 - c2; tot += c4 - c00;
        for (int c = 0; c < CNB; ++c) out[lane * CNB + c] = st[lane][c];
    }
    if (lane == 0) { cyc[0] = h1 / reps; cyc[1] = cr / reps; cyc[2] = h2 / reps; cyc[3] = tot / reps; }
}


// piv_pipe with the hand-over of columns 4 ks .. 4 ks + 3 to a helper wave (on another SIMD) at pivot 4 ks + 3
template <int J, int E>
__device__ __forceinline__ void piv_pipe_h(double (&row)[CNB], double rn, double dg, double lp, double rp, int lane,
                                           double (*st)[CNB + 1], int* xf) {
    constexpr int B = E - 16;
    if constexpr (J < E) {
        const double lij = row[J] * rn;
        row[J] = lij;
        if constexpr (J + 1 < E) {
            const double own = dg - lij * lij;
            const double dgn = fma(-lij, lij, dg);
            double rep = 0.0;
            if constexpr (J + 2 < E) rep = lba::rep16<B>(lij, lane);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (J % 4 == 3) {
#pragma unroll
                for (int c = J - 3; c <= J; ++c) st[lane][c] = row[c];
                asm volatile("" ::: "memory");
                if (lane == 0) __hip_atomic_store(xf, (J + 1) / 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            const double sL = lba::readlane_d(lij, J + 1);
            double c = __builtin_amdgcn_rsq(own);
            lba::pin(c);
            lba::pipe_defer<J, E, 0>(row, rp, lp);
            double t = own * c;
            lba::pin(t);
            lba::pipe_defer<J, E, 1>(row, rp, lp);
            double e = fma(-t, c, 1.0);
            lba::pin(e);
            lba::pipe_defer<J, E, 2>(row, rp, lp);
            t = fma(0.375, e, 0.5);
            const double m = c * e;
            lba::pin(t);
            lba::pipe_defer<J, E, 3>(row, rp, lp);
            c = fma(m, t, c);
            lba::pin(c);
            lba::pipe_defer<J, E, 4>(row, rp, lp);
            row[J + 1] = fma(-lij, sL, row[J + 1]);
            const double rnn = lba::readlane_d(c, J + 1);
            piv_pipe_h<J + 1, E>(row, rnn, dgn, lij, rep, lane, st, xf);
        }
    }
}

// the helper wave: each k-step's three MFMAs once its columns are handed over, then the product out to columns
// 16..31 of rows 16..63 and the flag
__device__ __forceinline__ void cross_helper(double (*st)[CNB + 1], int lane, int* xf) {
    const int lr = lane & 15, kq = lane >> 4;
    lba::d4 acc[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[t] = lba::d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        while (__hip_atomic_load(xf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < ks + 1) __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        double op[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) op[t] = st[16 * (t + 1) + lr][4 * ks + kq];
#pragma unroll
        for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(op[t], op[0], acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) st[16 * (t + 1) + kq + 4 * q][16 + lr] = acc[t][q];
    asm volatile("" ::: "memory");
    if (lane == 0) __hip_atomic_store(xf + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__global__ __launch_bounds__(128) void k_helper(const double* A, double* out, unsigned long long* cyc, int reps) {
    __shared__ double st[2 * CNB][CNB + 1];
    __shared__ int xf[2];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long h1 = 0, cr = 0, h2 = 0, tot = 0;
    for (int rp = 0; rp < reps; ++rp) {
        if (wave == 0) for (int c = 0; c < CNB; ++c) st[lane][c] = A[lane * CNB + c];
        if (threadIdx.x == 0) { xf[0] = 0; xf[1] = 0; }
        __syncthreads();
        if (wave == 1) {
            cross_helper(st, lane, xf);
        } else {
            const unsigned long long c00 = clock64();
            double row[CNB];
#pragma unroll
            for (int c = 0; c < CNB; ++c) row[c] = st[lane][c];
            const double dg0 = st[lane][lane & 31];
            lba::pin(row[0]);
            const unsigned long long c0 = clock64();
            piv_pipe_h<0, 16>(row, lba::readlane_d(lba::rsqrt_nr(row[0]), 0), dg0, 0.0, 0.0, lane, st, xf);
#pragma unroll
            for (int c = 12; c < 16; ++c) st[lane][c] = row[c];
            asm volatile("" ::: "memory");
            if (lane == 0) __hip_atomic_store(xf, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            lba::pin(row[15]);
            const unsigned long long c1 = clock64();
            while (__hip_atomic_load(xf + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
            asm volatile("" ::: "memory");
            const double dg2 = dg0 - st[lane][lane & 31];
#pragma unroll
            for (int c = 0; c < 16; ++c) row[16 + c] -= st[lane][16 + c];
            lba::pin(row[16]);
            const unsigned long long c2 = clock64();
            lba::piv_pipe<16, CNB>(row, lba::readlane_d(lba::rsqrt_nr(row[16]), 16), dg2, 0.0, 0.0, lane);
            lba::pin(row[31]);
            const unsigned long long c3 = clock64();
#pragma unroll
            for (int c = 0; c < CNB; ++c) st[lane][c] = row[c];
            lba::wave_sync();
            const unsigned long long c4 = clock64();
            h1 += c1 - c0; cr += c2 - c1; h2 += c3 - c2; tot += c4 - c00;
            for (int c = 0; c < CNB; ++c) out[lane * CNB + c] = st[lane][c];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { cyc[0] = h1 / reps; cyc[1] = cr / reps; cyc[2] = h2 / reps; cyc[3] = tot / reps; }
}

// 16 (or 12) dependent-free fp64 MFMAs back to back, 4 (or 3) accumulators: the cross update's matrix-core floor
template <int T>
__global__ __launch_bounds__(64) void k_mfma(const double* A, double* out, unsigned long long* cyc, int reps) {
    const int lane = threadIdx.x;
    double a = A[lane], b = A[64 + lane];
    unsigned long long tot = 0;
    lba::d4 acc[4];
    for (int t = 0; t < 4; ++t) acc[t] = lba::d4{0.0, 0.0, 0.0, 0.0};
    for (int rp = 0; rp < reps; ++rp) {
        const unsigned long long c0 = clock64();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
            for (int t = 0; t < T; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
        asm volatile("" : "+v"(acc[0]));
        asm volatile("" : "+v"(acc[T - 1]));
        tot += clock64() - c0;
    }
    double s = 0.0;
    for (int t = 0; t < T; ++t) s += acc[t][0] + acc[t][3];
    out[lane] = s;
    if (lane == 0) cyc[0] = tot / reps;
}
}  // namespace

int main() {
    double *A, *F0, *F1, *F2, *F3;
    unsigned long long* cyc;
    (void)hipMalloc(&cyc, 64 * 8);
    (void)hipMalloc(&A, 64 * 32 * 8);
    (void)hipMalloc(&F0, 64 * 32 * 8);
    (void)hipMalloc(&F1, 64 * 32 * 8);
    (void)hipMalloc(&F2, 64 * 32 * 8);
    (void)hipMalloc(&F3, 64 * 32 * 8);
    double h[64 * 32];
    unsigned s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) / 16777216.0 - 0.5; };
    double G[32][40];
    for (int r = 0; r < 32; ++r)
        for (int k = 0; k < 40; ++k) G[r][k] = rnd();
    for (int r = 0; r < 32; ++r)
        for (int c = 0; c < 32; ++c) {
            double v = r == c ? 0.5 : 0.0;
            for (int k = 0; k < 40; ++k) v += G[r][k] * G[c][k];
            h[r * 32 + c] = v;
        }
    for (int r = 32; r < 64; ++r)
        for (int c = 0; c < 32; ++c) h[r * 32 + c] = rnd();
    (void)hipMemcpy(A, h, sizeof h, hipMemcpyHostToDevice);
    const char* names[4] = {"cur ", "skip", "fold", "help"};
    for (int rep = 0; rep < 3; ++rep)
        for (int v = 0; v < 4; ++v) {
            if (v == 0) k_stages<0><<<1, 64>>>(A, F0, cyc, 50);
            else if (v == 1) k_stages<1><<<1, 64>>>(A, F1, cyc, 50);
            else if (v == 2) k_stages<2><<<1, 64>>>(A, F2, cyc, 50);
            else k_helper<<<1, 128>>>(A, F3, cyc, 50);
            if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
            unsigned long long hh[4];
            (void)hipMemcpy(hh, cyc, 32, hipMemcpyDeviceToHost);
            printf("%s: first half %llu, cross update %llu, second half %llu, whole %llu cycles\n", names[v], hh[0], hh[1],
                   hh[2], hh[3]);
        }
    for (int rep = 0; rep < 2; ++rep) {
        unsigned long long c16, c12;
        k_mfma<4><<<1, 64>>>(A, F0 + 0, cyc, 50);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&c16, cyc, 8, hipMemcpyDeviceToHost);
        k_mfma<3><<<1, 64>>>(A, F0 + 0, cyc, 50);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&c12, cyc, 8, hipMemcpyDeviceToHost);
        printf("16 fp64 MFMAs %llu cycles, 12: %llu cycles\n", c16, c12);
    }
    // (k_mfma wrote F0: recompute the reference)
    k_stages<0><<<1, 64>>>(A, F0, cyc, 1);
    k_stages<1><<<1, 64>>>(A, F1, cyc, 1);
    k_stages<2><<<1, 64>>>(A, F2, cyc, 1);
    k_helper<<<1, 128>>>(A, F3, cyc, 1);
    (void)hipDeviceSynchronize();
    double f3[64 * 32];
    (void)hipMemcpy(f3, F3, sizeof f3, hipMemcpyDeviceToHost);
    double f0[64 * 32], f1[64 * 32], f2[64 * 32];
    (void)hipMemcpy(f0, F0, sizeof f0, hipMemcpyDeviceToHost);
    (void)hipMemcpy(f1, F1, sizeof f1, hipMemcpyDeviceToHost);
    (void)hipMemcpy(f2, F2, sizeof f2, hipMemcpyDeviceToHost);
    int nbit = 0, nbit2 = 0, nbit3 = 0;
    for (int r = 0; r < 64; ++r)
        for (int c = 0; c < 32; ++c)
            if (r >= 32 || c <= r) {
                nbit += memcmp(&f0[r * 32 + c], &f1[r * 32 + c], 8) != 0;
                nbit2 += memcmp(&f0[r * 32 + c], &f2[r * 32 + c], 8) != 0;
                nbit3 += memcmp(&f0[r * 32 + c], &f3[r * 32 + c], 8) != 0;
            }
    printf("read entries that differ bitwise from cur: skip %d, fold %d, help %d\n", nbit, nbit2, nbit3);
    return 0;
}
