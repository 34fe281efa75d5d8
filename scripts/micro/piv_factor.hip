// (Builds against the kernels of commit f8904ce or earlier: piv_seq and factor_pair were removed from the product
// library in round 5; `git show f8904ce:amc-slam_amd/csrc/lba_kernels.hip` restores the version it includes.)
// The stacked 64 x 32 panel factorisation: the single-wave two-level sequence of k_chol_flow (piv_seq /
// cross_update / piv_seq), its software-pipelined form (factor_pipe) and the pair of waves (factor_pair), on an idle GPU: cycles (clock64 of wave 0 between two workgroup barriers) and both results
// against a long-double Cholesky on the host.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 piv_factor4.hip -o /tmp/pf4 && /tmp/pf4
#include "../../amc-slam_amd/csrc/lba_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstring>

namespace {
__global__ __launch_bounds__(256) void k_old(const double* A, double* out, unsigned long long* cyc, int reps) {
    __shared__ double st[2 * lba::CNB][lba::CNB + 1];
    const int tid = threadIdx.x, lane = tid & 63;
    unsigned long long tot = 0;
    for (int rp = 0; rp < reps; ++rp) {
        for (int e = tid; e < 64 * 32; e += 256) st[e >> 5][e & 31] = A[e];
        __syncthreads();
        const unsigned long long c0 = clock64();
        if (tid < 64) {
            double row[lba::CNB];
#pragma unroll
            for (int c = 0; c < lba::CNB; ++c) row[c] = st[lane][c];
            bool bad = lane == 0 && !(row[0] > 0.0);
            lba::piv_seq<0, 16>(row, lba::readlane_d(lba::rsqrt_nr(row[0]), 0), lane, bad);
            lba::cross_update(row, st, lane);
            bad = bad || (lane == 16 && !(row[16] > 0.0));
            lba::piv_seq<16, lba::CNB>(row, lba::readlane_d(lba::rsqrt_nr(row[16]), 16), lane, bad);
#pragma unroll
            for (int c = 0; c < lba::CNB; ++c) st[lane][c] = row[c];
        }
        __syncthreads();
        tot += clock64() - c0;
        for (int e = tid; e < 64 * 32; e += 256) out[e] = st[e >> 5][e & 31];
        __syncthreads();
    }
    if (tid == 0) cyc[0] = tot / reps;
}

__global__ __launch_bounds__(256) void k_pipe(const double* A, double* out, unsigned long long* cyc, int reps) {
    __shared__ double st[2 * lba::CNB][lba::CNB + 1];
    const int tid = threadIdx.x, lane = tid & 63;
    unsigned long long tot = 0;
    int badc = 0;
    for (int rp = 0; rp < reps; ++rp) {
        for (int e = tid; e < 64 * 32; e += 256) st[e >> 5][e & 31] = A[e];
        __syncthreads();
        const unsigned long long c0 = clock64();
        if (tid < 64) {
            bool bad;
            lba::factor_pipe(st, lane, bad);
            badc += __ballot(bad) != 0;
        }
        __syncthreads();
        tot += clock64() - c0;
        for (int e = tid; e < 64 * 32; e += 256) out[e] = st[e >> 5][e & 31];
        __syncthreads();
    }
    if (tid == 0) { cyc[0] = tot / reps; cyc[1] = badc; }
}

__global__ __launch_bounds__(128) void k_pair(const double* A, double* out, unsigned long long* cyc, int reps) {
    __shared__ double st[2 * lba::CNB][lba::CNB + 1];
    __shared__ double colbuf[lba::CNB][64];
    __shared__ int cflag[8];
    const int tid = threadIdx.x;
    if (tid < 8) cflag[tid] = 0;
    unsigned long long tot = 0;
    for (int rp = 0; rp < reps; ++rp) {
        for (int e = tid; e < 64 * 32; e += 128) st[e >> 5][e & 31] = A[e];
        __syncthreads();
        const unsigned long long c0 = clock64();
        bool bad;
        lba::factor_pair(st, colbuf, cflag, rp + 1, tid >> 6, bad);
        __syncthreads();
        tot += clock64() - c0;
        for (int e = tid; e < 64 * 32; e += 128) out[e] = st[e >> 5][e & 31];
        __syncthreads();
    }
    if (tid == 0) cyc[0] = tot / reps;
}

// factor_pair with stamps: wave a end, wave b consumption end (start of its pivots), wave b end
__global__ __launch_bounds__(128) void k_pair_t(const double* A, unsigned long long* cyc, int reps) {
    __shared__ double st[2 * lba::CNB][lba::CNB + 1];
    __shared__ double colbuf[lba::CNB][64];
    __shared__ int cflag[8];
    const int tid = threadIdx.x, lane = tid & 63, half = tid >> 6;
    if (tid < 8) cflag[tid] = 0;
    unsigned long long ta = 0, tb0 = 0, tb1 = 0;
    for (int rp = 0; rp < reps; ++rp) {
        for (int e = tid; e < 64 * 32; e += 128) st[e >> 5][e & 31] = A[e];
        __syncthreads();
        const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
        double row[lba::CNB];
        const double dg0 = st[lane][lane & 31];
        if (half == 0) {
#pragma unroll
            for (int c = 0; c < 16; ++c) row[c] = st[lane][c];
            lba::piv_pipe_pub<0>(row, lba::readlane_d(lba::rsqrt_nr(row[0]), 0), dg0, 0.0, 0.0, lane, colbuf, cflag, rp + 1);
            lba::pin(row[15]);
            ta += __builtin_amdgcn_s_memrealtime() - c0;
#pragma unroll
            for (int c = 0; c < 16; ++c) st[lane][c] = row[c];
        } else {
#pragma unroll
            for (int c = 16; c < lba::CNB; ++c) row[c] = st[lane][c];
            double dg = dg0;
            for (int g = 0; g < 16; g += lba::PAIR_GROUP) {
                while (__hip_atomic_load(cflag + g / lba::PAIR_GROUP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != rp + 1) {}
                asm volatile("" ::: "memory");
                lba::pair_consume<0>(row, dg, colbuf, g, lane);
            }
            lba::pin(row[16]);
            tb0 += __builtin_amdgcn_s_memrealtime() - c0;
            lba::piv_pipe<16, lba::CNB>(row, lba::readlane_d(lba::rsqrt_nr(row[16]), 16), dg, 0.0, 0.0, lane);
            lba::pin(row[31]);
            tb1 += __builtin_amdgcn_s_memrealtime() - c0;
#pragma unroll
            for (int c = 16; c < lba::CNB; ++c) st[lane][c] = row[c];
        }
        __syncthreads();
    }
    if (tid == 0) cyc[0] = ta / reps;
    if (tid == 64) { cyc[1] = tb0 / reps; cyc[2] = tb1 / reps; }
}

// factor_pipe's stages timed: first half, cross update, second half
__global__ __launch_bounds__(64) void k_pipe_t(const double* A, unsigned long long* cyc, int reps) {
    __shared__ double st[2 * lba::CNB][lba::CNB + 1];
    const int lane = threadIdx.x;
    unsigned long long h1 = 0, cr = 0, h2 = 0;
    for (int rp = 0; rp < reps; ++rp) {
        for (int c = 0; c < lba::CNB; ++c) st[lane][c] = A[lane * lba::CNB + c];
        lba::wave_sync();
        double row[lba::CNB];
#pragma unroll
        for (int c = 0; c < lba::CNB; ++c) row[c] = st[lane][c];
        const double dg0 = st[lane][lane & 31];
        lba::pin(row[0]);
        const unsigned long long c0 = clock64();
        lba::piv_pipe<0, 16>(row, lba::readlane_d(lba::rsqrt_nr(row[0]), 0), dg0, 0.0, 0.0, lane);
        lba::pin(row[15]);
        const unsigned long long c1 = clock64();
        double dg2 = 0.0;
        lba::cross_update(row, st, lane, dg0, &dg2);
        lba::pin(row[16]);
        const unsigned long long c2 = clock64();
        lba::piv_pipe<16, lba::CNB>(row, lba::readlane_d(lba::rsqrt_nr(row[16]), 16), dg2, 0.0, 0.0, lane);
        lba::pin(row[31]);
        const unsigned long long c3 = clock64();
        h1 += c1 - c0; cr += c2 - c1; h2 += c3 - c2;
        double sum = 0.0;
#pragma unroll
        for (int c = 0; c < lba::CNB; ++c) sum += row[c];
        if (sum == 1.2345) cyc[7] = 1;
    }
    if (lane == 0) { cyc[0] = h1 / reps; cyc[1] = cr / reps; cyc[2] = h2 / reps; }
}

}  // namespace

int main() {
    double *A, *F0, *F1, *F2;
    unsigned long long* cyc;
    (void)hipMalloc(&cyc, 64 * 8);
    (void)hipMalloc(&A, 64 * 32 * 8);
    (void)hipMalloc(&F0, 64 * 32 * 8);
    (void)hipMalloc(&F1, 64 * 32 * 8);
    (void)hipMalloc(&F2, 64 * 32 * 8);
    // SPD diagonal block (rows 0..31, a random Gram matrix + diagonal) and a random tile below (rows 32..63)
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
    // host reference: L of the diagonal block, L(i, j) = A(i, j) L^-T for the tile
    long double L[64][32] = {};
    for (int j = 0; j < 32; ++j) {
        long double d = h[j * 32 + j];
        for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k];
        L[j][j] = sqrtl(d);
        for (int i = j + 1; i < 64; ++i) {
            long double v = h[i * 32 + j];
            for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k];
            L[i][j] = v / L[j][j];
        }
    }
    unsigned long long hc[2];
    const char* names[3] = {"single wave (2-level, piv_seq)", "-", "single wave pipelined (factor_pipe)"};
    for (int pass = 0; pass < 3; pass += 2) {
        for (int rep = 0; rep < 3; ++rep) {
            if (pass == 0) k_old<<<1, 256>>>(A, F0, cyc, 20);
            else k_pipe<<<1, 256>>>(A, F2, cyc, 20);
            if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
            (void)hipMemcpy(hc, cyc, 16, hipMemcpyDeviceToHost);
            printf("%s: %llu cycles per stacked factorisation%s\n", names[pass], hc[0],
                   pass && hc[1] ? " BAD PIVOT REPORTED" : "");
        }
    }
    double f0[64 * 32], f1[64 * 32], f2[64 * 32];
    (void)hipMemcpy(f0, F0, sizeof f0, hipMemcpyDeviceToHost);
    (void)hipMemcpy(f1, F1, sizeof f1, hipMemcpyDeviceToHost);
    (void)hipMemcpy(f2, F2, sizeof f2, hipMemcpyDeviceToHost);
    for (int rep = 0; rep < 3; ++rep) {
        unsigned long long hh[3];
        k_pipe_t<<<1, 64>>>(A, cyc, 20);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(hh, cyc, 24, hipMemcpyDeviceToHost);
        printf("factor_pipe stages: first half %llu, cross update %llu, second half %llu cycles\n", hh[0], hh[1], hh[2]);
    }
    double *F3;
    (void)hipMalloc(&F3, 64 * 32 * 8);
    for (int rep = 0; rep < 3; ++rep) {
        k_pair<<<1, 128>>>(A, F3, cyc, 20);
        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
        (void)hipMemcpy(hc, cyc, 8, hipMemcpyDeviceToHost);
        printf("factor_pair (2 waves): %llu cycles per stacked factorisation\n", hc[0]);
    }
    {
        double f3[64 * 32];
        (void)hipMemcpy(f3, F3, sizeof f3, hipMemcpyDeviceToHost);
        double e3 = 0, mx3 = 0;
        for (int r = 0; r < 64; ++r)
            for (int c = 0; c < 32; ++c) {
                if (r < 32 && c > r) continue;
                mx3 = fmax(mx3, fabs((double)L[r][c]));
                e3 = fmax(e3, fabs(f3[r * 32 + c] - (double)L[r][c]));
            }
        printf("factor_pair max |L - L_ref| / max|L| = %.2e\n", e3 / mx3);
    }
    for (int rep = 0; rep < 3; ++rep) {
        unsigned long long hh[3];
        k_pair_t<<<1, 128>>>(A, cyc, 20);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(hh, cyc, 24, hipMemcpyDeviceToHost);
        printf("factor_pair stamps (s_memrealtime, 100 MHz ticks x 24 ~ cycles): wave a done %llu, wave b starts pivots %llu, done %llu\n", hh[0], hh[1], hh[2]);
    }
    int nbit = 0;
    for (int r = 0; r < 64; ++r)
        for (int c = 0; c < 32; ++c)
            if ((r >= 32 || c <= r) && memcmp(&f0[r * 32 + c], &f2[r * 32 + c], 8) != 0) ++nbit;
    printf("factor_pipe vs piv_seq: %d entries differ bitwise\n", nbit);
    double e0 = 0, e1 = 0, d01 = 0, mx = 0;
    for (int r = 0; r < 64; ++r)
        for (int c = 0; c < 32; ++c) {
            if (r < 32 && c > r) continue;
            const double ref = (double)L[r][c];
            mx = fmax(mx, fabs(ref));
            e0 = fmax(e0, fabs(f0[r * 32 + c] - ref));
            e1 = fmax(e1, fabs(f1[r * 32 + c] - ref));
            d01 = fmax(d01, fabs(f0[r * 32 + c] - f1[r * 32 + c]));
        }
    (void)e1; (void)d01;
    printf("max |L - L_ref| / max|L|: single wave %.2e\n", e0 / mx);
    return 0;
}
