// (Builds against the kernels of commit f8904ce or earlier: piv_seq and factor_pair were removed from the product
// library in round 5; `git show f8904ce:amc-slam_amd/csrc/lba_kernels.hip` restores the version it includes.)
// Single-wave instruction costs on gfx950 (one workgroup of 64 threads on an otherwise idle GPU), in
// clock64 cycles per instruction: fp64 FMA (independent / dependent chain), v_readlane_b32 pairs feeding
// an FMA, DPP64 row-broadcast FMA, ds_bpermute pairs; and the stacked 64 x 32 panel factorisation of
// k_chol_flow with readlane or DPP64 broadcasts (LBA_CHOL_DPP).  Builds against the library's kernels file (the device functions are there).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DLBA_CHOL_DPP=0 piv_cost.hip -o /tmp/pc0
#include "../../amc-slam_amd/csrc/lba_kernels.hip"

#include <cstdio>

namespace {
constexpr int N = 256;

__global__ __launch_bounds__(64) void k_ops(double* out, unsigned long long* cyc, double a0) {
    const int lane = threadIdx.x;
    double x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = a0 + j + lane;
    double r = a0 * lane;
    // 1. independent FMAs (8 chains)
    unsigned long long c0 = clock64();
    for (int i = 0; i < N / 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) { x[j] = fma(x[j], 1.0000001, 1e-7); lba::pin(x[j]); }
    unsigned long long c1 = clock64();
    // 2. dependent FMA chain
    for (int i = 0; i < N; ++i) { r = fma(r, 1.0000001, 1e-7); lba::pin(r); }
    unsigned long long c2 = clock64();
    // 3. readlane_d broadcast + FMA (the original rank-1 update step)
    for (int i = 0; i < N / 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) { x[j] = fma(-r, lba::readlane_d(x[(j + 1) & 7], j), x[j]); lba::pin(x[j]); }
    unsigned long long c3 = clock64();
    // 4. DPP64 row-broadcast FMA
    for (int i = 0; i < N / 8; ++i) {
        lba::fmac_bcast<1>(x[0], x[7], r); lba::fmac_bcast<2>(x[1], x[7], r);
        lba::fmac_bcast<3>(x[2], x[7], r); lba::fmac_bcast<4>(x[3], x[7], r);
        lba::fmac_bcast<5>(x[4], x[7], r); lba::fmac_bcast<6>(x[5], x[7], r);
        lba::fmac_bcast<7>(x[6], x[0], r); lba::fmac_bcast<8>(x[7], x[1], r);
    }
    unsigned long long c4 = clock64();
    // 5. ds_bpermute pairs (rep16), dependent
    for (int i = 0; i < N / 8; ++i) { r = lba::rep16<0>(r, lane) + 1e-9; lba::pin(r); }
    unsigned long long c5 = clock64();
    double s = r;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
    if (s == 1.2345) out[0] = s;
    if (lane == 0) {
        cyc[0] = (c1 - c0);
        cyc[1] = (c2 - c1);
        cyc[2] = (c3 - c2);
        cyc[3] = (c4 - c3);
        cyc[4] = (c5 - c4);
    }
}

// the stacked panel factorisation exactly as k_chol_flow's factor lambda (two halves + cross update)
__global__ __launch_bounds__(64) void k_factor(const double* A, double* out, unsigned long long* cyc, int reps) {
    __shared__ double st[2 * lba::CNB][lba::CNB + 1];
    const int lane = threadIdx.x;
    unsigned long long tot = 0, h1 = 0, cr = 0;
    for (int rp = 0; rp < reps; ++rp) {
        for (int c = 0; c < lba::CNB; ++c) st[lane][c] = A[lane * lba::CNB + c];
        lba::wave_sync();
        double row[lba::CNB];
#pragma unroll
        for (int c = 0; c < lba::CNB; ++c) row[c] = st[lane][c];
        bool bad = false;
        lba::pin(row[0]);
        const unsigned long long c0 = clock64();
        lba::piv_seq<0, 16>(row, lba::readlane_d(lba::rsqrt_nr(row[0]), 0), lane, bad);
        lba::pin(row[15]);
        const unsigned long long c1 = clock64();
        lba::cross_update(row, st, lane);
        lba::pin(row[16]);
        const unsigned long long c2 = clock64();
        lba::piv_seq<16, lba::CNB>(row, lba::readlane_d(lba::rsqrt_nr(row[16]), 16), lane, bad);
        lba::pin(row[31]);
        const unsigned long long c3 = clock64();
        tot += c3 - c0;
        h1 += c1 - c0;
        cr += c2 - c1;
#pragma unroll
        for (int c = 0; c < lba::CNB; ++c) out[lane * lba::CNB + c] = row[c];
        if (bad) out[0] = -1.0;
    }
    if (lane == 0) { cyc[0] = tot / reps; cyc[1] = h1 / reps; cyc[2] = cr / reps; }
}
}  // namespace

int main() {
    double *o, *A, *F;
    unsigned long long* cyc;
    (void)hipMalloc(&o, 64 * 8);
    (void)hipMalloc(&cyc, 64 * 8);
    (void)hipMalloc(&A, 64 * 32 * 8);
    (void)hipMalloc(&F, 64 * 32 * 8);
    // SPD diagonal block (rows 0..31) and a tile below (rows 32..63)
    double h[64 * 32];
    for (int r = 0; r < 64; ++r)
        for (int c = 0; c < 32; ++c) h[r * 32 + c] = (r == c) ? 40.0 + r : 1.0 / (1.0 + r + c);
    (void)hipMemcpy(A, h, sizeof h, hipMemcpyHostToDevice);
    unsigned long long hc[8];
    for (int rep = 0; rep < 3; ++rep) {
        k_ops<<<1, 64>>>(o, cyc, 1.0);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(hc, cyc, 5 * 8, hipMemcpyDeviceToHost);
        printf("cycles per op (single wave): fma indep %.2f  fma dep %.2f  readlane_d+fma %.2f  fmac_dpp %.2f  "
               "rep16 dep %.2f\n", hc[0] / (double)N, hc[1] / (double)N, hc[2] / (double)N, hc[3] / (double)N,
               hc[4] / (double)(N / 8));
    }
    for (int rep = 0; rep < 3; ++rep) {
        k_factor<<<1, 64>>>(A, F, cyc, 20);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(hc, cyc, 24, hipMemcpyDeviceToHost);
        printf("stacked factor (DPP=%d%s): %llu cycles (first half %llu, cross update %llu)\n", LBA_CHOL_DPP,
#ifdef LBA_EXP_NO_UPDATE
               " chain only",
#else
               "",
#endif
               hc[0], hc[1], hc[2]);
    }
    double f[64 * 32];
    (void)hipMemcpy(f, F, sizeof f, hipMemcpyDeviceToHost);
    double cs = 0;
    for (int i = 0; i < 64 * 32; ++i) cs += f[i] * (1 + (i % 7));
    printf("checksum %.17g\n", cs);

    return 0;
}
