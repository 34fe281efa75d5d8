// Phase cost of gp_pair_prep (the GP-pair sample rebuild of k_update) in isolation: one 64-thread
// workgroup, synthetic pair, s_memrealtime stamps after each phase (the k_update stamps' layout), run
// repeatedly so the second and later launches show warm caches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 prep_cost.hip -o /tmp/prep_cost
#include "../../amc-slam_amd/csrc/lba_kernels.hip"

#include <cstdio>
#include <vector>

namespace {
__global__ void k_prep(lba::DevProblem P, const double* ka, const double* kb, double* gps, unsigned long long* st,
                       int reps) {
    for (int r = 0; r < reps; ++r) {
        if (threadIdx.x == 0) st[16 * r + 15] = __builtin_amdgcn_s_memrealtime();
        lba::gp_pair_prep(P, gps, 0, ka, kb, 1, st + 16 * r);
        __syncthreads();
        if (threadIdx.x == 0) st[16 * r + 14] = __builtin_amdgcn_s_memrealtime();
    }
}
}  // namespace

int main() {
    lba::DevProblem P{};
    const int ns = 3;
    int s0[2] = {0, ns};
    double ts[ns] = {100.03, 100.05, 100.07};
    double ka[16] = {0.01, -0.02, 0.03, 0.999, 1.0, 2.0, 1.5, 4.0, 0.1, 0, 0, 0, 0.1, 100.0, 60.0, 0};
    double kb[16] = {0.012, -0.019, 0.05, 0.998, 1.4, 2.1, 1.5, 4.1, 0.0, 0, 0, 0, 0.12, 100.1, 60.0, 0};
    int* d_s0;
    double *d_ts, *d_ka, *d_kb, *d_gps;
    unsigned long long* d_st;
    (void)hipMalloc(&d_s0, sizeof(s0));
    (void)hipMalloc(&d_ts, sizeof(ts));
    (void)hipMalloc(&d_ka, sizeof(ka));
    (void)hipMalloc(&d_kb, sizeof(kb));
    (void)hipMalloc(&d_gps, sizeof(double) * 156 * ns);
    const int reps = 4;
    (void)hipMalloc(&d_st, sizeof(unsigned long long) * 16 * reps);
    (void)hipMemcpy(d_s0, s0, sizeof(s0), hipMemcpyHostToDevice);
    (void)hipMemcpy(d_ts, ts, sizeof(ts), hipMemcpyHostToDevice);
    (void)hipMemcpy(d_ka, ka, sizeof(ka), hipMemcpyHostToDevice);
    (void)hipMemcpy(d_kb, kb, sizeof(kb), hipMemcpyHostToDevice);
    P.gp_s0 = d_s0;
    P.gps_t = d_ts;
    for (int launch = 0; launch < 3; ++launch) {
        hipLaunchKernelGGL(k_prep, dim3(1), dim3(64), 0, 0, P, d_ka, d_kb, d_gps, d_st, reps);
        (void)hipDeviceSynchronize();
        std::vector<unsigned long long> h(16 * reps);
        (void)hipMemcpy(h.data(), d_st, h.size() * 8, hipMemcpyDeviceToHost);
        for (int r = 0; r < reps; ++r) {
            const unsigned long long* x = h.data() + 16 * r;
            const unsigned long long c[7] = {x[15], x[0], x[1], x[2], x[3], x[4], x[5]};
            printf("launch %d rep %d (us): log+AdI %.2f  Jr^-1+ad %.2f  w2/A1 %.2f  B1/D %.2f  samples %.2f  N %.2f\n",
                   launch, r, (c[1] - c[0]) / 100.0, (c[2] - c[1]) / 100.0, (c[3] - c[2]) / 100.0,
                   (c[4] - c[3]) / 100.0, (c[5] - c[4]) / 100.0, (c[6] - c[5]) / 100.0);
        }
    }
    return 0;
}
