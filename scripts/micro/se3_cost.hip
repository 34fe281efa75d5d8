// Single-lane cycle cost of the SE(3) maps on the k_update chain (gfx950): se3_exp, se3_log,
// right_jac_inv, sin / cos / sqrt / division alone (clock64, one wave, lane 0's chain).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 se3_cost.hip -o /tmp/se3_cost
#include "../../amc-slam_amd/csrc/lba_kernels.hip"

#include <cstdio>

namespace {
__global__ void k_cost(const double* in, double* out, unsigned long long* cyc) {
    if (threadIdx.x != 0) return;
    double xi[6];
    for (int i = 0; i < 6; ++i) xi[i] = in[i];
    double acc = 0.0;
    unsigned long long t0 = clock64();
    lba::SE3 T = lba::se3_exp(xi);
    acc += T.q.x + T.t[0];
    lba::pin(acc);
    unsigned long long t1 = clock64();
    double lg[6];
    lba::se3_log(T, lg);
    acc += lg[0];
    lba::pin(acc);
    unsigned long long t2 = clock64();
    double J[36];
    lba::right_jac_inv(lg, J);
    acc += J[0] + J[35];
    lba::pin(acc);
    unsigned long long t3 = clock64();
    double s = sin(acc * 1e-3 + xi[0]);
    lba::pin(s);
    unsigned long long t4 = clock64();
    double c = cos(s);
    lba::pin(c);
    unsigned long long t5 = clock64();
    double q = sqrt(c + 2.0);
    lba::pin(q);
    unsigned long long t6 = clock64();
    double d = 1.0 / (q + xi[1]);
    lba::pin(d);
    unsigned long long t7 = clock64();
    double at = atan(d);
    lba::pin(at);
    unsigned long long t8 = clock64();
    out[0] = acc + s + c + q + d + at;
    cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; cyc[4] = t5 - t4;
    cyc[5] = t6 - t5; cyc[6] = t7 - t6; cyc[7] = t8 - t7;
}
}  // namespace

int main() {
    double h[6] = {0.1, -0.2, 0.3, 0.05, -0.04, 0.02}, *in, *out;
    unsigned long long *cyc, hc[8];
    (void)hipMalloc(&in, 48);
    (void)hipMalloc(&out, 8);
    (void)hipMalloc(&cyc, 64);
    (void)hipMemcpy(in, h, 48, hipMemcpyHostToDevice);
    for (int r = 0; r < 3; ++r) {
        k_cost<<<1, 64>>>(in, out, cyc);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(hc, cyc, 64, hipMemcpyDeviceToHost);
        printf("cycles: se3_exp %llu  se3_log %llu  right_jac_inv %llu  sin %llu  cos %llu  sqrt %llu  div %llu  atan %llu\n",
               hc[0], hc[1], hc[2], hc[3], hc[4], hc[5], hc[6], hc[7]);
    }
    return 0;
}
