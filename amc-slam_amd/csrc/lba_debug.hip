// lba_debug.hip — device-side evaluation of the Lie-group primitives the kernels run (lba_math.hpp: Sophus
// se3 exp / log with the epsilon = 1e-10 branches, Thirdparty/Sophus/sophus/se3.hpp:223-252,761-781,
// so3.hpp:247-290,583-618; Pose3utils' RightJacobianPose3 / RightJacobianPose3Inv with the theta <= 1e-5
// series of LeftJacobianPose3Q and the theta^2 <= DBL_EPSILON identity of LeftJacobianRot3(Inv),
// src/Pose3utils.cc:5-46,48-73).  A window whose motion is a straight line drives those branches only
// rarely through the LM kernels, so the parity tests also evaluate them here, on the GPU, at the golden
// tangents of tests/golden (lba_debug_lie, include/amc_lba.h).  Diagnostics: not on the LM path.
#include <hip/hip_runtime.h>

#include "../../include/amc_lba.h"
#include "lba_math.hpp"

using namespace lba;

namespace {

constexpr int LIE_IN = 13;    // xi[6], q[4], t[3]
constexpr int LIE_OUT = 85;   // exp(xi): q[4] t[3]; log(q, t)[6]; Jr(xi)[36]; Jr^-1(xi)[36]

__global__ __launch_bounds__(64) void k_debug_lie(const double* __restrict__ in, double* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* a = in + (size_t)i * LIE_IN;
    double* o = out + (size_t)i * LIE_OUT;
    double xi[6];
    for (int k = 0; k < 6; ++k) xi[k] = a[k];
    const SE3 T = se3_exp(xi);
    o[0] = T.q.x; o[1] = T.q.y; o[2] = T.q.z; o[3] = T.q.w;
    o[4] = T.t[0]; o[5] = T.t[1]; o[6] = T.t[2];
    SE3 G;
    G.q = Quat{a[6], a[7], a[8], a[9]};
    G.t[0] = a[10]; G.t[1] = a[11]; G.t[2] = a[12];
    se3_log(G, o + 7);
    double J[9], Q[9];
    right_jac_blocks(xi, J, Q);   // Jr(xi) = [J, Q; 0, J]
    double* Jr = o + 13;
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c) {
            double v = 0.0;
            if (r < 3 && c < 3) v = J[r * 3 + c];
            else if (r < 3) v = Q[r * 3 + c - 3];
            else if (c >= 3) v = J[(r - 3) * 3 + c - 3];
            Jr[r * 6 + c] = v;
        }
    right_jac_inv(xi, o + 49);
}

}  // namespace

extern "C" int lba_debug_lie(int32_t device, int32_t n, const double* in, double* out) {
    if (n < 0 || (n > 0 && (!in || !out))) return LBA_E_ARG;
    if (n == 0) return LBA_OK;
    if (hipSetDevice(device) != hipSuccess) return LBA_E_HIP;
    double *d_in = nullptr, *d_out = nullptr;
    int rc = LBA_OK;
    if (hipMalloc(&d_in, sizeof(double) * LIE_IN * n) != hipSuccess ||
        hipMalloc(&d_out, sizeof(double) * LIE_OUT * n) != hipSuccess) {
        rc = LBA_E_HIP;
    } else if (hipMemcpy(d_in, in, sizeof(double) * LIE_IN * n, hipMemcpyHostToDevice) != hipSuccess) {
        rc = LBA_E_HIP;
    } else {
        hipLaunchKernelGGL(k_debug_lie, dim3((n + 63) / 64), dim3(64), 0, 0, d_in, d_out, n);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(out, d_out, sizeof(double) * LIE_OUT * n, hipMemcpyDeviceToHost) != hipSuccess)
            rc = LBA_E_HIP;
    }
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return rc;
}
