// Test-only probe (tests/test_gpu_parity.py::test_mfma_f64_layout): checks the lane layout of
// v_mfma_f64_16x16x4_f64 that k_schur's Schur products assume, with exact integer data.
//   A[i][k]: lane i + 16k;  B[k][j]: lane j + 16k;  C[i][j]: lane j + 16 (i % 4), register i / 4
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void probe(const double* A, const double* B, double* C) {
    const int l = threadIdx.x, i = l & 15, k = l >> 4;
    d4 c = {0.0, 0.0, 0.0, 0.0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(A[i * 4 + k], B[k * 16 + i], c, 0, 0, 0);
    for (int q = 0; q < 4; ++q) C[(k + 4 * q) * 16 + i] = c[q];
}

int main() {
    double hA[64], hB[64], hC[256], ref[256];
    for (int i = 0; i < 16; ++i)
        for (int k = 0; k < 4; ++k) hA[i * 4 + k] = (double)(i * 7 + k * 3 + 1);
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 16; ++j) hB[k * 16 + j] = (double)(k * 5 - j + 2);
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += hA[i * 4 + k] * hB[k * 16 + j];
            ref[i * 16 + j] = s;
        }
    double *dA, *dB, *dC;
    if (hipMalloc(&dA, sizeof hA) || hipMalloc(&dB, sizeof hB) || hipMalloc(&dC, sizeof hC)) return 2;
    (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    if (hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (int e = 0; e < 256; ++e) bad += hC[e] != ref[e];
    std::printf("mfma_f64_16x16x4 layout: %d / 256 mismatches\n", bad);
    return bad ? 1 : 0;
}
