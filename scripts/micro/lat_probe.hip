// Latency microbenchmark (diagnostics): cycles per dependent step of the operations on the
// Cholesky pivot chain, one wave, clock64() around 1024-step dependent chains.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double rl(double v, int lane) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, lane);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

__global__ void probe(double* out, long long* cyc, double seed) {
    const int lane = threadIdx.x;
    double a = seed + lane * 1e-3, b = 1.0000001;
    __shared__ double sh[64];
    long long t0, t1;
    // 1. dependent fp64 FMA
    t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < 1024; ++i) a = fma(a, b, 1e-9);
    t1 = clock64();
    if (lane == 0) cyc[0] = t1 - t0;
    // 2. dependent rsq_f64
    double r = a;
    t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < 1024; ++i) r = __builtin_amdgcn_rsq(r) + 0.5;
    t1 = clock64();
    if (lane == 0) cyc[1] = t1 - t0;
    // 3. dependent readlane(double) + fma
    double x = a;
    t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < 1024; ++i) x = fma(rl(x, i & 63), b, 1e-9);
    t1 = clock64();
    if (lane == 0) cyc[2] = t1 - t0;
    // 4. LDS write -> read round trip (same wave) + fma
    double y = a;
    t0 = clock64();
    for (int i = 0; i < 1024; ++i) {
        sh[lane] = y;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        y = fma(sh[(lane + 1) & 63], b, 1e-9);
    }
    t1 = clock64();
    if (lane == 0) cyc[3] = t1 - t0;
    // 5. independent fp64 FMA throughput (8 chains)
    double c[8];
    for (int k = 0; k < 8; ++k) c[k] = a + k;
    t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < 1024; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = fma(c[k], b, 1e-9);
    t1 = clock64();
    if (lane == 0) cyc[4] = t1 - t0;
    double s = 0;
    for (int k = 0; k < 8; ++k) s += c[k];
    out[lane] = a + r + x + y + s;
}

int main() {
    double* o;
    long long* c;
    if (hipMalloc(&o, 64 * 8) || hipMalloc(&c, 8 * 8)) return 2;
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, o, c, 1.5);
    long long h[8];
    if (hipMemcpy(h, c, 8 * 8, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    const char* names[5] = {"fma_f64 dependent", "rsq_f64 dependent (+add)", "readlane_d + fma dependent",
                            "LDS write->read + fma", "fma_f64 x8 independent (per fma)"};
    for (int k = 0; k < 5; ++k)
        std::printf("%-34s %7.1f cycles/step\n", names[k], h[k] / 1024.0 / (k == 4 ? 8.0 : 1.0));
    return 0;
}
