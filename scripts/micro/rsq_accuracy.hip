// Accuracy of v_rsq_f64 and of its refinements (one Newton step, two Newton steps, one cubic step)
// against 1/sqrt in long double on the host.  hipcc --offload-arch=gfx950 -O3 rsq_accuracy.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include <random>

__global__ void k(const double* d, double* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x = d[i];
    double r = __builtin_amdgcn_rsq(x);
    out[4 * i] = r;
    double hh = 0.5 * x;
    double n1 = r * (1.5 - r * (hh * r));
    out[4 * i + 1] = n1;
    out[4 * i + 2] = n1 * (1.5 - n1 * (hh * n1));
    double t = x * r, e = fma(-t, r, 1.0), p = fma(0.375, e, 0.5), ce = r * e;
    out[4 * i + 3] = fma(ce, p, r);
}

int main() {
    const int n = 1 << 20;
    std::vector<double> h(n);
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> U(-30.0, 30.0), M(1.0, 2.0);
    for (int i = 0; i < n; ++i) h[i] = M(g) * std::ldexp(1.0, (int)U(g));
    double *dd, *dout;
    hipMalloc(&dd, n * 8); hipMalloc(&dout, 4 * n * 8);
    hipMemcpy(dd, h.data(), n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dd, dout, n);
    std::vector<double> o(4 * n);
    hipMemcpy(o.data(), dout, 4 * n * 8, hipMemcpyDeviceToHost);
    const char* names[4] = {"rsq", "rsq+newton", "rsq+2 newton", "rsq+cubic"};
    for (int v = 0; v < 4; ++v) {
        long double maxrel = 0; double maxulp = 0;
        for (int i = 0; i < n; ++i) {
            long double ref = 1.0L / sqrtl((long double)h[i]);
            long double rel = fabsl((o[4 * i + v] - ref) / ref);
            if (rel > maxrel) maxrel = rel;
            double ulp = (double)(rel / 2.220446049250313e-16L);
            if (ulp > maxulp) maxulp = ulp;
        }
        printf("%-14s max rel %.3Le  (%.2f ulp)\n", names[v], maxrel, maxulp);
    }
    return 0;
}
