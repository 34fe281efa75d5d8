// Launch-boundary floor on MI355X: back-to-back launches in one stream, timed with events.
//   empty 1-WG kernel; 1-WG kernel after a kernel that dirtied 1 MB; 100-WG kernel reading 1 MB.
// hipcc --offload-arch=gfx950 -O3 launch_floor.hip -o /tmp/launch_floor && /tmp/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int* p) { if (threadIdx.x == 0 && p[0] == 12345) p[1] = 1; }
__global__ void k_dirty(double* a, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) a[i] = a[i] + 1.0;
}
__global__ void k_read(const double* a, int n, double* o) {
    double s = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) s += a[i];
    if (s == 1234.5) o[0] = s;
}

int main() {
    int* p; double* a; double* o;
    (void)hipMalloc(&p, 64); (void)hipMemset(p, 0, 64);
    const int n = 1 << 17;   // 1 MB of doubles
    (void)hipMalloc(&a, n * 8); (void)hipMemset(a, 0, n * 8); (void)hipMalloc(&o, 64);
    hipStream_t s; (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    auto run = [&](const char* name, auto body, int reps) {
        for (int w = 0; w < 20; ++w) body();
        (void)hipStreamSynchronize(s);
        (void)hipEventRecord(e0, s);
        for (int r = 0; r < reps; ++r) body();
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-44s %8.2f us per launch\n", name, 1e3 * ms / reps);
    };
    run("empty 1-WG", [&] { hipLaunchKernelGGL(k_empty, 1, 64, 0, s, p); }, 2000);
    run("empty 256-WG", [&] { hipLaunchKernelGGL(k_empty, 256, 256, 0, s, p); }, 2000);
    run("empty 1024-WG", [&] { hipLaunchKernelGGL(k_empty, 1024, 256, 0, s, p); }, 2000);
    run("dirty 1 MB (256 WG) + empty 1-WG (pair)", [&] {
        hipLaunchKernelGGL(k_dirty, 256, 256, 0, s, a, n);
        hipLaunchKernelGGL(k_empty, 1, 64, 0, s, p); }, 1000);
    run("dirty 1 MB (256 WG) alone", [&] { hipLaunchKernelGGL(k_dirty, 256, 256, 0, s, a, n); }, 1000);
    run("read 1 MB (256 WG)", [&] { hipLaunchKernelGGL(k_read, 256, 256, 0, s, a, n, o); }, 1000);
    run("dirty 8 MB (1024 WG)", [&] { hipLaunchKernelGGL(k_dirty, 1024, 256, 0, s, a, n); }, 200);
    return 0;
}
