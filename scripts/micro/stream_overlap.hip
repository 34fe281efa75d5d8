// Two questions before overlapping the reduced-camera factorisation with the sweep on MI355X (round 5):
//  1. what does a cross-stream dependency cost per LM trial?  The trial pattern with stand-in kernels:
//     stream A: sweep -> wait(flow done) -> update -> finalize -> record(A done);
//     stream B: wait(A done of the previous trial) -> flow -> record(flow done);
//     against the same four launches on one stream.
//  2. do CU-masked streams (hipExtStreamCreateWithCUMask) keep a 1071-workgroup sweep (52 KB of LDS, 3 per CU)
//     and a 32-workgroup "flow" (1 per CU) on disjoint CUs, and how soon does a flow workgroup that polls a
//     counter see the sweep's tiles complete?
// hipcc --offload-arch=gfx950 -O3 stream_overlap.hip -o /tmp/stream_overlap && /tmp/stream_overlap
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)
typedef __attribute__((address_space(1))) int gi32_t;

__device__ __forceinline__ unsigned hw_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
    return v;
}
__device__ __forceinline__ unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}

__global__ void k_tiny(int* p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1; }

// sweep stand-in: every workgroup spins for `us` microseconds, stamps (start, end, placement), then bumps `done`
__global__ __launch_bounds__(256) void k_sweep(unsigned long long* st, int* done, int us) {
    extern __shared__ double shm[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    shm[threadIdx.x] = 1.0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)us * 100) __builtin_amdgcn_s_sleep(4);
    __syncthreads();
    if (threadIdx.x == 0) {
        st[4 * blockIdx.x] = t0;
        st[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        st[4 * blockIdx.x + 2] = hw_id();
        st[4 * blockIdx.x + 3] = xcc_id() + (shm[0] > 0.0 ? 0 : 1);
        __hip_atomic_fetch_add((gi32_t*)done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// flow stand-in: stamps its start, polls `done` until it reaches `want` (bounded), stamps when it saw it
__global__ __launch_bounds__(256, 1) void k_flow(unsigned long long* st, const int* done, int want) {
    extern __shared__ double shm[];
    if (threadIdx.x == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned spins = 0;
        while (__hip_atomic_load((gi32_t*)done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want && ++spins < (1u << 24))
            __builtin_amdgcn_s_sleep(2);
        shm[0] = (double)spins;
        st[4 * blockIdx.x] = t0;
        st[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        st[4 * blockIdx.x + 2] = hw_id();
        st[4 * blockIdx.x + 3] = xcc_id() + (shm[0] > 1e30 ? 16 : 0);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    int* dp;
    CK(hipMalloc(&dp, 64));
    CK(hipMemset(dp, 0, 64));
    // ---- 1. cross-stream dependency cost per trial
    hipStream_t A, B;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    const int T = 400;
    std::vector<hipEvent_t> ea(T + 1), eb(T + 1);
    for (int i = 0; i <= T; ++i) {
        CK(hipEventCreateWithFlags(&ea[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&eb[i], hipEventDisableTiming));
    }
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipDeviceSynchronize());
        double t0 = now_us();
        for (int t = 0; t < T; ++t) {
            k_tiny<<<1, 64, 0, A>>>(dp);
            k_tiny<<<1, 64, 0, A>>>(dp);
            k_tiny<<<1, 64, 0, A>>>(dp);
            k_tiny<<<1, 64, 0, A>>>(dp);
        }
        CK(hipStreamSynchronize(A));
        const double one = (now_us() - t0) / T;
        CK(hipEventRecord(ea[0], A));
        CK(hipDeviceSynchronize());
        t0 = now_us();
        for (int t = 0; t < T; ++t) {
            CK(hipStreamWaitEvent(B, ea[t], 0));
            k_tiny<<<1, 64, 0, B>>>(dp);   // flow
            CK(hipEventRecord(eb[t], B));
            k_tiny<<<1, 64, 0, A>>>(dp);   // sweep
            CK(hipStreamWaitEvent(A, eb[t], 0));
            k_tiny<<<1, 64, 0, A>>>(dp);   // update
            k_tiny<<<1, 64, 0, A>>>(dp);   // finalize
            CK(hipEventRecord(ea[t + 1], A));
        }
        CK(hipStreamSynchronize(A));
        const double two = (now_us() - t0) / T;
        std::printf("trial of 4 tiny launches: one stream %.2f us, two streams with 2 event waits %.2f us (+%.2f)\n", one, two,
                    two - one);
    }
    // ---- 2. CU-masked streams
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int nw = (ncu + 31) / 32;
    std::vector<uint32_t> ma(nw, 0), mb(nw, 0);
    const int nflow = 32;
    for (int c = 0; c < ncu; ++c) (c % (ncu / nflow) == 0 ? mb : ma)[c / 32] |= 1u << (c % 32);
    hipStream_t SA, SB;
    CK(hipExtStreamCreateWithCUMask(&SA, nw, ma.data()));
    CK(hipExtStreamCreateWithCUMask(&SB, nw, mb.data()));
    const int ntile = 1071;
    unsigned long long *sts, *stf;
    int* done;
    CK(hipMalloc(&sts, 8 * 4 * ntile));
    CK(hipMalloc(&stf, 8 * 4 * nflow));
    CK(hipMalloc(&done, 4));
    CK(hipFuncSetAttribute((const void*)k_flow, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024));
    CK(hipFuncSetAttribute((const void*)k_sweep, hipFuncAttributeMaxDynamicSharedMemorySize, 52 * 1024));
    for (int mode = 0; mode < 2; ++mode) {
        hipStream_t sa = mode ? SA : A, sb = mode ? SB : B;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemset(done, 0, 4));
            CK(hipDeviceSynchronize());
            k_flow<<<nflow, 256, 100 * 1024, sb>>>(stf, done, ntile / 4);
            k_sweep<<<ntile, 256, 52 * 1024, sa>>>(sts, done, 30);
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> hs(4 * ntile), hf(4 * nflow);
            CK(hipMemcpy(hs.data(), sts, 8 * hs.size(), hipMemcpyDeviceToHost));
            CK(hipMemcpy(hf.data(), stf, 8 * hf.size(), hipMemcpyDeviceToHost));
            unsigned long long s0 = ~0ull, s1 = 0;
            for (int i = 0; i < ntile; ++i) { s0 = std::min(s0, hs[4 * i]); s1 = std::max(s1, hs[4 * i + 1]); }
            // the time the ntile/4-th tile ended
            std::vector<unsigned long long> ends(ntile);
            for (int i = 0; i < ntile; ++i) ends[i] = hs[4 * i + 1];
            std::sort(ends.begin(), ends.end());
            const unsigned long long tq = ends[ntile / 4 - 1];
            double fs = 1e30, fl = 0, fw = 0;
            int shared = 0;
            for (int f = 0; f < nflow; ++f) {
                fs = std::min(fs, ((double)hf[4 * f] - (double)s0) / 100.0);
                fl = std::max(fl, ((double)hf[4 * f] - (double)s0) / 100.0);
                fw = std::max(fw, ((double)hf[4 * f + 1] - (double)tq) / 100.0);
                for (int i = 0; i < ntile; ++i)
                    if (hs[4 * i + 2] >> 8 == hf[4 * f + 2] >> 8 && hs[4 * i + 3] == hf[4 * f + 3]) { ++shared; break; }
            }
            std::printf("%s: sweep span %.1f us; flow starts %.1f .. %.1f us after the sweep's first tile; flow saw the "
                        "quarter mark <= %.2f us after it; flow workgroups sharing a CU (hw_id>>8, xcc) with a tile: %d/%d\n",
                        mode ? "CU-masked streams" : "plain streams", (s1 - s0) / 100.0, fs, fl, fw, shared, nflow);
        }
    }
    std::printf("done\n");
    return 0;
}
