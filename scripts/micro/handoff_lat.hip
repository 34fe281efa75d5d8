// Hand-off latency between two workgroups of one launch on MI355X: a ping-pong of an 8 KB payload (one L tile of
// k_chol_flow) plus a flag, timed with s_memrealtime, for the workgroup pairs (0, 8) (one XCD under round-robin
// placement) and (0, 1) (two XCDs), each reporting its HW_REG_XCC_ID.
//   V0: payload stored sc1 (write-through), consumer sc1 loads -- k_chol_flow's protocol, valid across XCDs;
//   V1: payload stored plain (kept in the XCD's L2), consumer sc1 loads (L1 bypassed, L2-served) -- valid only
//       when both workgroups sit on one XCD; the consumer counts stale values, so a cross-XCD pair shows the hazard;
//   V2: the flag alone (no payload); V3: V0 with 16-byte sc1 stores / loads (two doubles per access, each load
//   waited for); V4: 16-byte sc1 buffer stores / loads (the compiler's own, loads in flight together).
// hipcc --offload-arch=gfx950 -O3 handoff_lat.hip -o /tmp/handoff_lat && /tmp/handoff_lat
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) int gi32_t;

__device__ __forceinline__ double ld_sc1(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store((gu64_t*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte sc1 load / store (global_load_dwordx4 / global_store_dwordx4 with sc1)
typedef double d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ d2v ld2_sc1(const double* p) {
    d2v v;
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ void st2_sc1(double* p, double a, double b) {
    d2v v = {a, b};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
}
typedef unsigned v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc8k(const double* p) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, 8192, 0x00020000);
}
__device__ __forceinline__ unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}

constexpr int PAY = 1024;   // doubles (8 KB)

template <int V>
__global__ __launch_bounds__(256) void k_pingpong(double* pay, int* flag, int a, int b, int rounds,
                                                  unsigned long long* out, int* err) {
    const int me = blockIdx.x;
    if (me != a && me != b) return;
    const int side = me == a ? 0 : 1;
    const int tid = threadIdx.x;
    __shared__ int ok;
    int bad = 0;
    if (tid == 0) out[2 + side] = xcc_id();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < rounds; ++r) {
        const int turn = r & 1;   // who produces this round
        if (turn == side) {
            if (V == 3) {
                for (int i = 2 * tid; i < PAY; i += 512) {
                    st2_sc1(pay + i, (double)(r * PAY + i), (double)(r * PAY + i + 1));
                }
            } else if (V == 4) {
                const __amdgpu_buffer_rsrc_t rs = rsrc8k(pay);
                for (int i = 2 * tid; i < PAY; i += 512) {
                    const long long a0 = __double_as_longlong((double)(r * PAY + i)), a1 = __double_as_longlong((double)(r * PAY + i + 1));
                    v4u q = {(unsigned)a0, (unsigned)(a0 >> 32), (unsigned)a1, (unsigned)(a1 >> 32)};
                    __builtin_amdgcn_raw_buffer_store_b128(q, rs, i * 8, 0, 16);
                }
            } else if (V != 2) {
                for (int i = tid; i < PAY; i += 256) {
                    const double v = (double)(r * PAY + i);
                    if (V == 0) st_sc1(pay + i, v);
                    else pay[i] = v;
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) __hip_atomic_store((gi32_t*)flag, r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (tid == 0) {
                unsigned spins = 0;
                while (__hip_atomic_load((gi32_t*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != r + 1)
                    if (++spins > (1u << 24)) break;
                ok = 1;
            }
            __syncthreads();
            if (V == 3) {
                for (int i = 2 * tid; i < PAY; i += 512) {
                    d2v q = ld2_sc1(pay + i);
                    if (q.x != (double)(r * PAY + i) || q.y != (double)(r * PAY + i + 1)) ++bad;
                }
            } else if (V == 4) {
                const __amdgpu_buffer_rsrc_t rs = rsrc8k(pay);
                v4u q[2];
                for (int m = 0; m < 2; ++m) q[m] = __builtin_amdgcn_raw_buffer_load_b128(rs, (2 * tid + 512 * m) * 8, 0, 16);
                for (int m = 0; m < 2; ++m) {
                    const int i = 2 * tid + 512 * m;
                    const double x = __longlong_as_double(((long long)q[m].y << 32) | q[m].x);
                    const double y = __longlong_as_double(((long long)q[m].w << 32) | q[m].z);
                    if (x != (double)(r * PAY + i) || y != (double)(r * PAY + i + 1)) ++bad;
                }
            } else if (V != 2) {
                for (int i = tid; i < PAY; i += 256)
                    if (ld_sc1(pay + i) != (double)(r * PAY + i)) ++bad;
            }
            __syncthreads();
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && side == 0) out[0] = t1 - t0;
    if (bad) atomicAdd(err, bad);
}

int main() {
    double* pay; int* flag; unsigned long long* out; int* err;
    (void)hipMalloc(&pay, PAY * 8); (void)hipMalloc(&flag, 256); (void)hipMalloc(&out, 64); (void)hipMalloc(&err, 4);
    const int rounds = 4000;
    auto run = [&](auto kern, const char* name, int a, int b) {
        unsigned long long h[4];
        int e = 0;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipMemset(flag, 0, 256); (void)hipMemset(err, 0, 4); (void)hipMemset(pay, 0, PAY * 8);
            hipLaunchKernelGGL(kern, dim3(16), dim3(256), 0, 0, pay, flag, a, b, rounds, out, err);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(h, out, 32, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
        printf("%-28s pair (%d,%d) xcc (%llu,%llu): %7.3f us per one-way hand-off, stale values %d\n", name, a, b, h[2], h[3],
               h[0] / 100.0 / rounds, e);   // s_memrealtime: 100 MHz
    };
    run(k_pingpong<0>, "V0 sc1 stores, sc1 loads", 0, 8);
    run(k_pingpong<0>, "V0 sc1 stores, sc1 loads", 0, 1);
    run(k_pingpong<1>, "V1 plain stores, sc1 loads", 0, 8);
    run(k_pingpong<1>, "V1 plain stores, sc1 loads", 0, 1);
    run(k_pingpong<2>, "V2 flag only", 0, 8);
    run(k_pingpong<2>, "V2 flag only", 0, 1);
    run(k_pingpong<3>, "V3 16-B sc1 stores / loads", 0, 8);
    run(k_pingpong<3>, "V3 16-B sc1 stores / loads", 0, 1);
    run(k_pingpong<4>, "V4 16-B sc1 buffer st / ld", 0, 8);
    run(k_pingpong<4>, "V4 16-B sc1 buffer st / ld", 0, 1);
    return 0;
}
