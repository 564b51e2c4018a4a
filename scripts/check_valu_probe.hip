// check_valu_probe.hip -- is the RS(17,3) read-only check bound by its arithmetic?
// k_gf_check runs at 0.81-0.83 of HBM where the bare reads of the same twenty 200,000-B shards
// run at 0.87 (rw_probe.hip), and its clock drops to ~1.8 GHz under the load.  This probe
// streams those twenty shards exactly like the bare reads (NT loads, one 256-thread workgroup
// per (stripe, 4 KiB chunk), every load of a lane in flight, OR-fold, no stores) and adds M
// split-table multiplies per loaded dword -- the k_gf_apply multiply (3 v_perm_b32 + 2
// v_bitop3_b32), pinned with inline asm -- M = 0 .. 4.  The real check does ~3 per data dword
// (three syndrome rows); folding its equal-coefficient pairs first would leave ~1.6.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/check_valu_probe.hip -o scripts/check_valu_probe && ./scripts/check_valu_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const gu32x4 *)p); }

// one multiply-shaped step on a dword: three byte permutes and two 3-input bit ops
__device__ __forceinline__ uint32_t mul_step(uint32_t x, uint32_t lo, uint32_t hi, uint32_t acc) {
    uint32_t a, b, c;
    asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(a) : "s"(lo), "v"(hi), "v"(x));
    asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(b) : "v"(hi), "s"(lo), "v"(x));
    asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(c) : "s"(lo), "v"(hi), "v"(a));
    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(a) : "v"(a), "v"(b), "v"(c));
    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(acc) : "v"(acc), "v"(a), "v"(x));
    return acc;
}

template <int M>
__global__ void __launch_bounds__(256) k_check(const uint8_t *pool, uint32_t *sink, int64_t pitch, int chunks,
                                               uint32_t lo, uint32_t hi_s) {
    const uint32_t hi = hi_s + (threadIdx.x >> 10);  // uniform value held in a VGPR
    const int64_t stripe = blockIdx.x / chunks, chunk = blockIdx.x % chunks;
    const uint8_t *in = pool + stripe * 20 * pitch + chunk * 4096 + threadIdx.x * 16;
    u32x4 x[20];
#pragma unroll
    for (int i = 0; i < 20; ++i) x[i] = ldnt(in + (int64_t)i * pitch);
    uint32_t acc[3][4] = {};  // three rows x four dwords: twelve independent chains, as in k_gf_check
#pragma unroll
    for (int i = 0; i < 20; ++i) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const uint32_t v = x[i][d];
#pragma unroll
            for (int m = 0; m < M; ++m) acc[m % 3][d] = mul_step(v, lo + (uint32_t)m, hi, acc[m % 3][d]);
            if constexpr (M == 0) acc[i % 3][d] |= v;
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) r |= acc[k][0] | acc[k][1] | acc[k][2] | acc[k][3];
    if (__builtin_amdgcn_ballot_w64(r == 0x9E3779B9u) != 0 && (threadIdx.x & 63) == 0) sink[blockIdx.x & 1023] = r;
}

template <int M>
float run(const uint8_t *pool, uint32_t *sink, int64_t pitch, int64_t stripes) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int chunks = (int)(pitch / 4096);
    std::vector<float> ms;
    for (int rep = 0; rep < 6; ++rep) {
        float t = 0;
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k_check<M>), dim3((unsigned)(stripes * chunks)), dim3(256), 0, 0, pool, sink, pitch, chunks,
                           0x03020100u, 0x07060504u);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&t, e0, e1);
        if (rep) ms.push_back(t);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
}

int main() {
    const int64_t pitch = 200000, stripes = 4096;
    uint8_t *pool = nullptr;
    uint32_t *sink = nullptr;
    if (hipMalloc(&pool, stripes * 20 * pitch) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) return 1;
    (void)hipMemset(pool, 0x5A, stripes * 20 * pitch);
    (void)hipDeviceSynchronize();
    const double bytes = (double)stripes * 20 * (pitch / 4096) * 4096.0;
    for (int round = 0; round < 2; ++round) {
        float ms[5] = {run<0>(pool, sink, pitch, stripes), run<1>(pool, sink, pitch, stripes),
                       run<2>(pool, sink, pitch, stripes), run<3>(pool, sink, pitch, stripes),
                       run<4>(pool, sink, pitch, stripes)};
        for (int m = 0; m < 5; ++m)
            printf("{\"probe\": \"check_valu\", \"round\": %d, \"mul_per_dword\": %d, \"ms\": %.4f, \"frac\": %.4f}\n",
                   round, m, ms[m], bytes / (ms[m] * 1e-3) / 8e12);
        fflush(stdout);
    }
    return 0;
}
