// valu_probe.hip -- issue rate of the VALU instructions the GF(256) apply kernel
// uses (v_perm_b32, v_bitop3_b32, v_and_b32, v_lshrrev_b32, v_xor_b32) next to
// v_fma_f32, on every SIMD of the chip.  Each wave runs 8 independent chains of
// one instruction kind; the result is wave-instructions per SIMD per cycle,
// with cycles from s_memtime inside each wave (shader clock).
//
//   hipcc --offload-arch=gfx950 -O3 scripts/valu_probe.hip -o scripts/valu_probe && ./scripts/valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;

// One instruction per chain step, pinned with inline asm so the compiler cannot
// fold or hoist it.
template <int KIND>
__device__ __forceinline__ void step(uint32_t &v, uint32_t s, uint32_t t, uint32_t u) {
    // SGPR operand s, VGPR operands t, u (both wave-uniform in value).
    if constexpr (KIND == 0) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(v) : "s"(s), "v"(t));
    if constexpr (KIND == 1) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(v) : "v"(u), "v"(t));
    if constexpr (KIND == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v) : "s"(s), "v"(t));
    if constexpr (KIND == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v) : "v"(u), "v"(t));
    if constexpr (KIND == 4) asm volatile("v_and_b32 %0, %1, %0" : "+v"(v) : "s"(s));
    if constexpr (KIND == 5) asm volatile("v_and_b32 %0, %1, %0" : "+v"(v) : "v"(u));
    if constexpr (KIND == 6) asm volatile("v_and_b32 %0, 0x7070707, %0" : "+v"(v));
    if constexpr (KIND == 7) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(v));
    if constexpr (KIND == 8) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(v) : "s"(s));
    if constexpr (KIND == 9) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v) : "v"(u));
    if constexpr (KIND == 10) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v) : "v"(u), "v"(t));
    if constexpr (KIND == 11) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v) : "s"(s), "v"(t));
    if constexpr (KIND == 12) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v) : "s"(s));
    if constexpr (KIND == 13) asm volatile("v_and_b32 %0, 7, %0" : "+v"(v));
    if constexpr (KIND == 14) asm volatile("v_add_u32 %0, %1, %0" : "+v"(v) : "v"(u));
    if constexpr (KIND == 15) asm volatile("v_pk_add_u16 %0, %1, %0" : "+v"(v) : "v"(u));
}

template <int KIND>
__global__ void __launch_bounds__(256) k_probe(uint32_t *out, uint64_t *cycles, uint32_t s) {
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * 2654435761u + i;
    const uint32_t t = threadIdx.x & 7u;
    const uint32_t u = s + (threadIdx.x >> 10);  // same value in every lane, held in a VGPR
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) step<KIND>(v[i], s, t, u);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x == 0) cycles[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char *name, int instr_per_inner, int waves_per_simd) {
    const int cus = 256, blocks = cus * waves_per_simd;  // 256 threads = one wave per SIMD per block
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipMalloc(&cyc, (size_t)blocks * 8);
    hipLaunchKernelGGL(k_probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, cyc, 0x03020100u);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, cyc, 0x03020100u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    uint64_t *h = new uint64_t[blocks];
    hipMemcpy(h, cyc, (size_t)blocks * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks; ++i) mean += (double)h[i];
    mean /= blocks;
    // Per SIMD: waves_per_simd waves each issued kIters * 8 * instr_per_inner instructions.
    const double instr = (double)kIters * 8 * instr_per_inner * waves_per_simd;
    const double wall_cyc_per_instr = ms * 1e-3 * 2.4e9 / instr;  // at the 2.4 GHz max clock
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"memtime_ticks_per_wave\": %.0f, \"ms\": %.3f, "
           "\"simd_cycles_per_wave_instr_at_2.4GHz\": %.3f, \"wave_instr_per_s_chip\": %.3e}\n",
           name, waves_per_simd, mean, ms, wall_cyc_per_instr, instr * 1024 / (ms * 1e-3));
    delete[] h;
    hipFree(out);
    hipFree(cyc);
}

int main() {
    const char *names[] = {"v_perm_b32 sgpr,vgpr,vgpr", "v_perm_b32 vgpr,vgpr,vgpr", "v_bitop3_b32 vgpr,sgpr,vgpr",
                           "v_bitop3_b32 vgpr,vgpr,vgpr", "v_and_b32 sgpr,vgpr", "v_and_b32 vgpr,vgpr",
                           "v_and_b32 literal,vgpr", "v_lshrrev_b32 inline,vgpr", "v_lshrrev_b32 sgpr,vgpr",
                           "v_xor_b32 vgpr,vgpr", "v_fma_f32 vgpr,vgpr,vgpr", "v_fma_f32 vgpr,sgpr,vgpr",
                           "v_xor_b32 sgpr,vgpr", "v_and_b32 inline,vgpr", "v_add_u32 vgpr,vgpr", "v_pk_add_u16 vgpr,vgpr"};
    for (int w : {4, 8}) {
        run<0>(names[0], 1, w); run<1>(names[1], 1, w); run<2>(names[2], 1, w); run<3>(names[3], 1, w);
        run<4>(names[4], 1, w); run<5>(names[5], 1, w); run<6>(names[6], 1, w); run<7>(names[7], 1, w);
        run<8>(names[8], 1, w); run<9>(names[9], 1, w); run<10>(names[10], 1, w); run<11>(names[11], 1, w);
        run<12>(names[12], 1, w); run<13>(names[13], 1, w); run<14>(names[14], 1, w); run<15>(names[15], 1, w);
    }
    return 0;
}
