// Probe: the operand order of v_bitop3_b32's truth table on gfx950.  Prints
// bitop3(0xF0F0F0F0, 0xCCCCCCCC, 0xAAAAAAAA, T) for a few tables T: with src0 as the
// table index's most significant bit the result equals T replicated.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned *in, unsigned *out) {
    const unsigned a = in[0], b = in[1], c = in[2];
    out[0] = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE4);
    out[1] = __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
    out[2] = __builtin_amdgcn_bitop3_b32(a, b, c, 0xC8);
    out[3] = __builtin_amdgcn_bitop3_b32(a, b, c, 0x80);
}
int main() {
    unsigned h[3] = {0xF0F0F0F0u, 0xCCCCCCCCu, 0xAAAAAAAAu}, r[4];
    unsigned *d_in, *d_out;
    hipMalloc(&d_in, 12); hipMalloc(&d_out, 16);
    hipMemcpy(d_in, h, 12, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(1), 0, 0, d_in, d_out);
    hipMemcpy(r, d_out, 16, hipMemcpyDeviceToHost);
    printf("E4 -> %08x  96 -> %08x  C8 -> %08x  80 -> %08x\n", r[0], r[1], r[2], r[3]);
    return 0;
}
