// bits.hpp -- bit-sliced GF(256) arithmetic shared by the k_gf_bits kernel
// (apply_bits.hip) and its host emulation (CompiledMap::emulate_bits, the plan
// self-test).  The same functions run on both sides, so the self-test checks the
// arithmetic the device executes, not a restatement of it.
//
// A lane holds 32 bytes of a sub-chunk as 8 dwords.  transpose8 turns them into 8
// bit planes: plane i holds bit i of all 32 bytes (in a fixed, self-inverse bit
// order).  In planes, multiplication by 2 in GF(2^8) (polynomial 0x11D,
// Galois.java:43) is a renaming plus 3 XORs (xtime8), so the multiples 2^k x of an
// input cost 3 XORs each, and c.x = XOR of 2^k x over the set bits k of c
// (GF(2)-linearity).  acc_pair adds the multiples selected by 2 bits of c with one
// (3-input) XOR per plane.
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

namespace ecx {
namespace bits {

// a ^ b ^ c: one v_bitop3_b32 on gfx950 (0x96 = a^b^c).
__host__ __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}

// m ? a : b, bitwise: one v_bfi_b32 (D = S0 & S1 | ~S0 & S2).
__host__ __device__ __forceinline__ uint32_t sel(uint32_t m, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
#else
    return (a & m) | (b & ~m);
#endif
}

// acc ^= a and acc ^= a ^ b in place.  On the device the accumulator is an in/out
// operand of the instruction, so the register allocator keeps every row's planes in
// the same registers on every path through the scalar branches of acc_pair (as plain
// expressions, each branch produced new registers and the join copied them back:
// a v_mov per plane and branch).
__host__ __device__ __forceinline__ void xor_into(uint32_t &acc, uint32_t a) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm("v_xor_b32 %0, %0, %1" : "+v"(acc) : "v"(a));
#else
    acc ^= a;
#endif
}

__host__ __device__ __forceinline__ void xor2_into(uint32_t &acc, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(acc) : "v"(a), "v"(b));
#else
    acc ^= a ^ b;
#endif
}

// One delta-swap stage between dwords a and b at bit distance s over mask m: the
// bits of a outside m and the bits of b inside m (shifted by s) trade places.  An
// involution, so the inverse transpose runs the stages in reverse order.  With m in
// a VGPR each select is one full-rate v_bfi_b32 (a literal mask would become an
// SGPR operand, which gfx950 issues at half rate).
__host__ __device__ __forceinline__ void swap_stage(uint32_t &a, uint32_t &b, int s, uint32_t m) {
    const uint32_t na = sel(m, a, b << s);
    const uint32_t nb = sel(m, a >> s, b);
    a = na;
    b = nb;
}

struct Masks {
    uint32_t m4, m2, m1;  // 0x0F0F0F0F, 0x33333333, 0x55555555
};

// 8 dwords (32 bytes) -> 8 bit planes, in place: after the three stages dword i
// holds bit i of every byte.
__host__ __device__ __forceinline__ void transpose8(uint32_t (&x)[8], const Masks &k) {
#pragma unroll
    for (int d = 0; d < 4; ++d) swap_stage(x[d], x[d + 4], 4, k.m4);
#pragma unroll
    for (int d = 0; d < 8; d += 4) {
        swap_stage(x[d], x[d + 2], 2, k.m2);
        swap_stage(x[d + 1], x[d + 3], 2, k.m2);
    }
#pragma unroll
    for (int d = 0; d < 8; d += 2) swap_stage(x[d], x[d + 1], 1, k.m1);
}

// 8 bit planes -> 8 dwords (the inverse of transpose8).
__host__ __device__ __forceinline__ void untranspose8(uint32_t (&x)[8], const Masks &k) {
#pragma unroll
    for (int d = 0; d < 8; d += 2) swap_stage(x[d], x[d + 1], 1, k.m1);
#pragma unroll
    for (int d = 0; d < 8; d += 4) {
        swap_stage(x[d], x[d + 2], 2, k.m2);
        swap_stage(x[d + 1], x[d + 3], 2, k.m2);
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) swap_stage(x[d], x[d + 4], 4, k.m4);
}

// y = 2 x in planes: x^8 = x^4 + x^3 + x^2 + 1 (0x11D).
__host__ __device__ __forceinline__ void xtime8(const uint32_t (&x)[8], uint32_t (&y)[8]) {
    y[0] = x[7];
    y[1] = x[0];
    y[2] = x[1] ^ x[7];
    y[3] = x[2] ^ x[7];
    y[4] = x[3] ^ x[7];
    y[5] = x[4];
    y[6] = x[5];
    y[7] = x[6];
}

__host__ __device__ __forceinline__ void xor_in(uint32_t (&acc)[8], const uint32_t (&a)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) xor_into(acc[i], a[i]);
}

__host__ __device__ __forceinline__ void xor_in2(uint32_t (&acc)[8], const uint32_t (&a)[8], const uint32_t (&b)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) xor2_into(acc[i], a[i], b[i]);
}

// acc ^= b0 X0 + b1 X1 for the two bits b of `pr` (wave-uniform): one XOR per plane.
// On the device the three cases and their scalar branches are one asm block with
// the accumulator planes as in/out operands: the compiler sees straight-line code,
// so no row's planes are ever copied between registers at a branch join (as C++
// branches, the structurized control flow copied each row's 8 planes at every join).
__host__ __device__ __forceinline__ void acc_pair(uint32_t (&acc)[8], const uint32_t (&x0)[8],
                                                  const uint32_t (&x1)[8], uint32_t pr) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile(
        "s_cmp_eq_u32 %16, 0\n"
        "s_cbranch_scc1 3f\n"
        "s_cmp_eq_u32 %16, 3\n"
        "s_cbranch_scc1 2f\n"
        "s_cmp_eq_u32 %16, 2\n"
        "s_cbranch_scc1 1f\n"
        "v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %9\n v_xor_b32 %2, %2, %10\n v_xor_b32 %3, %3, %11\n"
        "v_xor_b32 %4, %4, %12\n v_xor_b32 %5, %5, %13\n v_xor_b32 %6, %6, %14\n v_xor_b32 %7, %7, %15\n"
        "s_branch 3f\n"
        "1:\n"
        "v_xor_b32 %0, %0, %17\n v_xor_b32 %1, %1, %18\n v_xor_b32 %2, %2, %19\n v_xor_b32 %3, %3, %20\n"
        "v_xor_b32 %4, %4, %21\n v_xor_b32 %5, %5, %22\n v_xor_b32 %6, %6, %23\n v_xor_b32 %7, %7, %24\n"
        "s_branch 3f\n"
        "2:\n"
        "v_bitop3_b32 %0, %0, %8, %17 bitop3:0x96\n v_bitop3_b32 %1, %1, %9, %18 bitop3:0x96\n"
        "v_bitop3_b32 %2, %2, %10, %19 bitop3:0x96\n v_bitop3_b32 %3, %3, %11, %20 bitop3:0x96\n"
        "v_bitop3_b32 %4, %4, %12, %21 bitop3:0x96\n v_bitop3_b32 %5, %5, %13, %22 bitop3:0x96\n"
        "v_bitop3_b32 %6, %6, %14, %23 bitop3:0x96\n v_bitop3_b32 %7, %7, %15, %24 bitop3:0x96\n"
        "3:\n"
        : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]),
          "+v"(acc[7])
        : "v"(x0[0]), "v"(x0[1]), "v"(x0[2]), "v"(x0[3]), "v"(x0[4]), "v"(x0[5]), "v"(x0[6]), "v"(x0[7]), "s"(pr),
          "v"(x1[0]), "v"(x1[1]), "v"(x1[2]), "v"(x1[3]), "v"(x1[4]), "v"(x1[5]), "v"(x1[6]), "v"(x1[7])
        : "scc");
#else
    if (pr & 1) xor_in(acc, x0);
    if (pr & 2) xor_in(acc, x1);
#endif
}

// One plan entry against the tile's 8 accumulator rows: `p` is the input in planes;
// `rmask` the rows with a non-zero coefficient; `clo`/`chi` the coefficients of rows
// 0-3 / 4-7, one byte each.  The multiples 2^k x are generated two at a time (k, k+1)
// and every row adds the ones its coefficient's bits k, k+1 select: per row and bit
// pair one scalar-branched block of 8 XORs, so the code stays small (the kernel's
// whole loop fits the instruction cache) at ~24 vector ops per coefficient.
__host__ __device__ __forceinline__ void apply_entry_bits(uint32_t (&acc)[8][8], const uint32_t (&p)[8],
                                                          uint32_t rmask, uint32_t clo, uint32_t chi) {
    uint32_t x0[8], x1[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x0[i] = p[i];
    xtime8(x0, x1);
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
        if (k > 0) {
            uint32_t t[8];
            xtime8(x1, t);
            xtime8(t, x1);
#pragma unroll
            for (int i = 0; i < 8; ++i) x0[i] = t[i];
        }
        // rows outside rmask have coefficient 0 (the plan guarantees it), so their
        // bit pairs are 0 and acc_pair skips them
#pragma unroll
        for (int o = 0; o < 8; ++o) acc_pair(acc[o], x0, x1, ((o < 4 ? clo : chi) >> (8 * (o & 3) + k)) & 3u);
    }
    (void)rmask;
}

}  // namespace bits
}  // namespace ecx
