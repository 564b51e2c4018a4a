// apply_lut.hip -- k_gf_lut: the GF(256) map with per-byte table lookups in LDS.
//
// This is the textbook GPU form of the reference's loop, kept as a measured
// alternative to the split-table kernel, forced-only
// (ecx_tune "lds_lut"):
//
//   MODE 0 (log/antilog): LOG (u16, log 0 = 512) and EXP (1024 B: EXP[i] = 2^(i mod 255)
//           for i < 510, zero above, so a zero byte needs no branch) staged in LDS, as
//           Galois.multiply does it (Galois.java:184-200: EXP[LOG a + LOG b]).  Per
//           input byte one ds_read_u16 (its log), per byte and coefficient an add and
//           one ds_read_u8.
//   MODE 1 (product rows): the 256-B MULTIPLICATION_TABLE row (Galois.java:178,298-306)
//           of every (entry, row) coefficient of a single-tile map, built once per
//           workgroup from the plan's split tables, as InputOutputByteTableCodingLoop
//           indexes it (InputOutputByteTableCodingLoop.java:27-29,39-41): per byte and
//           coefficient one ds_read_u8.
//
// Coefficient 1 stays a plain XOR in both modes, so only the multiplies differ from
// k_gf_apply.  Workgroups are persistent (a grid-stride walk over (stripe, 4 KiB
// chunk, tile) units), so the tables are staged once per workgroup, not per chunk.
// Work decomposition per unit as k_gf_apply: 256 lanes x 16 bytes, 4 16-B loads per
// lane in flight, over the depth-4 padded plan.
#include "apply.hpp"

namespace ecx {

// LOG / EXP of GF(2^8) over x^8+x^4+x^3+x^2+1 (0x11D, generator 2: Galois.java:43,59-170),
// built at compile time.
struct LutTables {
    uint16_t log[256];
    uint8_t exp[1024];
    constexpr LutTables() : log(), exp() {
        uint32_t v = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = (uint8_t)v;
            exp[i + 255] = (uint8_t)v;
            log[v] = (uint16_t)i;
            v <<= 1;
            if (v & 0x100) v ^= 0x11D;
        }
        log[0] = 512;  // lands in the zero half of EXP for any log c <= 254
        for (int i = 510; i < 1024; ++i) exp[i] = 0;
    }
};
__constant__ LutTables kLut = LutTables();

constexpr int kLutThreads = kBlockThreads;
constexpr int kLutDepth = 4;

// c for row o of a plan entry: byte 1 of T0a, the product c * 1 (engine.hpp).
__device__ __forceinline__ uint32_t entry_coef(cu32 *r, int o) { return (r[4 + 5 * o] >> 8) & 0xFFu; }

template <int MODE, bool NTL>
__global__ void __launch_bounds__(kLutThreads, 2) k_gf_lut(ApplyArgs a, int64_t n_units) {
    __shared__ uint16_t s_log[256];
    __shared__ uint8_t s_exp[1024];
    extern __shared__ uint8_t s_rows[];  // MODE 1: [pairs][256]
    if (MODE == 0) {
        for (int i = threadIdx.x; i < 256; i += kLutThreads) s_log[i] = kLut.log[i];
        for (int i = threadIdx.x; i < 1024; i += kLutThreads) s_exp[i] = kLut.exp[i];
    } else {
        // One 256-B product row per (entry, row) with a general coefficient of tile 0, in
        // plan order; lane v computes c * v from the split tables.
        cu32 *tile = plan_ptr(a.tiles);
        cu32 *ent = plan_ptr(a.entries) + (int64_t)tile[0] * kEntryDwords;
        const int ecnt = (int)tile[1];
        const uint32_t v = threadIdx.x;
        int p = 0;
        for (int e = 0; e < ecnt; ++e) {
            cu32 *r = ent + (int64_t)e * kEntryDwords;
            const uint32_t mmul = r[1];
            for (int o = 0; o < kTileRows; ++o) {
                if (!(mmul & (1u << o))) continue;
                cu32 *t = r + 4 + 5 * o;
                const uint32_t i0 = v & 7u, i1 = (v >> 3) & 7u, i2 = v >> 6;
                const uint32_t b0 = ((i0 < 4 ? t[0] : t[1]) >> (8 * (i0 & 3))) & 0xFFu;
                const uint32_t b1 = ((i1 < 4 ? t[2] : t[3]) >> (8 * (i1 & 3))) & 0xFFu;
                const uint32_t b2 = (t[4] >> (8 * i2)) & 0xFFu;
                s_rows[p * 256 + v] = (uint8_t)(b0 ^ b1 ^ b2);
                ++p;
            }
        }
    }
    __syncthreads();

    const uint32_t lane16 = threadIdx.x * 16;
    for (int64_t u = blockIdx.x; u < n_units; u += gridDim.x) {
        const uint32_t tl = (uint32_t)(u % a.n_tiles);
        const int64_t rest = u / a.n_tiles;
        const int64_t c = a.chunk_begin + rest % a.n_chunks;
        const int64_t s = a.stripe_begin + rest / a.n_chunks;
        const int64_t cbase = c * kChunkBytes;
        cu32 *tile = plan_ptr(a.tiles) + __builtin_amdgcn_readfirstlane(tl) * kTileDwords;
        const int ecnt = (int)tile[1];
        const int nrows = (int)tile[2];
        cu32 *ent = plan_ptr(a.entries) + (int64_t)tile[0] * kEntryDwords;
        const uint8_t *ib = reinterpret_cast<const uint8_t *>(uniform64((uint64_t)(a.in + s * a.in_stripe_stride + cbase))) + lane16;
        auto load = [&](uint32_t slot) -> u32x4 {
            const uint8_t *p = slot == kDummySlot ? a.zero_page + lane16 : ib + (int64_t)slot * a.in_slot_stride;
            return ld16<NTL>(p);
        };
        u32x4 acc[kTileRows];
#pragma unroll
        for (int o = 0; o < kTileRows; ++o) acc[o] = (u32x4){0u, 0u, 0u, 0u};
        int p = 0;  // MODE 1: product row of the next general coefficient
        // Loads kLutDepth - 1 entries ahead, rotated through registers (a few v_mov per
        // entry): the entry loop is not unrolled, since unrolled copies of the branchy row
        // loop spill.
        u32x4 ring[kLutDepth];
#pragma unroll
        for (int k = 0; k < kLutDepth; ++k) ring[k] = ecnt > k ? load(ent[k * kEntryDwords]) : (u32x4){0u, 0u, 0u, 0u};
#pragma unroll 1
        for (int e = 0; e < ecnt; ++e) {
            cu32 *r = ent + (int64_t)e * kEntryDwords;
            const u32x4 x = ring[0];
#pragma unroll
            for (int k = 0; k + 1 < kLutDepth; ++k) ring[k] = ring[k + 1];
            if (e + kLutDepth < ecnt) ring[kLutDepth - 1] = load(r[kLutDepth * kEntryDwords]);
            const uint32_t mmul = r[1], mone = r[2];
            const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
            if (mmul) {
                uint32_t lx[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const uint32_t b = (xw[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                    lx[i] = MODE == 0 ? (uint32_t)s_log[b] : b;
                }
#pragma unroll
                for (int o = 0; o < kTileRows; ++o) {
                    if (!(mmul & (1u << o))) continue;
                    // MODE 0: EXP + log c; MODE 1: the pair's product row
                    const uint8_t *tab = MODE == 0 ? s_exp + s_log[entry_coef(r, o)] : s_rows + 256 * p;
                    ++p;
                    uint32_t w[4];
#pragma unroll
                    for (int d = 0; d < 4; ++d)
                        w[d] = (uint32_t)tab[lx[4 * d]] | ((uint32_t)tab[lx[4 * d + 1]] << 8) |
                               ((uint32_t)tab[lx[4 * d + 2]] << 16) | ((uint32_t)tab[lx[4 * d + 3]] << 24);
                    acc[o] ^= (u32x4){w[0], w[1], w[2], w[3]};
                }
            }
            if (mone) {
#pragma unroll
                for (int o = 0; o < kTileRows; ++o)
                    if (mone & (1u << o)) acc[o] ^= x;
            }
        }
        uint8_t *ob = reinterpret_cast<uint8_t *>(uniform64((uint64_t)(a.out + s * a.out_stripe_stride + cbase))) + lane16;
#pragma unroll
        for (int o = 0; o < kTileRows; ++o) {
            if (o < nrows) {
                uint8_t *q = ob + (int64_t)tile[4 + o] * a.out_slot_stride;
                u32x4 v = acc[o];
                if (a.accumulate) v ^= load16(q);
                st16<1>(q, v);
            }
        }
    }
}

void launch_lut(int mode, bool ntl, int pairs, int64_t n_units, hipStream_t stream, const ApplyArgs &a) {
    if (n_units <= 0) return;
    int dev = 0, cus = 256;
    check_hip(hipGetDevice(&dev), "hipGetDevice");
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const size_t lds = mode == 1 ? (size_t)pairs * 256 : 0;
    // one resident wave of workgroups: as many per CU as the occupancy allows
    auto grid_for = [&](const void *k) {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kLutThreads, lds) != hipSuccess || per_cu < 1)
            per_cu = 2;
        return (unsigned)std::min<int64_t>(n_units, (int64_t)cus * per_cu);
    };
#define ECX_LUT(M, L)                                                                    \
    if (mode == M && ntl == L) {                                                         \
        note_kernel("k_gf_lut", M, L);                                                   \
        const unsigned grid = grid_for(reinterpret_cast<const void *>(&k_gf_lut<M, L>));   \
        hipLaunchKernelGGL((k_gf_lut<M, L>), dim3(grid), dim3(kLutThreads), lds, stream, a, n_units); \
        return;                                                                          \
    }
    ECX_LUT(0, false) ECX_LUT(0, true) ECX_LUT(1, false) ECX_LUT(1, true)
#undef ECX_LUT
    throw Error(ECX_E_ILLEGAL_ARGUMENT, "no k_gf_lut instance for this shape");
}

}  // namespace ecx
