// apply_bits.hip -- k_gf_bits: the GF(256) map applied in bit-sliced form.
//
// Same work decomposition and plan (tiles of up to 8 output rows, one entry per
// input slot) as k_gf_apply (apply.hpp), but a lane owns 32 bytes of each
// sub-chunk -- bytes [16 l, 16 l + 16) and [2048 + 16 l, 2048 + 16 l + 16) of a
// 128-lane workgroup's 4 KiB chunk, so each of its two loads per entry is one
// fully coalesced 2 KiB wave access -- and multiplies in bit planes (bits.hpp):
//
//   per entry:   8 dwords -> 8 planes (48 full-rate ops), the multiples 2x .. 128x
//                (3 XORs each), then per row with coefficient c one (3-input) XOR
//                per plane for every bit pair (k, k+1) of c that is not zero;
//   per row:     the 8 accumulator planes back to 8 dwords at the tile's end.
//
// The split-table kernel spends 3 half-rate v_perm_b32 + 2 v_bitop3_b32 per dword and
// coefficient (8 full-rate issue slots, 64 per 32 bytes); here a coefficient costs
// ~24 slots per 32 bytes and an entry ~70 slots of fixed work, which matters for
// maps with many coefficients per input byte (Clay(10,4): 21.75 per output byte).
// Coefficients are wave-uniform scalars; the bit-pair cases are scalar branches.
#include "apply.hpp"
#include "bits.hpp"

namespace ecx {

// A VGPR holding `v`: the transpose masks must be vector operands (a literal in a
// VOP3 select becomes an SGPR operand, issued at half rate on gfx950).
__device__ __forceinline__ uint32_t vgpr_const(uint32_t v) {
    uint32_t r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "i"(v));
    return r;
}

template <bool NTL, int DEPTH>
__global__ void __launch_bounds__(kBitsThreads, DEPTH <= 2 ? 4 : 3) k_gf_bits(ApplyArgs a) {
    const uint32_t w = blockIdx.x;
    const uint32_t tl = w % (uint32_t)a.n_tiles;
    const uint32_t rest = w / (uint32_t)a.n_tiles;
    const int64_t c = a.chunk_begin + (int64_t)(rest % (uint32_t)a.n_chunks);
    const int64_t s = a.stripe_begin + (int64_t)(rest / (uint32_t)a.n_chunks);
    const int64_t cbase = c * kChunkBytes;
    const uint64_t in_base = uniform64((uint64_t)(a.in + s * a.in_stripe_stride + cbase));
    const uint64_t out_base = uniform64((uint64_t)(a.out + s * a.out_stripe_stride + cbase));
    cu32 *tile = plan_ptr(a.tiles) + __builtin_amdgcn_readfirstlane(tl) * kTileDwords;
    const int ebeg = (int)tile[0];
    const int ecnt = (int)tile[1];
    const int nrows = (int)tile[2];
    cu32 *be = plan_ptr(a.bentries) + (int64_t)ebeg * kBitsEntryDwords;
    const uint32_t voff = threadIdx.x * 16;

    // Inputs through a buffer descriptor over this stripe chunk: the slot's offset is
    // a scalar soffset, the lane's two 16-B pieces the voffset and voffset + 2 KiB
    // (launch_apply checks that every slot offset fits 31 bits).  Padding entries and
    // the refills past the end of the tile read the zero page through a second
    // descriptor; their row mask is 0, so nothing is applied.
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(in_base), 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t zrsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.zero_page), 0, kChunkBytes, 0x00020000);
    struct In {
        u32x4 lo, hi;
    };
    auto load = [&](uint32_t slot) -> In {
        const bool dummy = slot == kDummySlot;
        const __amdgpu_buffer_rsrc_t rs = dummy ? zrsrc : rsrc;
        const uint32_t soff = dummy ? 0u : slot * (uint32_t)a.in_slot_stride;
        const auto v0 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, (int)soff, NTL ? 2 : 0);
        const auto v1 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(voff + kChunkBytes / 2), (int)soff,
                                                              NTL ? 2 : 0);
        return In{(u32x4){(uint32_t)v0[0], (uint32_t)v0[1], (uint32_t)v0[2], (uint32_t)v0[3]},
                  (u32x4){(uint32_t)v1[0], (uint32_t)v1[1], (uint32_t)v1[2], (uint32_t)v1[3]}};
    };

    const bits::Masks mk{vgpr_const(0x0F0F0F0Fu), vgpr_const(0x33333333u), vgpr_const(0x55555555u)};
    uint32_t acc[8][8];
#pragma unroll
    for (int o = 0; o < 8; ++o)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[o][i] = 0u;

    // Load ring of DEPTH entries (each entry list is padded to a multiple of DEPTH):
    // consume a slot, refill it DEPTH entries ahead.  The loop body is the only copy
    // of the entry code (DEPTH copies of ~6 KiB), so there is no peeled tail: the
    // refills past the end read the zero page (rmask 0 entries are never applied).
    if (ecnt > 0) {
        In ring[DEPTH];
#pragma unroll
        for (int u = 0; u < DEPTH; ++u) ring[u] = load(be[u * kBitsEntryDwords]);
        for (int e0 = 0; e0 < ecnt; e0 += DEPTH) {
#pragma unroll
            for (int u = 0; u < DEPTH; ++u) {
                cu32 *r = be + (int64_t)(e0 + u) * kBitsEntryDwords;
                const uint32_t rmask = r[1];
                const uint32_t clo = r[2], chi = r[3];
                const int nxt = e0 + u + DEPTH;
                const uint32_t nslot = nxt < ecnt ? r[DEPTH * kBitsEntryDwords] : kDummySlot;
                if (rmask) {  // wave-uniform: padding entries carry no rows
                    uint32_t p[8] = {ring[u].lo.x, ring[u].lo.y, ring[u].lo.z, ring[u].lo.w,
                                     ring[u].hi.x, ring[u].hi.y, ring[u].hi.z, ring[u].hi.w};
                    bits::transpose8(p, mk);
                    bits::apply_entry_bits(acc, p, rmask, clo, chi);
                }
                ring[u] = load(nslot);
            }
        }
    }
#pragma unroll
    for (int o = 0; o < 8; ++o) {
        if (o < nrows) {
            bits::untranspose8(acc[o], mk);
            uint8_t *p = reinterpret_cast<uint8_t *>(out_base) + voff + (int64_t)tile[4 + o] * a.out_slot_stride;
            u32x4 v0 = (u32x4){acc[o][0], acc[o][1], acc[o][2], acc[o][3]};
            u32x4 v1 = (u32x4){acc[o][4], acc[o][5], acc[o][6], acc[o][7]};
            if (a.accumulate) {  // wave-uniform branch
                v0 ^= load16(p);
                v1 ^= load16(p + kChunkBytes / 2);
            }
            st16<1>(p, v0);
            st16<1>(p + kChunkBytes / 2, v1);
        }
    }
}

void launch_bits(bool ntl, int depth, dim3 grid, hipStream_t stream, const ApplyArgs &a) {
    const dim3 blk(kBitsThreads);
#define ECX_BITS(NTL, D)                                                      \
    if (ntl == NTL && depth == D) {                                           \
        note_kernel("k_gf_bits", NTL, D);                                     \
        hipLaunchKernelGGL((k_gf_bits<NTL, D>), grid, blk, 0, stream, a);     \
        return;                                                               \
    }
    ECX_BITS(false, 2) ECX_BITS(false, 4) ECX_BITS(true, 2) ECX_BITS(true, 4)
#undef ECX_BITS
    throw Error(ECX_E_ILLEGAL_ARGUMENT, "no k_gf_bits instance for this shape");
}

}  // namespace ecx
