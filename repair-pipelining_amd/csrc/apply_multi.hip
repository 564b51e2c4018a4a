// apply_multi.hip -- k_gf_apply_multi: single-tile maps, U consecutive (stripe, chunk) units per
// workgroup with ONE load ring running across them (ecx_tune "units").
//
// In k_gf_apply a workgroup loads its unit's inputs, multiplies, stores its output rows and exits:
// the stores are the last memory operations of the workgroup, issued when no load of it is in flight.
// Here the ring's last group of unit k refills with unit k+1's first entries, so unit k's stores
// leave while unit k+1's loads are already on their way (RS(17,3)'s encode loses ~0.45 ms per launch
// to its three write streams).  Every padded entry count is a multiple of
// DEPTH, so unit boundaries fall on ring groups; the choice between refilling from the next unit and
// not refilling (the workgroup's last unit) is one uniform branch per unit.
#include "apply.hpp"

namespace ecx {

// Bases of unit u of the launch: stripe-major (or staggered) order as k_gf_apply's unit_of; the
// shard's partial last chunk (TAIL) reads its last full window and stores only the partial lanes.
template <int THREADS, bool TAIL>
__device__ __forceinline__ void multi_unit(const ApplyArgs &a, uint32_t u, uint32_t nst, uint32_t lane16,
                                           uint64_t &in, uint64_t &out, bool &store) {
    int64_t s, c;
    unit_of(u, (uint32_t)a.n_chunks, nst, a.chunk_major, (uint32_t)a.stagger, s, c);
    s += a.stripe_begin;
    c += a.chunk_begin;
    int64_t cbase = c * (THREADS * 16);
    store = true;
    if constexpr (TAIL) {
        if (c == a.tail_chunk) {
            cbase = a.nbytes - THREADS * 16;
            store = lane16 >= (uint32_t)(THREADS * 16 - a.tail_bytes);
        }
    }
    in = uniform64((uint64_t)(a.in + s * a.in_stripe_stride + cbase));
    out = uniform64((uint64_t)(a.out + s * a.out_stripe_stride + cbase));
}

// (one wave per SIMD fewer than k_gf_apply's shapes: the per-unit bases and the store block need the room)
#define ECX_MULTI_BOUNDS(DEPTH) (DEPTH >= 16 ? 3 : 4)

template <int DEPTH, int ROWS, int U, int THREADS, bool TAIL>
__global__ void __launch_bounds__(THREADS, ECX_MULTI_BOUNDS(DEPTH)) k_gf_apply_multi(ApplyArgs a) {
    const uint32_t total = (uint32_t)a.multi_total;  // units (stripe, chunk) in this launch
    const uint32_t nst = total / (uint32_t)a.n_chunks;
    const uint32_t u0 = logical_block(a.xcd_group, 1u, (uint32_t)a.xcd_run) * (uint32_t)U;
    const uint32_t nu = total - u0 < (uint32_t)U ? total - u0 : (uint32_t)U;  // units of this workgroup
    cu32 *tile = plan_ptr(a.tiles);
    const int ecnt = (int)tile[1];  // padded to a multiple of DEPTH, > 0 (launch_apply_core)
    const int nrows = (int)tile[2];
    cu32 *ent = plan_ptr(a.entries) + (int64_t)tile[0] * kEntryDwords;
    const uint32_t lane16 = threadIdx.x * 16;
    // the units' bases, kept uniform; unit k of the entry stream e = k * ecnt + entry
    uint64_t ib[U], ob[U];
    bool st[U];
#pragma unroll
    for (int k = 0; k < U; ++k) multi_unit<THREADS, TAIL>(a, u0 + (k < (int)nu ? k : 0), nst, lane16, ib[k], ob[k], st[k]);
    auto in_of = [&](int k) -> uint64_t {  // select chain: no dynamic indexing of a register array
        uint64_t b = ib[0];
#pragma unroll
        for (int j = 1; j < U; ++j) b = k == j ? ib[j] : b;
        return b;
    };
    auto load = [&](uint64_t base, uint32_t slot) -> u32x4 {  // padding entries read the zero page
        return ld16<true>(slot == kDummySlot ? a.zero_page + lane16
                                             : reinterpret_cast<const uint8_t *>(base) + lane16 +
                                                   (int64_t)slot * a.in_slot_stride);
    };
    auto store_unit = [&](int k, u32x4 (&acc)[ROWS]) {
        uint64_t o = ob[0];
        bool sl = st[0];
#pragma unroll
        for (int j = 1; j < U; ++j) {
            o = k == j ? ob[j] : o;
            sl = k == j ? st[j] : sl;
        }
        uint8_t *p0 = reinterpret_cast<uint8_t *>(o) + lane16;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            if (r < nrows) {
                uint8_t *p = p0 + (int64_t)tile[4 + r] * a.out_slot_stride;
                u32x4 v = acc[r];
                if (a.accumulate) v ^= load16(p);  // wave-uniform branch
                if (sl) st16<1>(p, v);
            }
            acc[r] = (u32x4){0u, 0u, 0u, 0u};
        }
    };
    u32x4 acc[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r] = (u32x4){0u, 0u, 0u, 0u};
    const int total_e = (int)nu * ecnt;
    u32x4 ring[DEPTH];
#pragma unroll
    for (int u = 0; u < DEPTH; ++u) ring[u] = load(ib[0], ent[u * kEntryDwords]);
    // One ring over the workgroup's entry stream: a group never straddles two units (ecnt is a
    // multiple of DEPTH); the group that ends a unit refills from the next one, then stores.
    const int last = total_e - DEPTH;
    for (int e0 = 0; e0 < last; e0 += DEPTH) {
        const int k = e0 / ecnt, kn = (e0 + DEPTH) / ecnt;
        cu32 *grp = ent + (int64_t)(e0 - k * ecnt) * kEntryDwords;
        cu32 *nxt = ent + (int64_t)(e0 + DEPTH - kn * ecnt) * kEntryDwords;
        const uint64_t nb = in_of(kn);
#pragma unroll
        for (int u = 0; u < DEPTH; ++u) {
            apply_entry<false, ROWS>(grp + (int64_t)u * kEntryDwords, ring[u], acc, nullptr);
            ring[u] = load(nb, nxt[u * kEntryDwords]);
        }
        if (kn != k) store_unit(k, acc);  // uniform: unit k is complete, unit kn's loads are in flight
    }
    cu32 *grp = ent + (int64_t)(ecnt - DEPTH) * kEntryDwords;
#pragma unroll
    for (int u = 0; u < DEPTH; ++u) apply_entry<false, ROWS>(grp + (int64_t)u * kEntryDwords, ring[u], acc, nullptr);
    store_unit((int)nu - 1, acc);
}

void launch_multi(int units, int depth, int threads, bool tail, dim3 grid, hipStream_t stream, const ApplyArgs &a) {
#define ECX_MULTI(U, D, T, TL)                                                                   \
    if (units == U && depth == D && threads == T && tail == TL) {                                \
        note_kernel("k_gf_apply_multi", D, kTileRows, U, T, TL);                                  \
        hipLaunchKernelGGL((k_gf_apply_multi<D, kTileRows, U, T, TL>), grid, dim3(T), 0, stream, a); \
        return;                                                                                  \
    }
    ECX_MULTI(2, 8, 256, false) ECX_MULTI(4, 8, 256, false) ECX_MULTI(2, 20, 256, false) ECX_MULTI(4, 20, 256, false)
    ECX_MULTI(2, 8, 256, true) ECX_MULTI(4, 8, 256, true) ECX_MULTI(2, 4, 256, false) ECX_MULTI(4, 4, 256, false)
    ECX_MULTI(2, 8, 64, false) ECX_MULTI(4, 8, 64, false) ECX_MULTI(2, 4, 64, false) ECX_MULTI(4, 4, 64, false)
#undef ECX_MULTI
    throw Error(ECX_E_ILLEGAL_ARGUMENT, "no k_gf_apply_multi instance for this launch shape");
}

}  // namespace ecx
