// kernels.hip -- CDNA4 (gfx950) kernels of the GF(256) erasure engine.
//
// k_gf_apply applies one compiled GF(256) map (engine.hpp) to a batch of
// stripes.  It replaces the reference's per-(input,output) byte loop
// (InputOutputByteTableCodingLoop.java:27-29,39-41) and, through the planner,
// the whole stage sequence of ClayCodeErasureDecodingStep.doDecodeSingle /
// doDecodeMulti and ReedSolomon.decodeMissing in ONE pass over HBM:
//
//   * a 256-thread workgroup owns one (stripe, 4 KiB chunk, output tile);
//     each lane owns 16 consecutive byte positions of every sub-chunk;
//   * per input entry the lane issues one coalesced 16-B load (a wave moves
//     1 KiB contiguous per instruction) -- the next entry's load is issued
//     before the current one is consumed;
//   * the byte is split into 3+3+2 bits once per input, and every GF multiply
//     is three v_perm_b32 table lookups over four bytes (tables are wave-
//     uniform scalar loads from the plan) plus XOR into register accumulators;
//     coefficient 1 is a bare XOR (LRC local parity);
//   * no LDS, no MFMA: this is HBM-bound byte work.
#include "engine.hpp"

#include <type_traits>

namespace ecx {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

// The plan is read-only for the whole launch: read it through the constant
// address space so every access is a scalar (s_load) fetch even in loops that
// also store outputs (the compiler cannot otherwise prove no aliasing).
typedef const __attribute__((address_space(4))) uint32_t cu32;
typedef const __attribute__((address_space(4))) u32x8 cu32x8;
__device__ __forceinline__ cu32 *plan_ptr(const uint32_t *p) { return (cu32 *)p; }

__host__ __device__ __forceinline__ bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// Global-memory accesses go through address_space(1) pointers so they compile to
// global_load / global_store: a flat access also counts in lgkmcnt and may alias
// LDS, which would force full waits at every scalar-load or LDS wait.
typedef __attribute__((address_space(1))) u32x4 gu32x4;
typedef __attribute__((address_space(1))) uint8_t gu8;

__device__ __forceinline__ u32x4 load16(const uint8_t *p) { return *(const gu32x4 *)p; }

__device__ __forceinline__ void store16(uint8_t *p, u32x4 v) { *(gu32x4 *)p = v; }

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
    if (NT) return __builtin_nontemporal_load((const gu32x4 *)p);
    return *(const gu32x4 *)p;
}

// Store policy: 0 plain, 1 non-temporal, 2 non-temporal + sc0 sc1 (system scope:
// the line is written through and dropped from L2; inline asm, as no builtin sets
// the scope bits on a store).  Stores are the last vector-memory operations of a
// tile, so the asm store's vmcnt entry is never waited on by compiler-counted loads.
template <int NT>
__device__ __forceinline__ void st16(uint8_t *p, u32x4 v) {
    if constexpr (NT == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if constexpr (NT == 1) __builtin_nontemporal_store(v, (gu32x4 *)p);
    else *(gu32x4 *)p = v;
}

// Byte-granular versions for the ragged tail / unaligned layouts.
__device__ __forceinline__ u32x4 load_partial(const uint8_t *p, int valid) {
    const gu8 *q = (const gu8 *)p;
    uint32_t w[4] = {0, 0, 0, 0};
    for (int b = 0; b < valid; ++b) w[b >> 2] |= (uint32_t)q[b] << (8 * (b & 3));
    u32x4 r;
    r.x = w[0];
    r.y = w[1];
    r.z = w[2];
    r.w = w[3];
    return r;
}

__device__ __forceinline__ void store_partial(uint8_t *p, u32x4 v, int valid) {
    gu8 *q = (gu8 *)p;
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (int b = 0; b < valid; ++b) q[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
}

// c*b for four packed bytes: three 8-entry lookups (v_perm_b32 selects bytes
// 0-3 from its second operand and 4-7 from its first), XOR-folded with the
// gfx950 three-input v_bitop3_b32 (0x96 = a^b^c).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t gf_mac4(uint32_t acc, uint32_t t0a, uint32_t t0b, uint32_t t1a, uint32_t t1b,
                                            uint32_t t2, uint32_t i0, uint32_t i1, uint32_t i2) {
    const uint32_t p0 = __builtin_amdgcn_perm(t0b, t0a, i0);
    const uint32_t p1 = __builtin_amdgcn_perm(t1b, t1a, i1);
    const uint32_t p2 = __builtin_amdgcn_perm(t2, t2, i2);
    return xor3(acc, p0, xor3(p1, p2, 0u));
}

// One plan entry (input slot) against the tile's accumulators.  The 40 table
// dwords are fetched as five 8-dword scalar loads that straddle the per-row
// groups, so they are issued once per entry (not sunk into the per-row
// branches); rows without a coefficient are skipped by scalar branches.
//
// A v_perm_b32 reads at most one SGPR, so an 8-entry table (two dwords) needs one
// of its dwords in a VGPR.  With TLDS the low dwords of both 8-entry tables of
// every row come from the workgroup's LDS copy of the plan (`lt`, one broadcast
// ds_read_b64 per row); otherwise each is copied from its SGPR with a v_mov.
template <bool TLDS>
__device__ __forceinline__ void apply_entry(cu32 *r, const u32x4 x, u32x4 (&acc)[kTileRows], const uint2 *lt) {
    const uint32_t mmul = r[1], mone = r[2];
    cu32x8 *tv = (cu32x8 *)(r + 4);
    const u32x8 v0 = tv[0], v1 = tv[1], v2 = tv[2], v3 = tv[3], v4 = tv[4];
    const uint32_t tb[40] = {v0[0], v0[1], v0[2], v0[3], v0[4], v0[5], v0[6], v0[7], v1[0], v1[1],
                             v1[2], v1[3], v1[4], v1[5], v1[6], v1[7], v2[0], v2[1], v2[2], v2[3],
                             v2[4], v2[5], v2[6], v2[7], v3[0], v3[1], v3[2], v3[3], v3[4], v3[5],
                             v3[6], v3[7], v4[0], v4[1], v4[2], v4[3], v4[4], v4[5], v4[6], v4[7]};
    // The byte split is computed before the mask is known (issuing it ahead of the
    // scalar branch hides the plan's s_load latency; wrapping it in `if (mmul)` cost
    // 20-25 % on the Clay maps).
    const u32x4 i0 = x & 0x07070707u;
    const u32x4 i1 = (x >> 3) & 0x07070707u;
    const u32x4 i2 = (x >> 6) & 0x03030303u;
#pragma unroll
    for (int o = 0; o < kTileRows; ++o) {
        if (mmul & (1u << o)) {
            const uint32_t *t = tb + 5 * o;
            uint32_t t0a = t[0], t1a = t[2];
            if (TLDS) {
                const uint2 la = lt[o];
                t0a = la.x;
                t1a = la.y;
            }
            acc[o].x = gf_mac4(acc[o].x, t0a, t[1], t1a, t[3], t[4], i0.x, i1.x, i2.x);
            acc[o].y = gf_mac4(acc[o].y, t0a, t[1], t1a, t[3], t[4], i0.y, i1.y, i2.y);
            acc[o].z = gf_mac4(acc[o].z, t0a, t[1], t1a, t[3], t[4], i0.z, i1.z, i2.z);
            acc[o].w = gf_mac4(acc[o].w, t0a, t[1], t1a, t[3], t[4], i0.w, i1.w, i2.w);
        }
    }
    // Coefficient 1 (LRC parity, Clay dot nodes): a bare v_xor_b32 per dword for each
    // such row, behind scalar branches.  (A masked v_bitop3 over all rows would read
    // the mask from an SGPR, and gfx950 issues a VALU op with an SGPR operand at half
    // rate: profiles/r01_valu_probe_operands.jsonl.)
    if (mone) {
#pragma unroll
        for (int o = 0; o < kTileRows; ++o)
            if (mone & (1u << o)) acc[o] ^= x;
    }
}

// Logical work index of this workgroup (blocks b and b+8 share an XCD under the
// round-robin dispatch of MI355X; a speed choice only, every mapping is a bijection).
// Multi-tile maps re-read inputs across the tiles of one (stripe, chunk) unit:
//   xcd_group 0: identity -- the T tiles of a unit are spread over all 8 XCDs;
//   xcd_group 1: XCD x runs the contiguous x-th eighth of the grid;
//   xcd_group 2: XCD x runs whole units x, x+8, x+16, ..., each unit's T tiles
//                back to back, so a unit's re-reads meet in one XCD's L2 while
//                all XCDs stream neighbouring units.  Units past the last full
//                group of 8 keep the identity mapping.
__device__ __forceinline__ uint32_t logical_block(int xcd_group, uint32_t n_tiles) {
    const uint32_t b = blockIdx.x;
    if (xcd_group == 0) return b;
    const uint32_t g = gridDim.x, xcd = b % 8, j = b / 8;
    if (xcd_group == 1) {
        const uint32_t q = g / 8, r = g % 8;
        return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
    }
    const uint32_t full = (g / (8 * n_tiles)) * (8 * n_tiles);
    if (b >= full) return b;
    return ((j / n_tiles) * 8 + xcd) * n_tiles + (j % n_tiles);
}

// One output tile over the workgroup's (or wave's) lanes x 16 bytes of one stripe.
// `ib` / `ob` point at this lane's 16 bytes of slot 0; `zoff` is this lane's offset
// into the zero page (recomputed at each padding load rather than kept live).
// NTL / NTS: non-temporal loads / stores.  Outputs are never re-read, so stores
// are always streamed; loads are streamed only when the map has one tile (no
// input is read twice), otherwise the re-reads of other tiles hit the caches.
// Wave-uniform 64-bit value into SGPRs (the block-index arithmetic goes through
// VALU division; keeping the bases scalar frees VGPRs for the load ring).
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

template <bool SAFE, bool NTL, int NTS, int DEPTH, bool TLDS, int THREADS>
__device__ __forceinline__ void apply_tile(const ApplyArgs &a, cu32 *tile, uint64_t in_base, uint64_t out_base,
                                           uint32_t lane16, int valid, uint2 *lds_tab) {
    const uint8_t *ib = reinterpret_cast<const uint8_t *>(in_base) + lane16;
    const uint32_t zoff = lane16;
    const int ebeg = (int)tile[0];
    const int ecnt = (int)tile[1];
    const int nrows = (int)tile[2];
    auto load = [&](uint32_t slot) -> u32x4 {  // padding entries read the zero page
        const uint8_t *p = slot == kDummySlot ? a.zero_page + zoff : ib + (int64_t)slot * a.in_slot_stride;
        return SAFE ? load_partial(p, valid) : ld16<NTL>(p);
    };

    u32x4 acc[kTileRows];
#pragma unroll
    for (int r = 0; r < kTileRows; ++r) acc[r] = (u32x4){0u, 0u, 0u, 0u};

    cu32 *ent = plan_ptr(a.entries) + (int64_t)ebeg * kEntryDwords;
    // TLDS: the tile's {T0a, T1a} table dwords (kAtabDwords per entry) go to LDS.
    // Their global loads are issued before the load ring so that waiting for them
    // does not wait for the ring; the ring loads overlap the LDS store and barrier.
    const int n16 = TLDS ? ecnt * (kAtabDwords / 4) : 0;  // 16-B pieces
    const gu32x4 *asrc = (const gu32x4 *)(a.atab + (int64_t)ebeg * kAtabDwords);
    u32x4 apiece = (u32x4){0u, 0u, 0u, 0u};
    // LDS addresses are VGPRs.  A base the compiler sees as uniform lives in an SGPR
    // and is copied by a v_mov before every row's ds_read; adding threadIdx.x times
    // a run-time zero (ApplyArgs::lane_zero) keeps it in a VGPR, so each read is the
    // base plus an immediate offset.
    uint2 *ltab = lds_tab + threadIdx.x * (uint32_t)a.lane_zero;
    if (TLDS && (int)threadIdx.x < n16) apiece = asrc[threadIdx.x];
    // Load ring of DEPTH 16-B loads per lane.  Each tile's entry count is a
    // multiple of DEPTH (padded on upload), so the refill inside the loop is
    // unconditional: a slot is consumed, then refilled, keeping DEPTH-1 loads in
    // flight during every entry's arithmetic, with compile-time vmcnt counts and
    // no register copies.  The last group is peeled and issues no refill.
    if (ecnt > 0) {
        u32x4 ring[DEPTH];
#pragma unroll
        for (int u = 0; u < DEPTH; ++u) ring[u] = load(ent[u * kEntryDwords]);
        if (TLDS) {
            u32x4 *dst = (u32x4 *)lds_tab;
            if ((int)threadIdx.x < n16) dst[threadIdx.x] = apiece;
            for (int i = threadIdx.x + THREADS; i < n16; i += THREADS) dst[i] = asrc[i];  // > THREADS / 4 entries
            __syncthreads();
        }
        const int last = ecnt - DEPTH;
        for (int e0 = 0; e0 < last; e0 += DEPTH) {
#pragma unroll
            for (int u = 0; u < DEPTH; ++u) {
                cu32 *r = ent + (int64_t)(e0 + u) * kEntryDwords;
                apply_entry<TLDS>(r, ring[u], acc, ltab + (e0 + u) * kTileRows);
                ring[u] = load(r[DEPTH * kEntryDwords]);
            }
        }
#pragma unroll
        for (int u = 0; u < DEPTH; ++u)
            apply_entry<TLDS>(ent + (int64_t)(last + u) * kEntryDwords, ring[u], acc, ltab + (last + u) * kTileRows);
    }
#pragma unroll
    for (int o = 0; o < kTileRows; ++o) {
        if (o < nrows) {
            uint8_t *p = reinterpret_cast<uint8_t *>(out_base) + lane16 + (int64_t)tile[4 + o] * a.out_slot_stride;
            u32x4 v = acc[o];
            if (a.accumulate) v ^= SAFE ? load_partial(p, valid) : load16(p);  // wave-uniform branch
            if (SAFE) store_partial(p, v, valid);
            else st16<NTS>(p, v);
        }
    }
}

// One workgroup = one (stripe, THREADS x 16-byte chunk, output tile): 256 threads and
// 4 KiB chunks by default, or one wave and 1 KiB chunks (ecx_tune "block_threads").
// TLDS: dynamic LDS holds the tile's low table dwords (launch_apply sizes it to the
// longest padded tile).
template <bool SAFE, bool NTL, int NTS, int DEPTH, bool TLDS, int THREADS>
__global__ void __launch_bounds__(THREADS, DEPTH == 2 ? 8 : (DEPTH == 4 ? 6 : 5)) k_gf_apply(ApplyArgs a) {
    extern __shared__ uint2 lds_tab[];
    const uint32_t w = logical_block(a.xcd_group, (uint32_t)a.n_tiles);
    const uint32_t tl = w % (uint32_t)a.n_tiles;
    const uint32_t rest = w / (uint32_t)a.n_tiles;
    // chunk_major: consecutive units take the same chunk of consecutive stripes
    // (a launch covers whole stripes, so gridDim.x / (n_tiles * n_chunks) is its stripe count).
    const uint32_t nst = gridDim.x / ((uint32_t)a.n_tiles * (uint32_t)a.n_chunks);
    const int64_t c = a.chunk_begin + (int64_t)(a.chunk_major ? rest / nst : rest % (uint32_t)a.n_chunks);
    const int64_t s = a.stripe_begin + (int64_t)(a.chunk_major ? rest % nst : rest / (uint32_t)a.n_chunks);
    const int64_t cbase = c * (THREADS * 16);
    int valid = 16;
    if (SAFE) {
        const int64_t v = a.nbytes - cbase - (int64_t)threadIdx.x * 16;
        valid = v <= 0 ? 0 : (v >= 16 ? 16 : (int)v);
    }
    apply_tile<SAFE, NTL, NTS, DEPTH, TLDS, THREADS>(a, plan_ptr(a.tiles) + __builtin_amdgcn_readfirstlane(tl) * kTileDwords,
                                            uniform64((uint64_t)(a.in + s * a.in_stripe_stride + cbase)),
                                            uniform64((uint64_t)(a.out + s * a.out_stripe_stride + cbase)),
                                            threadIdx.x * 16, valid, lds_tab);
}

// Multi-tile maps: one workgroup = one (stripe, 1 KiB chunk, tile GROUP), one
// wave per tile.  The tiles of a group share inputs (Clay(10,4): 8 tiles read
// 208 distinct inputs 320 times), so instead of each wave loading its own
// inputs, the group's union of inputs streams through LDS exactly once:
//
//   stage k: wave w stores union[k*G + w] (held in its load ring) to LDS buffer
//            k&1 and refills the ring DEPTH stages ahead; barrier; every wave
//            applies the entries of its tile whose union position falls in
//            stage k, reading the 1 KiB rows from LDS.
//
// Two LDS buffers make one barrier per stage enough: buffer k&1 is rewritten at
// stage k+2, after every wave has passed the barrier of stage k+1.  HBM reads
// are the algorithmic bytes (1.0x instead of the re-read factor); the union is
// padded with zero-page entries to whole ring groups so refills are branch-free.
template <bool SAFE, int DEPTH>
__global__ void __launch_bounds__(64 * kWaveGroup, DEPTH == 4 ? 6 : 5) k_gf_apply_lds(ApplyArgs a) {
    __shared__ u32x4 stage[2][kWaveGroup][64];  // 16 KiB
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t G = blockDim.x >> 6;
    const uint32_t b = blockIdx.x;
    const uint32_t g = b % (uint32_t)a.n_groups;
    const uint32_t rest = b / (uint32_t)a.n_groups;
    cu32 *grp = plan_ptr(a.groups) + g * kGroupDwords;
    const uint32_t tl = __builtin_amdgcn_readfirstlane(grp[wave]);
    const int nst = (int)(grp[9] / G);  // stages; a multiple of DEPTH
    cu32 *uni = plan_ptr(a.unions) + grp[8];
    const int64_t c = a.chunk_begin + (int64_t)(rest % (uint32_t)a.n_chunks);
    const int64_t s = a.stripe_begin + (int64_t)(rest / (uint32_t)a.n_chunks);
    const int64_t cbase = c * kWaveChunkBytes;
    const uint32_t lane16 = lane * 16;
    int valid = 16;
    if (SAFE) {
        const int64_t v = a.nbytes - cbase - (int64_t)lane16;
        valid = v <= 0 ? 0 : (v >= 16 ? 16 : (int)v);
    }
    const uint8_t *ib = reinterpret_cast<const uint8_t *>(uniform64((uint64_t)(a.in + s * a.in_stripe_stride + cbase))) + lane16;
    auto load = [&](uint32_t slot) -> u32x4 {
        const uint8_t *p = slot == kDummySlot ? a.zero_page + lane16 : ib + (int64_t)slot * a.in_slot_stride;
        return SAFE ? load_partial(p, valid) : ld16<true>(p);  // each union input is read once: stream it
    };

    const bool active = tl != kNoTile;
    cu32 *tile = plan_ptr(a.tiles) + (active ? tl : 0u) * kTileDwords;
    const int ecnt = active ? (int)tile[3] : 0;
    cu32 *ent = plan_ptr(a.entries) + (int64_t)tile[0] * kEntryDwords;
    int e = 0;
    uint32_t next_pos = ecnt > 0 ? ent[3] : 0xFFFFFFFFu;

    u32x4 acc[kTileRows];
#pragma unroll
    for (int r = 0; r < kTileRows; ++r) acc[r] = (u32x4){0u, 0u, 0u, 0u};

    auto consume = [&](int k, int buf) {  // entries of this tile staged at stage k
        const uint32_t hi = (uint32_t)(k + 1) * G;
        while (next_pos < hi) {
            cu32 *r = ent + (int64_t)e * kEntryDwords;
            apply_entry<false>(r, stage[buf][next_pos - (uint32_t)k * G][lane], acc, nullptr);
            ++e;
            next_pos = e < ecnt ? r[kEntryDwords + 3] : 0xFFFFFFFFu;
        }
    };

    u32x4 ring[DEPTH];
#pragma unroll
    for (int u = 0; u < DEPTH; ++u) ring[u] = load(uni[u * G + wave]);
    const int last = nst - DEPTH;
    for (int k0 = 0; k0 < last; k0 += DEPTH) {
#pragma unroll
        for (int u = 0; u < DEPTH; ++u) {
            const int k = k0 + u;
            stage[u & 1][wave][lane] = ring[u];  // DEPTH is even: k & 1 == u & 1
            ring[u] = load(uni[(k + DEPTH) * G + wave]);
            __syncthreads();
            consume(k, u & 1);
        }
    }
#pragma unroll
    for (int u = 0; u < DEPTH; ++u) {
        stage[u & 1][wave][lane] = ring[u];
        __syncthreads();
        consume(last + u, u & 1);
    }
    if (!active) return;
    uint8_t *ob = reinterpret_cast<uint8_t *>(uniform64((uint64_t)(a.out + s * a.out_stripe_stride + cbase))) + lane16;
    const int nrows = (int)tile[2];
#pragma unroll
    for (int o = 0; o < kTileRows; ++o) {
        if (o < nrows) {
            uint8_t *p = ob + (int64_t)tile[4 + o] * a.out_slot_stride;
            u32x4 v = acc[o];
            if (a.accumulate) v ^= SAFE ? load_partial(p, valid) : load16(p);
            if (SAFE) store_partial(p, v, valid);
            else st16<true>(p, v);
        }
    }
}

// Multi-tile maps, tile groups without staging: one workgroup = one (stripe, 1 KiB
// chunk, tile GROUP), one wave per tile, each wave loading its own entries directly.
// The group's tiles share inputs, and each tile's entry list is ordered by the
// group's staging schedule (engine.cpp align_group), so the waves of a workgroup --
// on one CU -- request a shared input at about the same time and the repeats are
// served by that CU's L1 / the XCD's L2 rather than by another CU's fetch.  No LDS,
// no barriers: a wave whose slot in the group is empty exits at once.
template <bool SAFE, int DEPTH>
__global__ void __launch_bounds__(64 * kWaveGroup, DEPTH == 4 ? 6 : 5) k_gf_apply_grp(ApplyArgs a) {
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t b = blockIdx.x;
    const uint32_t g = b % (uint32_t)a.n_groups;
    const uint32_t rest = b / (uint32_t)a.n_groups;
    const uint32_t tl = __builtin_amdgcn_readfirstlane(plan_ptr(a.groups)[g * kGroupDwords + wave]);
    if (tl == kNoTile) return;
    const int64_t c = a.chunk_begin + (int64_t)(rest % (uint32_t)a.n_chunks);
    const int64_t s = a.stripe_begin + (int64_t)(rest / (uint32_t)a.n_chunks);
    const int64_t cbase = c * kWaveChunkBytes;
    const uint32_t lane16 = lane * 16;
    int valid = 16;
    if (SAFE) {
        const int64_t v = a.nbytes - cbase - (int64_t)lane16;
        valid = v <= 0 ? 0 : (v >= 16 ? 16 : (int)v);
    }
    apply_tile<SAFE, false, SAFE ? 0 : 1, DEPTH, false, 64>(
        a, plan_ptr(a.tiles) + tl * kTileDwords, uniform64((uint64_t)(a.in + s * a.in_stripe_stride + cbase)),
        uniform64((uint64_t)(a.out + s * a.out_stripe_stride + cbase)), lane16, valid, nullptr);
}

namespace {
// Run-time launch shape -> template instance of k_gf_apply.
struct Shape {
    bool safe, ntl;
    int nts, depth;
    bool tlds;
    int threads;
};

template <bool SAFE, bool NTL, int NTS, int D, bool TLDS, int T>
void launch_k(dim3 grid, size_t lds, hipStream_t stream, const ApplyArgs &a) {
    hipLaunchKernelGGL((k_gf_apply<SAFE, NTL, NTS, D, TLDS, T>), grid, dim3(T), lds, stream, a);
}

template <int T>
void launch_shape_t(const Shape &s, dim3 grid, size_t lds, hipStream_t stream, const ApplyArgs &a) {
    if (s.safe) {  // the byte-safe kernel's ring must match the plan's padding
        if (s.depth == 2) return launch_k<true, false, 0, 2, false, T>(grid, 0, stream, a);
        return launch_k<true, false, 0, 4, false, T>(grid, 0, stream, a);
    }
    auto by_depth = [&](auto ntl, auto nts) {
        constexpr bool L = decltype(ntl)::value;
        constexpr int S = decltype(nts)::value;
        if (s.depth == 8) {
            if (s.tlds) launch_k<false, L, S, 8, true, T>(grid, lds, stream, a);
            else launch_k<false, L, S, 8, false, T>(grid, 0, stream, a);
        } else if (s.depth == 2) {
            if (s.tlds) launch_k<false, L, S, 2, true, T>(grid, lds, stream, a);
            else launch_k<false, L, S, 2, false, T>(grid, 0, stream, a);
        } else {
            if (s.tlds) launch_k<false, L, S, 4, true, T>(grid, lds, stream, a);
            else launch_k<false, L, S, 4, false, T>(grid, 0, stream, a);
        }
    };
    using t_ = std::true_type;
    using f_ = std::false_type;
    if (s.ntl) {
        if (s.nts == 2) by_depth(t_{}, std::integral_constant<int, 2>{});
        else by_depth(t_{}, std::integral_constant<int, 1>{});
    } else if (s.nts == 2) by_depth(f_{}, std::integral_constant<int, 2>{});
    else if (s.nts == 1) by_depth(f_{}, std::integral_constant<int, 1>{});
    else by_depth(f_{}, std::integral_constant<int, 0>{});
}
}  // namespace

void launch_apply(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride, uint8_t *out,
                  int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes, int64_t nbytes,
                  hipStream_t stream, bool accumulate) {
    if (nstripes <= 0 || nbytes <= 0 || cm.map().n_out == 0) return;
    const Tuning &tu = tuning();
    const bool waves = cm.n_tiles() > 1 && cm.n_groups() > 0 && tu.wave_groups;
    const int threads = tu.block_threads == 64 ? 64 : kBlockThreads;
    // Ring depth: per map, or forced (ecx_tune "depth"); depth 2 exists for the
    // 256-thread one-workgroup-per-tile kernel only.
    int depth = tu.depth ? tu.depth : cm.preferred_depth();
    if (depth == 2 && (waves || threads != kBlockThreads)) depth = 4;
    const DevicePlan &plan = cm.plan_for_current_device(depth);
    const bool aligned = aligned16(in) && aligned16(out) && (in_stripe_stride % 16 == 0) &&
                         (in_slot_stride % 16 == 0) && (out_stripe_stride % 16 == 0) && (out_slot_stride % 16 == 0);
    // Multi-tile maps can run as tile groups (one wave per tile, 1 KiB chunks); otherwise
    // one workgroup per (stripe, chunk, tile) with 4 KiB (256 threads) or 1 KiB (64) chunks.
    const int64_t chunk = waves ? kWaveChunkBytes : threads * 16;
    const int64_t full = aligned ? nbytes / chunk : 0;               // in units of `chunk`
    const int64_t tail_chunks = (nbytes - full * chunk + chunk - 1) / chunk;

    ApplyArgs a;
    a.in = in;
    a.out = out;
    a.entries = plan.entries;
    a.tiles = plan.tiles;
    a.groups = plan.groups;
    a.unions = plan.unions;
    a.atab = plan.atab;
    a.lane_zero = 0;
    a.chunk_major = tu.chunk_major;
    a.n_groups = cm.n_groups();
    a.zero_page = zero_page_for_current_device();
    a.in_stripe_stride = in_stripe_stride;
    a.in_slot_stride = in_slot_stride;
    a.out_stripe_stride = out_stripe_stride;
    a.out_slot_stride = out_slot_stride;
    a.nbytes = nbytes;
    a.n_tiles = cm.n_tiles();
    a.xcd_group = a.n_tiles > 1 ? tu.xcd_group : 0;
    a.accumulate = accumulate ? 1 : 0;

    auto run = [&](bool safe, int64_t chunk_begin, int64_t n_chunks) {
        if (n_chunks <= 0) return;
        a.chunk_begin = chunk_begin;
        a.n_chunks = n_chunks;
        const int64_t per_stripe = n_chunks * (waves ? a.n_groups : a.n_tiles);
        const int64_t max_blocks = (int64_t)1 << 30;
        const int64_t stripes_per_launch = std::max<int64_t>(1, max_blocks / per_stripe);
        for (int64_t s0 = 0; s0 < nstripes; s0 += stripes_per_launch) {
            const int64_t ns = std::min(stripes_per_launch, nstripes - s0);
            a.stripe_begin = s0;
            const dim3 grid((unsigned)(ns * per_stripe));
            if (waves) {
                const dim3 blk(64 * cm.group_size());
                if (tu.wave_groups == 2) {  // direct loads, no LDS staging
                    if (safe) hipLaunchKernelGGL((k_gf_apply_grp<true, 4>), grid, blk, 0, stream, a);
                    else if (depth == 8) hipLaunchKernelGGL((k_gf_apply_grp<false, 8>), grid, blk, 0, stream, a);
                    else hipLaunchKernelGGL((k_gf_apply_grp<false, 4>), grid, blk, 0, stream, a);
                    continue;
                }
                if (safe) hipLaunchKernelGGL((k_gf_apply_lds<true, 4>), grid, blk, 0, stream, a);
                else if (depth == 8) hipLaunchKernelGGL((k_gf_apply_lds<false, 8>), grid, blk, 0, stream, a);
                else hipLaunchKernelGGL((k_gf_apply_lds<false, 4>), grid, blk, 0, stream, a);
                continue;
            }
            Shape s;
            s.safe = safe;
            // Non-temporal policy: 0 never; 1 auto (NT stores, NT loads for single-tile maps); 2 always.
            const int ntmode = tu.nontemporal == 2 ? 2 : (tu.nontemporal == 1 ? (a.n_tiles == 1 ? 2 : 1) : 0);
            s.ntl = ntmode == 2;
            s.nts = ntmode == 0 ? 0 : (tu.store_scope ? 2 : 1);
            s.depth = depth;
            s.tlds = !safe && plan.max_tile_entries > 0 && plan.max_tile_entries <= kMaxLdsTileEntries &&
                     (tu.lds_tables == 2 || (tu.lds_tables == 1 && a.n_tiles > 1));
            s.threads = threads;
            const size_t lds = s.tlds ? (size_t)plan.max_tile_entries * kAtabDwords * 4 : 0;
            if (threads == 64) launch_shape_t<64>(s, grid, lds, stream, a);
            else launch_shape_t<kBlockThreads>(s, grid, lds, stream, a);
        }
    };
    run(false, 0, full);
    run(true, full, tail_chunks);
    check_hip(hipGetLastError(), "k_gf_apply launch");
}

// ---------------------------------------------------------------- synthetic data
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Byte i of the region is byte (i % 8) of splitmix64(seed + (i / 8) * golden).
__global__ void __launch_bounds__(256) k_fill_random(uint8_t *dst, int64_t nbytes, uint64_t seed) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 16;
    for (int64_t off = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; off < nbytes; off += stride) {
        const uint64_t w0 = splitmix64(seed + (uint64_t)(off / 8) * 0x9E3779B97F4A7C15ull);
        const uint64_t w1 = splitmix64(seed + (uint64_t)(off / 8 + 1) * 0x9E3779B97F4A7C15ull);
        if (off + 16 <= nbytes && aligned16(dst + off)) {
            u32x4 v;
            v.x = (uint32_t)w0;
            v.y = (uint32_t)(w0 >> 32);
            v.z = (uint32_t)w1;
            v.w = (uint32_t)(w1 >> 32);
            store16(dst + off, v);
        } else {
            for (int b = 0; b < 16 && off + b < nbytes; ++b) dst[off + b] = (uint8_t)((b < 8 ? w0 : w1) >> (8 * (b & 7)));
        }
    }
}

void launch_fill_random(uint8_t *dst, int64_t nbytes, uint64_t seed, hipStream_t stream) {
    if (nbytes <= 0) return;
    const int64_t granules = (nbytes + 15) / 16;
    const unsigned blocks = (unsigned)std::min<int64_t>((granules + 255) / 256, 256 * 32);
    hipLaunchKernelGGL(k_fill_random, dim3(blocks), dim3(256), 0, stream, dst, nbytes, seed);
    check_hip(hipGetLastError(), "k_fill_random launch");
}

// ---------------------------------------------------------------- bandwidth probes (diagnostics)
// Each workgroup streams a 16 KiB contiguous region: 4 x (256 lanes x 16 B).
template <bool NT>
__global__ void __launch_bounds__(256) k_probe_read(const uint8_t *src, int64_t nbytes, uint32_t *sink) {
    const int64_t base = (int64_t)blockIdx.x * 16384 + threadIdx.x * 16;
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = ld16<NT>(src + base + k * 4096);
    u32x4 x = v[0] ^ v[1] ^ v[2] ^ v[3];
    uint32_t r = x.x ^ x.y ^ x.z ^ x.w;
    if (r == 0x9E3779B9u) atomicXor(sink, r);  // practically never taken; keeps the loads live
}

template <bool NT>
__global__ void __launch_bounds__(256) k_probe_copy(const uint8_t *src, uint8_t *dst, int64_t nbytes) {
    const int64_t base = (int64_t)blockIdx.x * 16384 + threadIdx.x * 16;
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = ld16<NT>(src + base + k * 4096);
#pragma unroll
    for (int k = 0; k < 4; ++k) st16<NT>(dst + base + k * 4096, v[k]);
}

void launch_probe(int kind, const uint8_t *src, uint8_t *dst, int64_t nbytes, bool nt, hipStream_t stream) {
    const unsigned blocks = (unsigned)(nbytes / 16384);
    if (!blocks) return;
    if (kind == 0) {
        if (nt) hipLaunchKernelGGL(k_probe_read<true>, dim3(blocks), dim3(256), 0, stream, src, nbytes, (uint32_t *)dst);
        else hipLaunchKernelGGL(k_probe_read<false>, dim3(blocks), dim3(256), 0, stream, src, nbytes, (uint32_t *)dst);
    } else {
        if (nt) hipLaunchKernelGGL(k_probe_copy<true>, dim3(blocks), dim3(256), 0, stream, src, dst, nbytes);
        else hipLaunchKernelGGL(k_probe_copy<false>, dim3(blocks), dim3(256), 0, stream, src, dst, nbytes);
    }
    check_hip(hipGetLastError(), "probe launch");
}

// ---------------------------------------------------------------- verification
__global__ void __launch_bounds__(256) k_count_mismatch(const uint8_t *a, int64_t a_stride, const uint8_t *b,
                                                        int64_t b_stride, int64_t nrows, int64_t row_bytes,
                                                        uint64_t *count) {
    uint64_t n = 0;
    const int64_t total = nrows * row_bytes;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int64_t r = i / row_bytes, c = i - r * row_bytes;
        n += a[r * a_stride + c] != (b ? b[r * b_stride + c] : 0);
    }
    for (int sh = 32; sh > 0; sh >>= 1) n += __shfl_xor(n, sh);
    if ((threadIdx.x & 63) == 0 && n) atomicAdd((unsigned long long *)count, (unsigned long long)n);
}

void launch_count_mismatch(const uint8_t *a, int64_t a_stride, const uint8_t *b, int64_t b_stride, int64_t nrows,
                           int64_t row_bytes, uint64_t *d_count, hipStream_t stream) {
    const int64_t total = nrows * row_bytes;
    if (total <= 0) return;
    const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(k_count_mismatch, dim3(blocks), dim3(256), 0, stream, a, a_stride, b, b_stride, nrows, row_bytes,
                       d_count);
    check_hip(hipGetLastError(), "k_count_mismatch launch");
}

}  // namespace ecx
