// apply.hpp -- the one-workgroup-per-tile apply kernel (k_gf_apply) and its device
// helpers.  Included by kernels.hip (the tile-group kernels and launch_apply) and by
// the instantiation units apply_t256.hip / apply_t64.hip, which compile the
// k_gf_apply variants of each workgroup size in parallel.
#pragma once
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

// Byte-granular versions for the ragged tail / unaligned layouts.  A lane whose 16
// bytes all lie in range takes one 16-B access when its address is 16-B aligned, or
// four dword accesses when it is 4-B aligned (the tail chunk of a shard that is a
// multiple of 16 B but not of the chunk, e.g. 200,000 B); only the rest go by bytes.
typedef __attribute__((address_space(1))) uint32_t gu32;

__device__ __forceinline__ u32x4 load_partial(const uint8_t *p, int valid) {
    const uintptr_t al = (uintptr_t)p;
    if (valid == 16 && (al & 15) == 0) return load16(p);
    if (valid == 16 && (al & 3) == 0) {
        const gu32 *d = (const gu32 *)p;
        return (u32x4){d[0], d[1], d[2], d[3]};
    }
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
    const uintptr_t al = (uintptr_t)p;
    if (valid == 16 && (al & 15) == 0) {
        store16(p, v);
        return;
    }
    if (valid == 16 && (al & 3) == 0) {
        gu32 *d = (gu32 *)p;
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
        return;
    }
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
//
// ROWS < kTileRows: a specialisation for tiles of at most ROWS rows (small maps:
// RS decode of a few shards, LRC repair), whose accumulators then take 4*ROWS VGPRs.
template <bool TLDS, int ROWS = kTileRows>
__device__ __forceinline__ void apply_entry(cu32 *r, const u32x4 x, u32x4 (&acc)[ROWS], const uint2 *lt) {
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
    for (int o = 0; o < ROWS; ++o) {
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
        for (int o = 0; o < ROWS; ++o)
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
//   xcd_group 3: as 2 with runs of `run` consecutive units (all their tiles) per XCD,
//                for any map (single-tile maps: `run` neighbouring chunks per XCD).
__device__ __forceinline__ uint32_t logical_block(int xcd_group, uint32_t n_tiles, uint32_t run) {
    const uint32_t b = blockIdx.x;
    if (xcd_group == 0) return b;
    const uint32_t g = gridDim.x, xcd = b % 8, j = b / 8;
    if (xcd_group == 1) {
        const uint32_t q = g / 8, r = g % 8;
        return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
    }
    const uint32_t R = xcd_group == 3 ? run * n_tiles : n_tiles;
    const uint32_t full = (g / (8 * R)) * (8 * R);
    if (b >= full) return b;
    return ((j / R) * 8 + xcd) * R + (j % R);
}

// (stripe, chunk) of logical unit u of a launch over nst stripes x nc chunks (a bijection
// for every setting; a speed choice only):
//   stagger G > 1: G stripes interleaved unit by unit, stripe j of each group starting at
//                  chunk j*nc/G and wrapping, so the units in flight sit at G different
//                  offsets of their shards instead of one (many-stream maps whose shard
//                  pitch makes same-offset streams collide in HBM: scripts/addr_probe.hip);
//                  stripes past the last whole group keep the stripe-major order;
//   chunk_major:   chunk c of every stripe, then c + 1;
//   otherwise      stripe-major, a stripe's chunks back to back.
__device__ __forceinline__ void unit_of(uint32_t u, uint32_t nc, uint32_t nst, int chunk_major, uint32_t G,
                                        int64_t &s, int64_t &c) {
    if (G > 1) {
        const uint32_t span = G * nc, full = (nst / G) * span;
        if (u < full) {
            const uint32_t grp = u / span, w = u % span, j = w % G, k = w / G;
            s = (int64_t)grp * G + j;
            c = (int64_t)((k + (uint32_t)((uint64_t)j * nc / G)) % nc);
            return;
        }
    } else if (chunk_major) {
        s = u % nst;
        c = u / nst;
        return;
    }
    s = u / nc;
    c = u % nc;
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

template <bool SAFE, bool NTL, int NTS, int DEPTH, bool TLDS, int THREADS, int ROWS>
__device__ __forceinline__ void apply_tile(const ApplyArgs &a, cu32 *tile, uint64_t in_base, uint64_t out_base,
                                           uint32_t lane16, int valid, uint2 *lds_tab, bool store_lane = true) {
    const uint8_t *ib = reinterpret_cast<const uint8_t *>(in_base) + lane16;
    const uint32_t zoff = lane16;
    const int ebeg = (int)tile[0];
    const int ecnt = (int)tile[1];
    const int nrows = (int)tile[2];
    // TLDS kernels (multi-tile maps, where the multiply keeps the vector pipe busy)
    // load through a buffer descriptor over this workgroup's stripe chunk: the slot's
    // byte offset is a scalar soffset (s_mul of the plan's slot by the slot stride)
    // and the lane's 16 bytes the voffset, so an entry costs no VALU address
    // arithmetic (launch_apply checks that every offset fits 32 bits).  Padding
    // entries re-read the tile's first input (coefficient 0, an L2 hit) instead of
    // selecting the zero page.  Other kernels use 64-bit global addresses.
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t first_soff = 0;
    if constexpr (TLDS && !SAFE) {
        rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(in_base), 0, 0x7FFFFFFF, 0x00020000);
        if (ecnt > 0) first_soff = plan_ptr(a.entries)[(int64_t)ebeg * kEntryDwords] * (uint32_t)a.in_slot_stride;
    }
    auto load = [&](uint32_t slot) -> u32x4 {  // padding entries read the zero page
        if constexpr (TLDS && !SAFE) {
            const uint32_t soff = slot == kDummySlot ? first_soff : slot * (uint32_t)a.in_slot_stride;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)zoff, (int)soff, NTL ? 2 : 0);
            return (u32x4){(uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]};
        } else {
            const uint8_t *p = slot == kDummySlot ? a.zero_page + zoff : ib + (int64_t)slot * a.in_slot_stride;
            return SAFE ? load_partial(p, valid) : ld16<NTL>(p);
        }
    };

    u32x4 acc[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r] = (u32x4){0u, 0u, 0u, 0u};

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
                apply_entry<TLDS, ROWS>(r, ring[u], acc, ltab + (e0 + u) * kTileRows);
                ring[u] = load(r[DEPTH * kEntryDwords]);
            }
        }
#pragma unroll
        for (int u = 0; u < DEPTH; ++u)
            apply_entry<TLDS, ROWS>(ent + (int64_t)(last + u) * kEntryDwords, ring[u], acc,
                                    ltab + (last + u) * kTileRows);
    }
#pragma unroll
    for (int o = 0; o < ROWS; ++o) {
        if (o < nrows) {
            uint8_t *p = reinterpret_cast<uint8_t *>(out_base) + lane16 + (int64_t)tile[4 + o] * a.out_slot_stride;
            u32x4 v = acc[o];
            if (a.accumulate) v ^= SAFE ? load_partial(p, valid) : load16(p);  // wave-uniform branch
            if (SAFE) store_partial(p, v, valid);
            else if (store_lane) st16<NTS>(p, v);
        }
    }
}

// One workgroup = one (stripe, THREADS x 16-byte chunk, output tile): 256 threads and
// 4 KiB chunks by default, or one wave and 1 KiB chunks (ecx_tune "block_threads").
// TLDS: dynamic LDS holds the tile's low table dwords (launch_apply sizes it to the
// longest padded tile).
// ROWS < kTileRows: every tile of the map has at most ROWS rows (Shape::rows).
// TAIL (k_gf_apply_tail): the launch also covers a shard's partial last chunk (ApplyArgs::tail_chunk,
// its byte count a multiple of 16).  That workgroup covers the last THREADS x 16 bytes of the
// shard instead, and only the lanes on the partial chunk store -- a scalar base shift, no
// per-lane address change -- so the chunk needs no byte-safe launch of its own.  A kernel of its
// own: the branch alone, never taken, cost the other instances 0.1-1.2 % (profiles/r04_tail_ab.jsonl).
template <bool SAFE, bool NTL, int NTS, int DEPTH, bool TLDS, int THREADS, int ROWS, bool TAIL>
__device__ __forceinline__ void apply_unit(const ApplyArgs &a, uint2 *lds_tab) {
    const uint32_t w = logical_block(a.xcd_group, (uint32_t)a.n_tiles, (uint32_t)a.xcd_run);
    const uint32_t tl = w % (uint32_t)a.n_tiles;
    const uint32_t rest = w / (uint32_t)a.n_tiles;
    // (a launch covers whole stripes, so gridDim.x / (n_tiles * n_chunks) is its stripe count)
    const uint32_t nst = gridDim.x / ((uint32_t)a.n_tiles * (uint32_t)a.n_chunks);
    int64_t s, c;
    unit_of(rest, (uint32_t)a.n_chunks, nst, a.chunk_major, (uint32_t)a.stagger, s, c);
    s += a.stripe_begin;
    c += a.chunk_begin;
    int64_t cbase = c * (THREADS * 16);
    int valid = 16;
    bool store_lane = true;
    if (SAFE) {
        const int64_t v = a.nbytes - cbase - (int64_t)threadIdx.x * 16;
        valid = v <= 0 ? 0 : (v >= 16 ? 16 : (int)v);
    }
    if constexpr (TAIL) {
        if (c == a.tail_chunk) {
            cbase = a.nbytes - THREADS * 16;
            store_lane = threadIdx.x * 16 >= (uint32_t)(THREADS * 16 - a.tail_bytes);
        }
    }
    apply_tile<SAFE, NTL, NTS, DEPTH, TLDS, THREADS, ROWS>(a, plan_ptr(a.tiles) + __builtin_amdgcn_readfirstlane(tl) * kTileDwords,
                                            uniform64((uint64_t)(a.in + s * a.in_stripe_stride + cbase)),
                                            uniform64((uint64_t)(a.out + s * a.out_stripe_stride + cbase)),
                                            threadIdx.x * 16, valid, lds_tab, store_lane);
}

#define ECX_APPLY_BOUNDS(ROWS, DEPTH) \
    (ROWS < kTileRows ? (DEPTH >= 12 ? 5 : 6) : (DEPTH == 2 ? 8 : (DEPTH == 4 ? 6 : (DEPTH <= 8 ? 5 : (DEPTH <= 12 ? 4 : 3)))))

template <bool SAFE, bool NTL, int NTS, int DEPTH, bool TLDS, int THREADS, int ROWS>
__global__ void __launch_bounds__(THREADS, ECX_APPLY_BOUNDS(ROWS, DEPTH)) k_gf_apply(ApplyArgs a) {
    extern __shared__ uint2 lds_tab[];
    apply_unit<SAFE, NTL, NTS, DEPTH, TLDS, THREADS, ROWS, false>(a, lds_tab);
}

// Instances (apply_launch.inc): single-tile maps with NT loads and stores, SGPR tables and 8
// accumulator rows, depth 4 or 8; the parameters name the shape as k_gf_apply's do.
template <bool NTL, int NTS, int DEPTH, bool TLDS, int THREADS, int ROWS>
__global__ void __launch_bounds__(THREADS, ECX_APPLY_BOUNDS(ROWS, DEPTH)) k_gf_apply_tail(ApplyArgs a) {
    apply_unit<false, NTL, NTS, DEPTH, TLDS, THREADS, ROWS, true>(a, nullptr);
}

// Run-time launch shape of k_gf_apply, mapped onto a template instance by
// launch_shape_t<T> (apply_launch.inc; instantiated in apply_t256.hip / apply_t64.hip).
struct Shape {
    bool safe, ntl;
    int nts, depth;
    bool tlds;
    int threads;
    int rows;  // kTileRows, or 2 / 4 for maps whose tiles all have at most that many rows
    bool tail = false;  // k_gf_apply_tail: ApplyArgs::tail_chunk is in the launch
};

template <int T>
void launch_shape_t(const Shape &s, dim3 grid, size_t lds, hipStream_t stream, const ApplyArgs &a);

// k_gf_apply_skew (apply_skew.hip): single-tile maps, K = 2 or 4 chunks per workgroup
// with rotated chunk order; grid = stripes x chunk groups (ApplyArgs::n_chunks groups) x
// (4 KiB / (threads x 16)) columns.
void launch_skew(int k, int rows, int depth, bool ntl, int threads, dim3 grid, hipStream_t stream,
                 const ApplyArgs &a);

// k_gf_apply_multi (apply_multi.hip): single-tile maps, `units` consecutive (stripe, chunk) units per
// workgroup, one load ring across them; grid = ceil(ApplyArgs::multi_total / units).
void launch_multi(int units, int depth, int threads, bool tail, dim3 grid, hipStream_t stream, const ApplyArgs &a);

// k_gf_bits (apply_bits.hip): the bit-sliced kernel, 128-lane workgroups over 4 KiB
// chunks, ring depth 2 or 4; grid = stripes x chunks x tiles, as k_gf_apply.
void launch_bits(bool ntl, int depth, dim3 grid, hipStream_t stream, const ApplyArgs &a);

// k_gf_lut (apply_lut.hip): per-byte LDS table lookups -- mode 0 log/antilog, mode 1
// product rows (single-tile maps, `pairs` general coefficients) -- over n_units
// (stripe, 4 KiB chunk, tile) units of the depth-4 padded plan, persistent workgroups.
void launch_lut(int mode, bool ntl, int pairs, int64_t n_units, hipStream_t stream, const ApplyArgs &a);
constexpr int kLutMaxPairs = 256;  // mode 1: 64 KiB of product rows per workgroup at most

}  // namespace ecx
