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
#include "apply.hpp"
#include "map_rtc.hpp"

namespace ecx {

#if ECX_DIAG  // measured and rejected: `make DIAG=1` only
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
#endif  // ECX_DIAG

// Wide tiles: one 256-thread workgroup = one (stripe, 4 KiB chunk, pair of 8-row
// tiles A and B).  Each input of the pair's union is loaded once and applied to
// both halves (A's and B's entry tables), so a pair that shares inputs reads each of
// them once instead of twice.  16 accumulator rows; otherwise the loop of apply_tile
// (zero-page-padded ring of DEPTH loads, SGPR tables).
template <bool SAFE, bool NTL, int NTS, int DEPTH>
__global__ void __launch_bounds__(kBlockThreads, 4) k_gf_apply_wide(ApplyArgs a) {
    const uint32_t w = blockIdx.x % (uint32_t)a.n_wide;
    const uint32_t rest = blockIdx.x / (uint32_t)a.n_wide;
    const int64_t c = a.chunk_begin + (int64_t)(rest % (uint32_t)a.n_chunks);
    const int64_t s = a.stripe_begin + (int64_t)(rest / (uint32_t)a.n_chunks);
    const int64_t cbase = c * kChunkBytes;
    const uint32_t lane16 = threadIdx.x * 16;
    int valid = 16;
    if (SAFE) {
        const int64_t v = a.nbytes - cbase - (int64_t)lane16;
        valid = v <= 0 ? 0 : (v >= 16 ? 16 : (int)v);
    }
    cu32 *rec = plan_ptr(a.wtiles) + __builtin_amdgcn_readfirstlane(w) * kWideTileDwords;
    const uint64_t in_base = uniform64((uint64_t)(a.in + s * a.in_stripe_stride + cbase));
    const uint8_t *ib = reinterpret_cast<const uint8_t *>(in_base) + lane16;
    // Buffer-descriptor addressing as in apply_tile's TLDS kernels (apply.hpp): the
    // slot offset is a scalar soffset, padding re-reads the pair's first input.
    cu32 *went = plan_ptr(a.wentries) + (int64_t)rec[0] * kWideEntryDwords;
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t first_soff = 0;
    if constexpr (!SAFE) {
        rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(in_base), 0, 0x7FFFFFFF, 0x00020000);
        if (rec[1] > 0) first_soff = went[0] * (uint32_t)a.in_slot_stride;  // a pair with no inputs loads nothing
    }
    auto load = [&](uint32_t slot) -> u32x4 {
        if constexpr (!SAFE) {
            const uint32_t soff = slot == kDummySlot ? first_soff : slot * (uint32_t)a.in_slot_stride;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)lane16, (int)soff, NTL ? 2 : 0);
            return (u32x4){(uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]};
        } else {
            const uint8_t *p = slot == kDummySlot ? a.zero_page + lane16 : ib + (int64_t)slot * a.in_slot_stride;
            return load_partial(p, valid);
        }
    };
    u32x4 acc_a[kTileRows], acc_b[kTileRows];
#pragma unroll
    for (int r = 0; r < kTileRows; ++r) acc_a[r] = acc_b[r] = (u32x4){0u, 0u, 0u, 0u};
    const int ecnt = (int)rec[1];
    cu32 *ent = plan_ptr(a.wentries) + (int64_t)rec[0] * kWideEntryDwords;
    if (ecnt > 0) {
        u32x4 ring[DEPTH];
#pragma unroll
        for (int u = 0; u < DEPTH; ++u) ring[u] = load(ent[u * kWideEntryDwords]);
        const int last = ecnt - DEPTH;
        for (int e0 = 0; e0 < last; e0 += DEPTH) {
#pragma unroll
            for (int u = 0; u < DEPTH; ++u) {
                cu32 *r = ent + (int64_t)(e0 + u) * kWideEntryDwords;
                apply_entry<false>(r, ring[u], acc_a, nullptr);
                apply_entry<false>(r + kEntryDwords, ring[u], acc_b, nullptr);
                ring[u] = load(r[DEPTH * kWideEntryDwords]);
            }
        }
#pragma unroll
        for (int u = 0; u < DEPTH; ++u) {
            cu32 *r = ent + (int64_t)(last + u) * kWideEntryDwords;
            apply_entry<false>(r, ring[u], acc_a, nullptr);
            apply_entry<false>(r + kEntryDwords, ring[u], acc_b, nullptr);
        }
    }
    uint8_t *ob = reinterpret_cast<uint8_t *>(uniform64((uint64_t)(a.out + s * a.out_stripe_stride + cbase))) + lane16;
    const int rows_a = (int)rec[2], rows_b = (int)rec[3];
#pragma unroll
    for (int o = 0; o < kTileRows; ++o) {
        if (o < rows_a) {
            uint8_t *p = ob + (int64_t)rec[4 + o] * a.out_slot_stride;
            u32x4 v = acc_a[o];
            if (a.accumulate) v ^= SAFE ? load_partial(p, valid) : load16(p);
            if (SAFE) store_partial(p, v, valid);
            else st16<NTS>(p, v);
        }
        if (o < rows_b) {
            uint8_t *p = ob + (int64_t)rec[12 + o] * a.out_slot_stride;
            u32x4 v = acc_b[o];
            if (a.accumulate) v ^= SAFE ? load_partial(p, valid) : load16(p);
            if (SAFE) store_partial(p, v, valid);
            else st16<NTS>(p, v);
        }
    }
}

#if ECX_DIAG  // measured and rejected: `make DIAG=1` only
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
    apply_tile<SAFE, false, SAFE ? 0 : 1, DEPTH, false, 64, kTileRows>(
        a, plan_ptr(a.tiles) + tl * kTileDwords, uniform64((uint64_t)(a.in + s * a.in_stripe_stride + cbase)),
        uniform64((uint64_t)(a.out + s * a.out_stripe_stride + cbase)), lane16, valid, nullptr);
}
#endif  // ECX_DIAG

namespace {
// May a partial last chunk run in the main launch (apply.hpp: that workgroup re-reads the end of
// the previous chunk)?  Only if no output byte of the launch is an input byte of it: disjoint
// buffers, or one buffer laid out as [stripe][slot][bytes] whose output slots are not inputs.
bool outputs_never_read(const LinearMap &m, const uint8_t *in, int64_t iss, int64_t isl, const uint8_t *out,
                        int64_t oss, int64_t osl, int64_t nstripes, int64_t nbytes) {
    if (iss < 0 || isl < 0 || oss < 0 || osl < 0) return false;
    int max_in = 0, max_out = 0;
    for (int v : m.in_slot) max_in = std::max(max_in, v);
    for (int v : m.out_slot) max_out = std::max(max_out, v);
    const uintptr_t in_lo = (uintptr_t)in, out_lo = (uintptr_t)out;
    const uintptr_t in_hi = in_lo + (uintptr_t)((nstripes - 1) * iss + (int64_t)max_in * isl + nbytes);
    const uintptr_t out_hi = out_lo + (uintptr_t)((nstripes - 1) * oss + (int64_t)max_out * osl + nbytes);
    if (in_hi <= out_lo || out_hi <= in_lo) return true;
    const int max_slot = std::max(max_in, max_out);
    if (in != out || iss != oss || isl != osl || isl < nbytes || iss < (int64_t)(max_slot + 1) * isl) return false;
    for (int o : m.out_slot)
        for (int i : m.in_slot)
            if (o == i) return false;
    return true;
}

// pick: -1 = the static rules (skew on 4 MiB-multiple input slot pitches, one-wave
// workgroups for narrow maps otherwise); else shape + 8 * stagger with shape 0 = 256-thread
// workgroups over 4 KiB chunks, 1 = skewed chunks, 2 = one-wave workgroups over 1 KiB
// chunks, 3 = skewed chunks on one-wave workgroups (1 KiB columns, diagnostic build), and
// stagger the unit order (apply.hpp unit_of) -- the per-layout candidates
void launch_apply_core(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                       uint8_t *out, int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes,
                       int64_t nbytes, hipStream_t stream, bool accumulate, int pick,
                       hipEvent_t probe_start = nullptr) {
    if (nstripes <= 0 || nbytes <= 0 || cm.map().n_out == 0) return;
    const Tuning &tu = tuning();
    // (the lab kernels -- tile groups, bit-sliced, LDS lookup tables, residency caps -- exist
    // only in the diagnostic build, `make DIAG=1`; their knobs are refused otherwise)
    const bool waves = ECX_DIAG && cm.n_tiles() > 1 && cm.n_groups() > 0 && tu.wave_groups;
    // Non-temporal policy: 0 never; 1 auto (NT stores, NT loads for single-tile maps); 2 always.
    const int ntmode = tu.nontemporal == 2 ? 2 : (tu.nontemporal == 1 ? (cm.n_tiles() == 1 ? 2 : 1) : 0);
    const int nts = ntmode == 0 ? 0 : (tu.store_scope ? 2 : 1);
    // Launch shapes that exist (apply_launch.inc); anything else is clamped here.
    // Workgroup size: 256 threads over 4 KiB chunks; one wave over 1 KiB chunks when forced
    // (64) or, in auto (0), for single-tile maps of <= 2 rows over >= 8 inputs whose slot
    // pitch is not a 4 MiB multiple (RS(12,4) decode on its padded pitch: +2.4-2.8 %; every
    // other BASELINE map -- LRC encode's 4 rows included -- is 3-8 % slower on one wave,
    // profiles/r02_block_threads.jsonl).  3-row maps (RS(17,3) encode) run on 4 KiB
    // workgroups: 0-4 % faster than one wave once the byte-safe tail took 16-B accesses
    // (profiles/r03_rs_km.jsonl, r03_rs173_pitch.jsonl, r03_rs173_ab.jsonl).
    const int shape = pick < 0 ? -1 : pick & 7;
    const bool skew_pitch =
        pick < 0 ? in_slot_stride % ((int64_t)4 << 20) == 0 && cm.map().n_in >= 4 : (shape == 1 || shape == 3);
    const bool one_wave = tu.block_threads == 64 ||
                          (tu.block_threads == 0 && cm.n_tiles() == 1 && tu.bitslice != 2 && !tu.lds_lut &&
                           (pick < 0 ? cm.max_tile_rows() <= 2 && cm.map().n_in >= 8 && !skew_pitch
                                     : (shape == 2 || shape == 3)));
    int threads = one_wave && nts == 1 ? 64 : kBlockThreads;
    int rows = kTileRows;
    // Small-row kernel variants: forced (1), or auto (2) for maps of <= 2 rows over <= 4
    // inputs (LRC block repair: +2.5-3 %; wider narrow maps gain nothing or lose,
    // profiles/r02_small_tiles_ab.jsonl).
    const bool small = tu.small_tiles == 1 ||
                       (tu.small_tiles == 2 && cm.max_tile_rows() <= 2 && cm.map().n_in <= 4 && cm.n_tiles() == 1);
    if (small && !waves && threads == kBlockThreads && ntmode == 2 && nts == 1)
        rows = cm.max_tile_rows() <= 2 ? 2 : (cm.max_tile_rows() <= 4 ? 4 : kTileRows);
    int depth = tu.depth ? tu.depth : cm.preferred_depth();
    if (rows < kTileRows) {
        if (depth != 4 && depth != 8 && depth != 12) depth = 4;
    } else {
        if (depth == 2 && (waves || threads != kBlockThreads || nts != 1)) depth = 4;
        // deep rings (10-24) exist for single-tile maps with NT loads and stores and SGPR tables
        if (depth > 8 && (cm.n_tiles() != 1 || threads != kBlockThreads || ntmode != 2 ||
                          (nts != 1 && !(nts == 2 && depth == 20)) ||
                          tu.lds_tables == 2))
            depth = 8;
    }
    // Wide tiles (pairs of 8-row tiles) for multi-tile maps: auto (1) when pairing
    // saves at least 1/6 of the input reads (Clay(4,2) encode / repair {0,3}: 40 reads
    // over a 32-column union, +7-10 %; Clay(10,4) shortened: 80 over 76, where the
    // 16-row workgroup is 2x slower -- profiles/r01_wide.jsonl), forced (2), off (0).
    const bool offsets32 = in_slot_stride >= 0 &&
                           (int64_t)cm.max_in_slot() * in_slot_stride + kChunkBytes <= 0x7FFFFFFF;
    bool wide = (tu.wide_tiles == 2 || (tu.wide_tiles == 1 && cm.wide_sharing() >= 1.2)) && !waves &&
                      cm.n_wide_tiles() > 0 && threads == kBlockThreads && rows == kTileRows && offsets32;
    if (wide) depth = tu.depth == 8 || tu.depth == 4 ? tu.depth : cm.wide_depth();
    const bool aligned = aligned16(in) && aligned16(out) && (in_stripe_stride % 16 == 0) &&
                         (in_slot_stride % 16 == 0) && (out_stripe_stride % 16 == 0) && (out_slot_stride % 16 == 0);
    // Skewed chunk order (k_gf_apply_skew) for single-tile maps: forced (2 / 4 chunks),
    // or auto (1) when the input slot pitch is a multiple of 4 MiB -- the layouts whose
    // same-offset streams collide in HBM, where rotation recovers +10-17 %; on other
    // pitches it helps or costs by layout (profiles/r01_pitch_sweep.jsonl).  Auto needs
    // at least 4 input streams: one helper's partial sum (1 input) only loses.
    const bool skew_auto = skew_pitch;
    int skew = tu.skew_chunks == 1 ? (skew_auto ? 4 : 0) : tu.skew_chunks;
    const int skew_rows = cm.max_tile_rows() <= 2 ? 2 : (cm.max_tile_rows() <= 4 ? 4 : kTileRows);
    if (skew == 4 && skew_rows == kTileRows) skew = 2;  // 8 rows x 4 chunks would not fit the VGPRs
    // (one-wave workgroups take the skewed order over 1 KiB columns of <= 4-row maps in the
    // diagnostic build only: measured slower than the selected shapes)
    if (!(skew && cm.n_tiles() == 1 && !waves &&
          (threads == kBlockThreads || (ECX_DIAG && threads == 64 && skew_rows <= 4)) &&
          ntmode == 2 && nts == 1 && aligned && nbytes >= skew * kChunkBytes))
        skew = 0;
    if (skew) depth = depth == 4 || skew_rows == kTileRows ? 4 : 8;
    // Bit-sliced kernel (k_gf_bits, apply_bits.hip) for the full 4 KiB chunks: forced (2)
    // wherever it can run, or auto (1) for multi-tile maps that do not pair into wide
    // tiles -- the maps with many coefficients per input, where the split-table
    // kernel is bound by vector issue (Clay(10,4)).  Its ring is 4
    // deep (2 on request); the byte-safe tail then runs on the same padded plan.
    // (the chunk accounting below is in 4 KiB chunks only for 256-thread shapes)
    const bool bits_ok = aligned && offsets32 && !waves && threads == kBlockThreads && ntmode != 0 &&
                         nbytes >= kChunkBytes;
    bool bits = ECX_DIAG && bits_ok && !skew &&
                      (tu.bitslice == 2 || (tu.bitslice == 1 && cm.n_tiles() > 1 && !wide));
    if (bits) {
        depth = tu.depth == 2 ? 2 : 4;
        wide = false;  // the byte-safe tail runs k_gf_apply over the same padded tiles
    }
    // Generated bit-plane kernel (k_map_planes, map_rtc.hpp) for the full 4 KiB chunks:
    // forced (2) wherever it fits, or auto (1) for multi-tile maps of <= 16 rows whose
    // coefficients outnumber their used inputs 4x or more -- where the split tables are
    // bound by vector issue (the Clay(4,2) two-node repairs: 184 coefficients over 32
    // inputs) -- on batches big enough (>= 64 MiB of input) to amortise the one-time
    // hiprtc compile.  The byte-safe tail runs on the composed plan below.
    bool planes = false;
    if (tu.map_planes && aligned && offsets32 && !waves && nbytes >= kChunkBytes &&
        cm.map().n_out <= kPlanesMaxRows) {
        if (tu.map_planes == 2) {
            planes = true;
        } else if (cm.n_tiles() > 1) {
            int used = 0;
            for (int j = 0; j < cm.map().n_in; ++j)
                for (int o = 0; o < cm.map().n_out; ++o)
                    if (cm.map().at(o, j)) {
                        ++used;
                        break;
                    }
            planes = cm.map().nnz() >= 4 * used && nstripes * (nbytes / kChunkBytes) * used >= 16384;
        }
        // auto falls back to the composed kernels when the generated one cannot be built here
        planes = planes && cm.planes() != nullptr && (tu.map_planes == 2 || cm.planes()->available(accumulate));
    }
    if (planes) {
        skew = 0;
        bits = false;
    }
    // LDS lookup-table kernel (k_gf_lut, apply_lut.hip), forced only: 1 = log/antilog, 2 =
    // product rows for single-tile maps of <= kLutMaxPairs general coefficients.  Full
    // 4 KiB chunks of aligned layouts on the depth-4 padded plan; the byte-safe tail
    // runs k_gf_apply on the same plan.
    int lut_pairs = 0;  // general coefficients (counted only when the kernel is asked for)
    if (tu.lds_lut == 2)
        for (int o = 0; o < cm.map().n_out; ++o)
            for (int j = 0; j < cm.map().n_in; ++j) lut_pairs += cm.map().at(o, j) > 1;
    const bool lut = ECX_DIAG && tu.lds_lut && aligned && !waves && nbytes >= kChunkBytes && threads == kBlockThreads &&
                     (tu.lds_lut == 1 || (cm.n_tiles() == 1 && lut_pairs <= kLutMaxPairs));
    if (lut) {
        planes = bits = wide = false;
        skew = 0;
        depth = 4;
    }
    // Several units per workgroup with one ring across them (k_gf_apply_multi, ecx_tune "units"):
    // single-tile maps on the default NT shape, rings of 4 / 8 (and 20 on 256 threads)
    [[maybe_unused]] const bool multi = ECX_DIAG && tu.units > 1 && cm.n_tiles() == 1 && !waves && !wide && !bits && !lut && !planes && !skew &&
                       rows == kTileRows && ntmode == 2 && nts == 1 && tu.lds_tables != 2 &&
                       (depth == 4 || depth == 8 || (depth == 20 && threads == kBlockThreads));
    const DevicePlan &plan = cm.plan_for_current_device(depth);
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
    a.wentries = plan.wentries;
    a.wtiles = plan.wtiles;
    a.bentries = plan.bentries;
    a.n_wide = cm.n_wide_tiles();
    a.lane_zero = 0;
    a.chunk_major = tu.chunk_major;
    a.stagger = pick < 0 ? tu.stagger : pick >> 3;
    a.n_groups = cm.n_groups();
    a.zero_page = zero_page_for_current_device();
    a.in_stripe_stride = in_stripe_stride;
    a.in_slot_stride = in_slot_stride;
    a.out_stripe_stride = out_stripe_stride;
    a.out_slot_stride = out_slot_stride;
    a.nbytes = nbytes;
    a.n_tiles = cm.n_tiles();
    // Single-tile maps whose input slots are not 128-B aligned: consecutive chunks of a slot
    // share a boundary cache line, fetched twice from HBM unless both chunks run on one XCD
    // (one L2) -- runs of consecutive units per XCD (RS(17,3) on 200,000-B shards: reads
    // 1.035x the algorithmic bytes, +5 % with the runs, profiles/r03_rs173_xcd_align.jsonl).
    const bool misaligned128 = ((uintptr_t)in % 128) != 0 || in_stripe_stride % 128 != 0 || in_slot_stride % 128 != 0;
    a.xcd_group = (a.n_tiles > 1 || tu.xcd_group == 3)
                      ? tu.xcd_group
                      : (tu.xcd_group == 0 && tu.xcd_misaligned && misaligned128 ? 3 : 0);
    a.xcd_run = tu.xcd_run;
    a.accumulate = accumulate ? 1 : 0;
    a.tail_chunk = -1;
    a.tail_bytes = 0;
    a.multi_total = 0;

    bool tail_launch = false;  // the next non-safe run covers the partial last chunk (k_gf_apply_tail)
    auto run = [&](bool safe, int64_t chunk_begin, int64_t n_chunks) {
        if (n_chunks <= 0) return;
        a.chunk_begin = chunk_begin;
        a.n_chunks = n_chunks;
        const int64_t per_stripe = n_chunks * (waves ? a.n_groups : (wide ? a.n_wide : a.n_tiles));
        const int64_t max_blocks = (int64_t)1 << 30;
        const int64_t stripes_per_launch = std::max<int64_t>(1, max_blocks / per_stripe);
        for (int64_t s0 = 0; s0 < nstripes; s0 += stripes_per_launch) {
            const int64_t ns = std::min(stripes_per_launch, nstripes - s0);
            a.stripe_begin = s0;
            const dim3 grid((unsigned)(ns * per_stripe));
#if ECX_DIAG
            if (waves) {
                const dim3 blk(64 * cm.group_size());
                if (!safe) note_kernel(tu.wave_groups == 2 ? "k_gf_apply_grp" : "k_gf_apply_lds", false, depth == 8 ? 8 : 4);
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
            if (bits && !safe) {
                if (chunk != kChunkBytes) throw Error(ECX_E_ILLEGAL_ARGUMENT, "k_gf_bits needs 4 KiB chunks");
                launch_bits(ntmode == 2, depth, grid, stream, a);
                continue;
            }
#endif  // ECX_DIAG
            if (wide) {
                const dim3 blk(kBlockThreads);
                const bool ntl = ntmode == 2 || (ntmode == 1 && a.n_wide == 1);  // one pair: no re-reads
                if (!safe) note_kernel("k_gf_apply_wide", false, ntl, 1, depth);
                if (safe) hipLaunchKernelGGL((k_gf_apply_wide<true, false, 0, 4>), grid, blk, 0, stream, a);
                else if (depth == 8) {
                    if (ntl) hipLaunchKernelGGL((k_gf_apply_wide<false, true, 1, 8>), grid, blk, 0, stream, a);
                    else hipLaunchKernelGGL((k_gf_apply_wide<false, false, 1, 8>), grid, blk, 0, stream, a);
                } else {
                    if (ntl) hipLaunchKernelGGL((k_gf_apply_wide<false, true, 1, 4>), grid, blk, 0, stream, a);
                    else hipLaunchKernelGGL((k_gf_apply_wide<false, false, 1, 4>), grid, blk, 0, stream, a);
                }
                continue;
            }
#if ECX_DIAG
            if (multi && !safe) {  // measured slower on every single-tile map: DESIGN.md section 4.5
                a.multi_total = ns * per_stripe;
                launch_multi(tu.units, depth, threads, tail_launch,
                             dim3((unsigned)((a.multi_total + tu.units - 1) / tu.units)), stream, a);
                continue;
            }
#endif
            Shape s;
            s.safe = safe;
            s.ntl = ntmode == 2;
            s.nts = nts;
            s.depth = depth;
            // TLDS kernels address inputs through a buffer descriptor with 32-bit slot
            // offsets (apply.hpp): every slot's chunk must lie within 2 GiB of the stripe chunk.
            s.tlds = !safe && rows == kTileRows && plan.max_tile_entries > 0 && offsets32 &&
                     plan.max_tile_entries <= kMaxLdsTileEntries &&
                     (tu.lds_tables == 2 || (tu.lds_tables == 1 && a.n_tiles > 1));
            s.threads = threads;
            s.rows = rows;
            s.tail = tail_launch && !safe;
            // Residency cap (ecx_tune "occ_lds"): dummy LDS per workgroup.  Auto: the many-stream
            // single-tile maps (>= 8 inputs, rings of <= 8 loads) at 4 waves per SIMD -- 4
            // 256-thread or 16 one-wave workgroups per CU -- instead of the 5 their registers allow.
            size_t occ = ECX_DIAG && tu.occ_lds > 0 ? (size_t)tu.occ_lds : 0;
            if (ECX_DIAG && tu.occ_lds < 0 && !safe && a.n_tiles == 1 && cm.map().n_in >= 8 && depth <= 8)
                occ = kLdsPerCu / (kOccWavesPerSimd * kSimdsPerCu / (threads / 64));
            const size_t lds = (s.tlds ? (size_t)plan.max_tile_entries * kAtabDwords * 4 : 0) + occ;
            if (threads == 64) launch_shape_t<64>(s, grid, lds, stream, a);
            else launch_shape_t<kBlockThreads>(s, grid, lds, stream, a);
        }
    };
    const uint64_t notes0 = kernel_notes();
    int64_t first = 0;  // first full chunk left to the one-chunk kernels
    // a layout probe's start: after the host-side work (plan upload on first use), so the
    // probe times the kernels alone; a failed record only drops that probe
    if (probe_start && hipEventRecord(probe_start, stream) != hipSuccess) (void)hipGetLastError();
#if ECX_DIAG
    if (lut) {
        a.chunk_begin = 0;
        a.n_chunks = full;
        a.stripe_begin = 0;
        launch_lut(tu.lds_lut - 1, ntmode == 2, lut_pairs, nstripes * full * a.n_tiles, stream, a);
        first = full;
    }
#endif
    if (planes) {
        const int64_t n4k = nbytes / kChunkBytes;
        cm.planes()->launch(in, in_stripe_stride, in_slot_stride, out, out_stripe_stride, out_slot_stride, nstripes, n4k,
                            accumulate, stream);
        first = n4k * kChunkBytes / chunk;
    }
    if (skew) {
        const int64_t cols = kChunkBytes / chunk;  // workgroups per 4 KiB chunk (4 for one wave)
        const int64_t groups = full / (skew * cols);
        a.chunk_begin = 0;
        a.n_chunks = groups;
        const int64_t max_blocks = (int64_t)1 << 30;
        const int64_t stripes_per_launch = std::max<int64_t>(1, max_blocks / (groups * cols));
        for (int64_t s0 = 0; s0 < nstripes; s0 += stripes_per_launch) {
            const int64_t ns = std::min(stripes_per_launch, nstripes - s0);
            a.stripe_begin = s0;
            launch_skew(skew, skew_rows, depth, true, threads, dim3((unsigned)(ns * groups * cols)), stream, a);
        }
        first = groups * skew * cols;  // in units of `chunk`
    }
    // A partial last chunk whose byte count is a multiple of 16 (RS(17,3) on the published
    // 200,000-B shards: 48 full 4 KiB chunks and 3,392 B) runs in the same k_gf_apply launch
    // as the full chunks, as a workgroup over the shard's last chunk-sized window whose lanes
    // store only the partial chunk (apply.hpp); otherwise the byte-safe kernel takes it in a
    // launch of its own.
    const int64_t tail_len = nbytes - full * chunk;
    const bool fuse_tail = aligned && full >= 1 && tail_len > 0 && tail_len % 16 == 0 && (depth == 4 || depth == 8) &&
                           cm.n_tiles() == 1 && rows == kTileRows && ntmode == 2 && nts == 1 && tu.lds_tables != 2 &&
                           !waves && !wide && !bits && !lut && outputs_never_read(cm.map(), in, in_stripe_stride, in_slot_stride, out,
                                                      out_stripe_stride, out_slot_stride, nstripes, nbytes);
    if (fuse_tail) {
        a.tail_chunk = full;
        a.tail_bytes = (int)tail_len;
        // (a launch of the partial chunk alone is not the launch's kernel of record)
        const std::string noted = first == full ? last_kernel() : std::string();
        tail_launch = true;
        run(false, first, full + 1 - first);
        tail_launch = false;
        if (first == full) set_last_kernel(noted);
    } else {
        run(false, first, full - first);
        run(true, full, tail_chunks);
    }
    if (kernel_notes() != notes0 && !planes)  // a composed-map kernel of record was launched here
        set_last_shape_order("stagger=" + std::to_string(a.stagger) + " xcd_group=" + std::to_string(a.xcd_group) +
                             " xcd_run=" + std::to_string(a.xcd_group == 3 ? a.xcd_run : 0) +
                             (skew ? " skew=" + std::to_string(skew) : std::string()));
    check_hip(hipGetLastError(), "k_gf_apply launch");
}
}  // namespace

// Launch shape per batch layout, measured on the caller's own launches.  The many-stream
// single-tile maps (RS decode / encode: >= 8 input streams, <= 4 rows) move 0.63-0.79 of
// HBM depending only on where their streams sit: same-offset streams whose addresses differ
// in the bits the HBM interleave does not spread (a 4 MiB shard pitch, or 1 MiB + 4 KiB,
// whose stripes collide) queue on one bank (scripts/addr_probe.hip), and
// no static rule predicts which shape -- 4 KiB or one-wave workgroups, skewed chunks,
// staggered stripes -- is fastest at a given pitch (scripts/layout_sweep.py).  So for a
// new layout (map, strides, size classes of the shard and the batch, device) the first calls run the
// candidates in turn, each launch bracketed by two events on the caller's stream; the
// events are read without blocking on later calls, and once every candidate has
// kLayoutSamples timings the fastest median is kept for that layout.  Every candidate
// computes the same bytes, and nothing is launched that the caller did not ask for: the
// exploration costs only the slower candidates' launches.  Batches under kLayoutMinBytes of
// input, streams being captured and forced shapes use the static rules.
constexpr int64_t kLayoutMinBytes = (int64_t)256 << 20;
constexpr int kLayoutSamples = 5;  // median of 5: 3 left a 2-5 % spread between fresh maps (scripts/select_check.py)
// candidate 0 = the static rules, then shape + 8 * stagger (launch_apply_core's pick)
constexpr int kLayoutCand[] = {-1, 0, 1, 2, 2 + 8 * 2, 2 + 8 * 8, 0 + 8 * 4};
constexpr int kLayoutNCand = (int)(sizeof(kLayoutCand) / sizeof(kLayoutCand[0]));

int layout_candidate_code(int cand) { return cand >= 0 && cand < kLayoutNCand ? kLayoutCand[cand] : -2; }

void launch_apply(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride, uint8_t *out,
                  int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes, int64_t nbytes,
                  hipStream_t stream, bool accumulate) {
    const Tuning &tu = tuning();
    const LinearMap &m = cm.map();
    const bool aligned = aligned16(in) && aligned16(out) && (in_stripe_stride % 16 == 0) &&
                         (in_slot_stride % 16 == 0) && (out_stripe_stride % 16 == 0) && (out_slot_stride % 16 == 0);
    const int64_t in_bytes = (int64_t)m.n_in * nbytes;  // per stripe
    bool select = tu.layout_select && tu.skew_chunks == 1 && tu.block_threads == 0 && tu.stagger == 0 &&
                  !tu.lds_lut && tu.bitslice != 2 && tu.nontemporal == 1 && tu.store_scope == 0 &&
                  cm.n_tiles() == 1 && m.n_in >= 8 && cm.max_tile_rows() <= 4 && aligned && in_slot_stride > 0 &&
                  nbytes >= 4 * kChunkBytes && nstripes * in_bytes >= kLayoutMinBytes;
    if (select) {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(stream, &cap) != hipSuccess) {
            (void)hipGetLastError();
            cap = hipStreamCaptureStatusActive;  // unknown: no events
        }
        select = cap == hipStreamCaptureStatusNone;
    }
    int dev = 0;
    check_hip(hipGetDevice(&dev), "hipGetDevice");
    if (!select) {
        launch_apply_core(cm, in, in_stripe_stride, in_slot_stride, out, out_stripe_stride, out_slot_stride, nstripes,
                          nbytes, stream, accumulate, -1);
        note_device_launch(dev, stream, nstripes * in_bytes);
        return;
    }
    // A layout is its strides, the size class of the shard (log2 of the byte count) and of the
    // batch (log2 of its input bytes), the mode and the device: callers whose batch sizes vary
    // from call to call share one selection instead of exploring anew at every size.
    auto log2i = [](int64_t v) { return (int64_t)(63 - __builtin_clzll((unsigned long long)std::max<int64_t>(v, 1))); };
    const std::array<int64_t, 8> key{in_slot_stride, in_stripe_stride, out_slot_stride, out_stripe_stride,
                                     log2i(nbytes), log2i(nstripes * in_bytes), (int64_t)accumulate, (int64_t)dev};
    uint64_t ticket = 0;
    const int cand = cm.next_layout_pick(key, kLayoutNCand, kLayoutSamples, dev, stream, &ticket);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (ticket) {
        if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
            (void)hipGetLastError();
            if (e0) (void)hipEventDestroy(e0);
            if (e1) (void)hipEventDestroy(e1);
            e0 = e1 = nullptr;
            cm.cancel_layout_probe(key, ticket);
            ticket = 0;
        }
    }
    try {
        launch_apply_core(cm, in, in_stripe_stride, in_slot_stride, out, out_stripe_stride, out_slot_stride, nstripes,
                          nbytes, stream, accumulate, kLayoutCand[cand], ticket ? e0 : nullptr);
    } catch (...) {
        if (ticket) {
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
            cm.cancel_layout_probe(key, ticket);
        }
        throw;
    }
    note_device_launch(dev, stream, nstripes * in_bytes);
    if (ticket) {
        if (hipEventRecord(e1, stream) == hipSuccess) {
            cm.fill_layout_probe(key, ticket, e0, e1);
        } else {
            (void)hipGetLastError();
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
            cm.cancel_layout_probe(key, ticket);
        }
    }
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
