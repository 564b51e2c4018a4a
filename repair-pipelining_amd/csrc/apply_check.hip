// apply_check.hip -- k_gf_check: ReedSolomon.isParityCorrect (ReedSolomon.java:129-178) over
// device-resident stripes, the "Check" half of ReedSolomonBenchmark (:73-87, :126-149).
//
// The check map of a code (ecx_api.cpp rs_check_map) has one row per parity shard p:
// syndrome_p = sum_i parityRows[p][i] * D_i  ^  P_p, which is all zero exactly when P_p is the
// parity of the data.  The kernel runs that map with k_gf_apply's plan, load ring and split-table
// arithmetic (apply.hpp) but never stores a syndrome: each lane OR-folds its rows in registers,
// each wave ballots the result, and a wave that saw a non-zero byte clears its stripe's verdict
// byte (launch_check sets every verdict to 1 first).  Nothing is written to the shards, so the
// read stream is the kernel's whole traffic: (k + m) * byte_count per stripe.
//
// A shard's partial last chunk (200,000-B shards: 48 full 4 KiB chunks and 3,392 B) runs in
// the same launch: its workgroup reads the shard's last 4 KiB window instead, so the bytes
// it shares with the previous chunk are checked twice -- harmless for a read-only check, and
// it keeps every load a full 16-B access (byte counts that are multiples of 16 on aligned
// layouts; otherwise a byte-safe launch covers the remainder).
#include "apply.hpp"

namespace ecx {

template <bool SAFE, int DEPTH, int ROWS>
__global__ void __launch_bounds__(kBlockThreads, ROWS < kTileRows ? (DEPTH >= 16 ? 4 : 5) : (DEPTH >= 16 ? 3 : 5)) k_gf_check(ApplyArgs a) {
    const uint32_t w = logical_block(a.xcd_group, (uint32_t)a.n_tiles, (uint32_t)a.xcd_run);
    const uint32_t tl = w % (uint32_t)a.n_tiles;
    const uint32_t rest = w / (uint32_t)a.n_tiles;
    const uint32_t nst = gridDim.x / ((uint32_t)a.n_tiles * (uint32_t)a.n_chunks);
    int64_t s, c;
    unit_of(rest, (uint32_t)a.n_chunks, nst, 0, (uint32_t)a.stagger, s, c);
    s += a.stripe_begin;
    c += a.chunk_begin;
    int64_t cbase = c * kChunkBytes;
    if (!SAFE && c == a.tail_chunk) cbase = a.nbytes - kChunkBytes;  // the shard's last full window
    const uint32_t lane16 = threadIdx.x * 16;
    int valid = 16;
    if (SAFE) {
        const int64_t v = a.nbytes - cbase - (int64_t)lane16;
        valid = v <= 0 ? 0 : (v >= 16 ? 16 : (int)v);
    }
    cu32 *tile = plan_ptr(a.tiles) + __builtin_amdgcn_readfirstlane(tl) * kTileDwords;
    const uint8_t *ib =
        reinterpret_cast<const uint8_t *>(uniform64((uint64_t)(a.in + s * a.in_stripe_stride + cbase))) + lane16;
    auto load = [&](uint32_t slot) -> u32x4 {  // padding entries read the zero page
        const uint8_t *p = slot == kDummySlot ? a.zero_page + lane16 : ib + (int64_t)slot * a.in_slot_stride;
        return SAFE ? load_partial(p, valid) : ld16<true>(p);
    };
    const int ecnt = (int)tile[1];  // padded to a multiple of DEPTH
    const int nrows = (int)tile[2];
    u32x4 acc[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r] = (u32x4){0u, 0u, 0u, 0u};
    cu32 *ent = plan_ptr(a.entries) + (int64_t)tile[0] * kEntryDwords;
    if (ecnt > 0) {
        u32x4 ring[DEPTH];
#pragma unroll
        for (int u = 0; u < DEPTH; ++u) ring[u] = load(ent[u * kEntryDwords]);
        const int last = ecnt - DEPTH;
        for (int e0 = 0; e0 < last; e0 += DEPTH) {
#pragma unroll
            for (int u = 0; u < DEPTH; ++u) {
                cu32 *r = ent + (int64_t)(e0 + u) * kEntryDwords;
                apply_entry<false, ROWS>(r, ring[u], acc, nullptr);
                ring[u] = load(r[DEPTH * kEntryDwords]);
            }
        }
#pragma unroll
        for (int u = 0; u < DEPTH; ++u)
            apply_entry<false, ROWS>(ent + (int64_t)(last + u) * kEntryDwords, ring[u], acc, nullptr);
    }
    uint32_t nz = 0;
#pragma unroll
    for (int o = 0; o < ROWS; ++o)
        if (o < nrows) nz |= acc[o].x | acc[o].y | acc[o].z | acc[o].w;
    // one vector byte store per wave that saw a mismatch (every writer stores the same 0)
    if (__builtin_amdgcn_ballot_w64(nz != 0) && (threadIdx.x & 63) == 0) {
        gu8 *v = (gu8 *)(a.out + s * a.out_stripe_stride);
        *v = 0;
    }
}

namespace {
template <bool SAFE, int D, int R>
void launch_check_k(dim3 grid, hipStream_t stream, const ApplyArgs &a) {
    if (!SAFE) note_kernel("k_gf_check", SAFE, D, R);
    hipLaunchKernelGGL((k_gf_check<SAFE, D, R>), grid, dim3(kBlockThreads), 0, stream, a);
}
}  // namespace

namespace {
// Clears verdict[s] when a syndrome byte of stripe s over bytes [0, nbytes) is non-zero (the
// verdicts were set to 1 by launch_check).
void launch_check_core(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                       uint8_t *verdict, int64_t nstripes, int64_t nbytes, hipStream_t stream) {
    // Ring depth 4 (forced 8 / 20 with ecx_tune "depth"): on RS(17,3) 200,000-B shards depth 4 reads
    // 0.83 of HBM, depth 8 and 20 0.80 -- the short ring leaves registers for more resident waves
    // (profiles/r05_check_sweep.jsonl).  Accumulator rows: 4 when every tile has at most 4 (RS with
    // m <= 4), else 8.
    const Tuning &tu = tuning();
    const int depth = tu.depth == 8 || tu.depth == 20 ? tu.depth : 4;
    const int rows = cm.max_tile_rows() <= 4 ? 4 : kTileRows;
    const bool aligned = aligned16(in) && in_stripe_stride % 16 == 0 && in_slot_stride % 16 == 0;
    const int64_t full = aligned ? nbytes / kChunkBytes : 0;
    const int64_t tail = nbytes - full * kChunkBytes;
    // the partial last chunk as a shifted full window (read-only: overlap is re-checked)
    const bool fuse_tail = aligned && full >= 1 && tail > 0 && tail % 16 == 0;
    const DevicePlan &plan = cm.plan_for_current_device(depth);
    const DevicePlan &plan4 = depth == 4 ? plan : cm.plan_for_current_device(4);

    ApplyArgs a{};
    a.in = in;
    a.out = verdict;
    a.zero_page = zero_page_for_current_device();
    a.in_stripe_stride = in_stripe_stride;
    a.in_slot_stride = in_slot_stride;
    a.out_stripe_stride = 1;
    a.out_slot_stride = 0;
    a.nbytes = nbytes;
    a.n_tiles = cm.n_tiles();
    a.stagger = tu.stagger;
    // inputs not 128-B aligned share a boundary line between neighbouring chunks: runs of
    // consecutive units per XCD keep both fetches in one L2 (as launch_apply_core does)
    const bool misaligned128 = ((uintptr_t)in % 128) != 0 || in_stripe_stride % 128 != 0 || in_slot_stride % 128 != 0;
    a.xcd_group = tu.xcd_group == 3 ? 3 : (tu.xcd_misaligned && misaligned128 ? 3 : 0);
    a.xcd_run = tu.xcd_run;
    a.tail_chunk = fuse_tail ? full : -1;
    auto run = [&](bool safe, const DevicePlan &p, int64_t chunk_begin, int64_t n_chunks) {
        if (n_chunks <= 0) return;
        a.entries = p.entries;
        a.tiles = p.tiles;
        a.chunk_begin = chunk_begin;
        a.n_chunks = n_chunks;
        const int64_t per_stripe = n_chunks * a.n_tiles;
        const int64_t stripes_per_launch = std::max<int64_t>(1, ((int64_t)1 << 30) / per_stripe);
        for (int64_t s0 = 0; s0 < nstripes; s0 += stripes_per_launch) {
            a.stripe_begin = s0;
            const dim3 grid((unsigned)(std::min(stripes_per_launch, nstripes - s0) * per_stripe));
            if (safe) {
                if (rows == 4) launch_check_k<true, 4, 4>(grid, stream, a);
                else launch_check_k<true, 4, kTileRows>(grid, stream, a);
            } else if (rows == 4) {
                if (depth == 20) launch_check_k<false, 20, 4>(grid, stream, a);
                else if (depth == 8) launch_check_k<false, 8, 4>(grid, stream, a);
                else launch_check_k<false, 4, 4>(grid, stream, a);
            } else {
                if (depth == 20) launch_check_k<false, 20, kTileRows>(grid, stream, a);
                else if (depth == 8) launch_check_k<false, 8, kTileRows>(grid, stream, a);
                else launch_check_k<false, 4, kTileRows>(grid, stream, a);
            }
        }
    };
    const uint64_t notes0 = kernel_notes();
    if (fuse_tail) {
        run(false, plan, 0, full + 1);
    } else {
        run(false, plan, 0, full);
        a.tail_chunk = -1;
        run(true, plan4, full, (tail + kChunkBytes - 1) / kChunkBytes);  // (not noted: byte-safe)
    }
    if (kernel_notes() != notes0)
        set_last_shape_order("stagger=" + std::to_string(a.stagger) + " xcd_group=" + std::to_string(a.xcd_group) +
                             " xcd_run=" + std::to_string(a.xcd_group == 3 ? a.xcd_run : 0));
    check_hip(hipGetLastError(), "k_gf_check launch");
}
}  // namespace

// verdict[s] = 1 when every parity shard of stripe s equals the parity of its
// data over bytes [0, nbytes) of each slot, else 0.  `cm` is a check map (rows = syndromes).
// A start that is not 16-B aligned (isParityCorrect's firstByte may be anything) on 16-B
// strides: the bytes up to the first 16-B boundary go to the byte-safe kernel, the rest to the
// vectorised one, so only the head (< 16 B per slot) pays the byte-safe rate.
void launch_check(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                  uint8_t *verdict, int64_t nstripes, int64_t nbytes, hipStream_t stream) {
    if (nstripes <= 0) return;
    check_hip(hipMemsetAsync(verdict, 1, (size_t)nstripes, stream), "hipMemsetAsync (verdicts)");
    if (nbytes <= 0 || cm.map().n_out == 0) return;
    const int64_t head = (int64_t)((16 - (uintptr_t)in % 16) % 16);
    if (head > 0 && head < nbytes && in_stripe_stride % 16 == 0 && in_slot_stride % 16 == 0) {
        launch_check_core(cm, in, in_stripe_stride, in_slot_stride, verdict, nstripes, head, stream);
        launch_check_core(cm, in + head, in_stripe_stride, in_slot_stride, verdict, nstripes, nbytes - head, stream);
    } else {
        launch_check_core(cm, in, in_stripe_stride, in_slot_stride, verdict, nstripes, nbytes, stream);
    }
    int dev = 0;
    check_hip(hipGetDevice(&dev), "hipGetDevice");
    note_device_launch(dev, stream, nstripes * nbytes * cm.map().n_in);
}

}  // namespace ecx
