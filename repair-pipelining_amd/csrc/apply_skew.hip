// apply_skew.hip -- k_gf_apply_skew: single-tile maps over K consecutive 4 KiB chunks
// per workgroup, with the chunk each input is read at rotated per entry.
//
// With one chunk per workgroup, the DEPTH loads a lane has in flight are DEPTH input
// slots at the same byte offset.  When the slot pitch is a large power of two
// (RS(12,4) shards of exactly 4 MiB, each its own stream) those addresses differ
// only above bit 22 and fall on one HBM bank in different rows, and the streams
// collide (0.63 of HBM against 0.77 with a 4 KiB pad).  Here a
// workgroup owns chunks c..c+K-1 of its stripe and walks its K x n entry sequence as
// K phases: in phase t entry e reads chunk (e + t) mod K, so consecutive loads in
// the ring alternate between K byte offsets.  THREADS = 64 (one wave, diagnostic build
// only): each 4 KiB chunk is split into four 1 KiB columns, one per workgroup, so a
// workgroup's K loads of a slot still sit 4 KiB apart (the spacing that separates
// colliding streams, profiles/r04_addr_pitch.jsonl) with the one-wave shape's footprint.  Entry e accumulates into the
// accumulators of chunk (e + t) mod K; with the entry count and DEPTH multiples of
// K that is physical accumulator set e mod K once the sets are rotated by one at
// every phase change (K rotations restore the identity before the stores).
#include "apply.hpp"

namespace ecx {

template <bool NTL, int DEPTH, int ROWS, int K, int THREADS>
__global__ void __launch_bounds__(THREADS, ROWS * K <= 8 ? 5 : 4) k_gf_apply_skew(ApplyArgs a) {
    static_assert(DEPTH % K == 0, "the ring must hold whole rotations");
    constexpr uint32_t kSub = kChunkBytes / (THREADS * 16);  // workgroups per 4 KiB chunk
    static_assert(kSub * THREADS * 16 == kChunkBytes, "a chunk is whole workgroup columns");
    const uint32_t col = blockIdx.x % kSub;
    int64_t s, g;  // stripe, chunk group
    unit_of(blockIdx.x / kSub, (uint32_t)a.n_chunks, gridDim.x / kSub / (uint32_t)a.n_chunks, 0, (uint32_t)a.stagger, s,
            g);
    s += a.stripe_begin;
    g += a.chunk_begin;
    const int64_t cbase = g * (int64_t)(K * kChunkBytes) + col * (THREADS * 16);
    const uint32_t lane16 = threadIdx.x * 16;
    cu32 *tile = plan_ptr(a.tiles);
    const uint8_t *ib = reinterpret_cast<const uint8_t *>(uniform64((uint64_t)(a.in + s * a.in_stripe_stride + cbase))) +
                        lane16;
    auto load = [&](uint32_t slot, int chunk) -> u32x4 {
        const uint8_t *p = slot == kDummySlot ? a.zero_page + lane16
                                              : ib + (int64_t)slot * a.in_slot_stride + chunk * kChunkBytes;
        return ld16<NTL>(p);
    };
    u32x4 acc[K][ROWS];
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc[k][r] = (u32x4){0u, 0u, 0u, 0u};
    auto rotate = [&]() {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const u32x4 t0 = acc[0][r];
#pragma unroll
            for (int k = 0; k + 1 < K; ++k) acc[k][r] = acc[k + 1][r];
            acc[K - 1][r] = t0;
        }
    };
    const int ecnt = (int)tile[1];  // padded to a multiple of DEPTH
    cu32 *ent = plan_ptr(a.entries) + (int64_t)tile[0] * kEntryDwords;
    if (ecnt > 0) {
        u32x4 ring[DEPTH];
#pragma unroll
        for (int u = 0; u < DEPTH; ++u) ring[u] = load(ent[u * kEntryDwords], u % K);
        int e0 = 0, t = 0;
        const int groups = K * (ecnt / DEPTH);
        for (int i = 0; i + 1 < groups; ++i) {
            int e1 = e0 + DEPTH, t1 = t;
            if (e1 == ecnt) {
                e1 = 0;
                t1 = t + 1;
            }
#pragma unroll
            for (int u = 0; u < DEPTH; ++u) {
                apply_entry<false, ROWS>(ent + (int64_t)(e0 + u) * kEntryDwords, ring[u], acc[u % K], nullptr);
                ring[u] = load(ent[(e1 + u) * kEntryDwords], (u + t1) & (K - 1));
            }
            if (t1 != t) rotate();
            e0 = e1;
            t = t1;
        }
#pragma unroll
        for (int u = 0; u < DEPTH; ++u)
            apply_entry<false, ROWS>(ent + (int64_t)(e0 + u) * kEntryDwords, ring[u], acc[u % K], nullptr);
        rotate();  // after phase K-1: set k holds chunk (k + K - 1) mod K; one more turn -> chunk k
    }
    const int nrows = (int)tile[2];
    uint8_t *ob = reinterpret_cast<uint8_t *>(uniform64((uint64_t)(a.out + s * a.out_stripe_stride + cbase))) + lane16;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int o = 0; o < ROWS; ++o) {
            if (o < nrows) {
                uint8_t *p = ob + k * kChunkBytes + (int64_t)tile[4 + o] * a.out_slot_stride;
                u32x4 v = acc[k][o];
                if (a.accumulate) v ^= load16(p);
                st16<1>(p, v);
            }
        }
}

void launch_skew(int k, int rows, int depth, bool ntl, int threads, dim3 grid, hipStream_t stream,
                 const ApplyArgs &a) {
#define ECX_SKEW(NTL, D, R, KK, T)                                                              \
    if (ntl == NTL && depth == D && rows == R && k == KK && threads == T) {                     \
        note_kernel("k_gf_apply_skew", NTL, D, R, KK, T);                                       \
        hipLaunchKernelGGL((k_gf_apply_skew<NTL, D, R, KK, T>), grid, dim3(T), 0, stream, a);   \
        return;                                                                                 \
    }
    ECX_SKEW(true, 4, 2, 2, 256) ECX_SKEW(true, 8, 2, 2, 256) ECX_SKEW(true, 4, 2, 4, 256) ECX_SKEW(true, 8, 2, 4, 256)
    ECX_SKEW(true, 4, 4, 2, 256) ECX_SKEW(true, 8, 4, 2, 256) ECX_SKEW(true, 4, 4, 4, 256) ECX_SKEW(true, 8, 4, 4, 256)
    ECX_SKEW(true, 4, 8, 2, 256)  // 8 rows x 2 chunks: depth 4 only (depth 8 spills)
#if ECX_DIAG
    // one-wave columns: measured and kept off -- 0.67-0.73 of HBM on the colliding RS pitches,
    // below the selected shapes, and 7-11 % below the one-chunk kernel elsewhere
    // (profiles/r04_layout_skewcheck.jsonl)
    ECX_SKEW(true, 4, 2, 2, 64) ECX_SKEW(true, 8, 2, 2, 64) ECX_SKEW(true, 4, 2, 4, 64) ECX_SKEW(true, 8, 2, 4, 64)
    ECX_SKEW(true, 4, 4, 2, 64) ECX_SKEW(true, 8, 4, 2, 64) ECX_SKEW(true, 4, 4, 4, 64) ECX_SKEW(true, 8, 4, 4, 64)
#endif
#undef ECX_SKEW
    throw Error(ECX_E_ILLEGAL_ARGUMENT, "no k_gf_apply_skew instance for this shape");
}

}  // namespace ecx
