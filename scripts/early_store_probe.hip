// early_store_probe.hip -- would the headline gain from storing output rows as soon as they are
// complete instead of all eight at the end of the workgroup?
// The Clay(4,2) e = 1 repair map pairs its rows: rows {0,4} read inputs {0,1,2,3,4,8,11}, {1,5}
// add {5,6,7,9,16}, {2,6} add {10,12,13,14,18}, {3,7} add {15,17,19}.  Taking the entries in that
// order, rows 0 and 4 are final after 7 entries, 1 and 5 after 12, 2 and 6 after 17, 3 and 7 after
// 20, so their stores can leave while later entries are still loading (ring depth 8) or being
// multiplied (depth 20).  The probe runs the headline's data movement ([S][20][32 KiB] helper
// sub-chunks read, [S][8][32 KiB] written, NT loads and stores, one 256-thread workgroup per
// (stripe, 4 KiB chunk)) with one split-table-shaped multiply (3 v_perm_b32 + 2 v_bitop3_b32,
// pinned with inline asm) per map coefficient and dword, stores at the end or as early as
// possible, ring depth 8 or 20.  Interleaved rounds, median launch, algorithmic GB/s.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/early_store_probe.hip -o scripts/early_store_probe && ./scripts/early_store_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <utility>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const gu32x4 *)p); }
__device__ __forceinline__ void stnt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (gu32x4 *)p); }

__device__ __forceinline__ uint32_t mul_acc(uint32_t x, uint32_t lo, uint32_t hi, uint32_t acc) {
    uint32_t a, b, c;
    asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(a) : "s"(lo), "v"(hi), "v"(x));
    asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(b) : "v"(hi), "s"(lo), "v"(x));
    asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(c) : "s"(lo), "v"(hi), "v"(a));
    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(a) : "v"(a), "v"(b), "v"(c));
    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(acc) : "v"(acc), "v"(a), "v"(x));
    return acc;
}

constexpr int64_t kB = 32768;
// the rows each input feeds, as a row bit mask
constexpr uint8_t rows_of(int in) {
    // rows {0,4}: 0,1,2,3,4,8,11 (row 4 without input 0); {1,5}: 4..9,16 (row 5 without 5);
    // {2,6}: 2,10..14,18 (row 6 without 10); {3,7}: 7,14..19 (row 7 without 15)
    uint8_t m = 0;
    if (in == 0 || in == 1 || in == 2 || in == 3 || in == 4 || in == 8 || in == 11) m |= 1;
    if (in == 1 || in == 2 || in == 3 || in == 4 || in == 8 || in == 11) m |= 16;
    if ((in >= 4 && in <= 9) || in == 16) m |= 2;
    if (in == 4 || (in >= 6 && in <= 9) || in == 16) m |= 32;
    if (in == 2 || (in >= 10 && in <= 14) || in == 18) m |= 4;
    if (in == 2 || (in >= 11 && in <= 14) || in == 18) m |= 64;
    if (in == 7 || (in >= 14 && in <= 19)) m |= 8;
    if (in == 7 || in == 14 || (in >= 16 && in <= 19)) m |= 128;
    return m;
}
// entry order (input slots)
constexpr int kOrderH[20] = {0, 1, 2, 3, 4, 8, 11, 5, 6, 7, 9, 16, 10, 12, 13, 14, 18, 15, 17, 19};
// rows final after entry e (of the order above): {0,4} after 6, {1,5} after 11, {2,6} after 16, {3,7} after 19
constexpr uint8_t done_after(int e) { return e == 6 ? 0x11 : e == 11 ? 0x22 : e == 16 ? 0x44 : e == 19 ? 0x88 : 0; }

// entry E of the ring: consume ring[E % D], refill it with entry E + D, multiply into the rows the
// input feeds, store the rows it completes (EARLY); every index a compile-time constant
template <int D, bool EARLY, int E>
__device__ __forceinline__ void entry(const uint8_t *in, uint8_t *o, u32x4 (&ring)[D], u32x4 (&acc)[8], uint32_t lo,
                                      uint32_t hi) {
    const u32x4 x = ring[E % D];
    if constexpr (E + D < 20) ring[E % D] = ldnt(in + (int64_t)kOrderH[E + D] * kB);
    constexpr uint8_t m = rows_of(kOrderH[E]);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        if (m & (1u << r)) {
#pragma unroll
            for (int d = 0; d < 4; ++d) acc[r][d] = mul_acc(x[d], lo + (uint32_t)(r * 20 + E), hi, acc[r][d]);
        }
    }
    if constexpr (EARLY) {
        constexpr uint8_t f = done_after(E);
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (f & (1u << r)) stnt(o + (int64_t)r * kB, acc[r]);
    }
}

template <int D, bool EARLY, int... E>
__device__ __forceinline__ void entries(const uint8_t *in, uint8_t *o, u32x4 (&ring)[D], u32x4 (&acc)[8], uint32_t lo,
                                        uint32_t hi, std::integer_sequence<int, E...>) {
    (entry<D, EARLY, E>(in, o, ring, acc, lo, hi), ...);
}

template <int D, bool EARLY>
__global__ void __launch_bounds__(256) k_early(const uint8_t *pool, uint8_t *out, int nchunks, uint32_t lo, uint32_t hs) {
    const uint32_t hi = hs + (threadIdx.x >> 10);
    const int64_t stripe = blockIdx.x / nchunks, chunk = blockIdx.x % nchunks;
    const uint8_t *in = pool + stripe * (20 * kB) + chunk * 4096 + threadIdx.x * 16;
    uint8_t *o = out + stripe * (8 * kB) + chunk * 4096 + threadIdx.x * 16;
    u32x4 acc[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = (u32x4){0u, 0u, 0u, 0u};
    u32x4 ring[D];
#pragma unroll
    for (int u = 0; u < D; ++u) ring[u] = ldnt(in + (int64_t)kOrderH[u] * kB);
    entries<D, EARLY>(in, o, ring, acc, lo, hi, std::make_integer_sequence<int, 20>{});
    if constexpr (!EARLY) {
#pragma unroll
        for (int r = 0; r < 8; ++r) stnt(o + (int64_t)r * kB, acc[r]);
    }
}

template <int D, bool EARLY>
float run(const uint8_t *a, uint8_t *b, int64_t stripes) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int nchunks = (int)(kB / 4096);
    std::vector<float> ms;
    for (int rep = 0; rep < 7; ++rep) {
        float t = 0;
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k_early<D, EARLY>), dim3((unsigned)(stripes * nchunks)), dim3(256), 0, 0, a, b, nchunks,
                           0x03020100u, 0x07060504u);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&t, e0, e1);
        if (rep) ms.push_back(t);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
}

int main() {
    const int64_t stripes = 1 << 15;  // the headline's resident pool: 20 GiB read, 8 GiB written per launch
    uint8_t *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, stripes * 20 * kB) != hipSuccess || hipMalloc(&b, stripes * 8 * kB) != hipSuccess) return 1;
    (void)hipMemset(a, 1, stripes * 20 * kB);
    (void)hipMemset(b, 2, stripes * 8 * kB);
    (void)hipDeviceSynchronize();
    const double bytes = (double)stripes * 28 * kB;
    for (int round = 0; round < 3; ++round) {
        const float t[4] = {run<20, false>(a, b, stripes), run<20, true>(a, b, stripes), run<8, false>(a, b, stripes),
                            run<8, true>(a, b, stripes)};
        const char *name[4] = {"depth20_end", "depth20_early", "depth8_end", "depth8_early"};
        for (int i = 0; i < 4; ++i)
            printf("{\"probe\": \"early_store\", \"round\": %d, \"case\": \"%s\", \"ms\": %.4f, \"frac\": %.4f}\n", round,
                   name[i], t[i], bytes / (t[i] * 1e-3) / 8e12);
        fflush(stdout);
    }
    return 0;
}
