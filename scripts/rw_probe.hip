// rw_probe.hip -- what does a write stream cost inside a many-stream read pattern?
// RS(17,3)'s encode (17 shards read, 3 written per stripe) runs at 0.69-0.70 of HBM where the
// read-only check over the same 20 shards runs at 0.81-0.83.  This bare
// probe (NT loads, XOR folds, NT stores, one 256-thread workgroup per (stripe, 4 KiB chunk),
// every load of a lane issued at once, stripe-major order) varies one thing at a time:
//   * reads : writes per stripe at a fixed number of streams (20:0, 17:3, 14:6, 10:10),
//   * the same 17:3 with fewer streams (17:0, 8:2 ...), the shard pitch (200,000 B, 200,064 B
//     = 128-B aligned, 256 KiB, 32 KiB), and writes in place or to a separate dense buffer.
// Full 4 KiB chunks only (the partial last chunk of a 200,000-B shard is left out of both the
// launch and the bytes).  Interleaved rounds, median launch, algorithmic GB/s over ~16 GB.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/rw_probe.hip -o scripts/rw_probe && ./scripts/rw_probe [pitch | rs124]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const gu32x4 *)p); }
__device__ __forceinline__ void stnt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (gu32x4 *)p); }

struct Layout {
    int64_t pitch;         // bytes between a stripe's shards
    int64_t stripe_bytes;  // bytes between stripes (input side)
    int64_t out_stripe;    // bytes between stripes of the output side
    int64_t out_pitch;     // bytes between a stripe's output rows
    int64_t out_first;     // offset of output row 0 inside its stripe
    int chunks;            // full 4 KiB chunks per shard
};

template <int R, int W>
__global__ void __launch_bounds__(256) k_rw(const uint8_t *pool, uint8_t *out, Layout l) {
    const int64_t stripe = blockIdx.x / l.chunks, chunk = blockIdx.x % l.chunks;
    const uint8_t *in = pool + stripe * l.stripe_bytes + chunk * 4096 + threadIdx.x * 16;
    u32x4 x[R];
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = ldnt(in + (int64_t)i * l.pitch);
    if constexpr (W == 0) {
        u32x4 s = x[0];
#pragma unroll
        for (int i = 1; i < R; ++i) s |= x[i];
        // a read-only pass must not be optimised away: one lane in 2^32 "stores"
        if (s.x == 0x9E3779B9u && s.y == 0x7F4A7C15u) *(gu32x4 *)(out + threadIdx.x * 16) = s;
    } else {
        uint8_t *o = out + stripe * l.out_stripe + l.out_first + chunk * 4096 + threadIdx.x * 16;
#pragma unroll
        for (int r = 0; r < W; ++r) {
            u32x4 acc = x[r % R];
#pragma unroll
            for (int i = 0; i < R; ++i)
                if (i != r % R) acc ^= (x[i] << (uint32_t)(r + 1)) | (x[i] >> (uint32_t)(31 - r));
            stnt(o + (int64_t)r * l.out_pitch, acc);
        }
    }
}

struct Case {
    const char *name;
    int r, w;
    int64_t pitch;
    bool in_place;
};

template <int R, int W>
float launch(const uint8_t *pool, uint8_t *out, const Layout &l, int64_t stripes) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const unsigned blocks = (unsigned)(stripes * l.chunks);
    std::vector<float> ms;
    for (int rep = 0; rep < 6; ++rep) {
        float t = 0;
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_rw<R, W>), dim3(blocks), dim3(256), 0, 0, pool, out, l);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&t, e0, e1);
        if (rep) ms.push_back(t);
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
}

float dispatch(int r, int w, const uint8_t *pool, uint8_t *out, const Layout &l, int64_t stripes) {
#define RW(R_, W_) \
    if (r == R_ && w == W_) return launch<R_, W_>(pool, out, l, stripes);
    RW(20, 0) RW(17, 3) RW(17, 0) RW(14, 6) RW(10, 10) RW(8, 2) RW(12, 2) RW(20, 8) RW(12, 4) RW(3, 17) RW(12, 0)
#undef RW
    return -1.f;
}

int main(int argc, char **argv) {
    // "pitch": 17:3 in place over a sweep of shard pitches (and a few separate-output points)
    const bool pitch_sweep = argc > 1 && std::string(argv[1]) == "pitch";
    // "rs124": RS(12,4)'s 2-erasure decode pattern (12 read, 2 written in place) over shard pitches
    const bool rs124 = argc > 1 && std::string(argv[1]) == "rs124";
    const Case rs124_cases[] = {
        {"12r2w_4m", 12, 2, 4194304, true},      {"12r2w_4m4k", 12, 2, 4194304 + 4096, true},
        {"12r2w_4m64k", 12, 2, 4194304 + 65536, true}, {"12r2w_2m", 12, 2, 2097152, true},
        {"12r2w_1m", 12, 2, 1048576, true},      {"12r2w_256k", 12, 2, 262144, true},
        {"12r0w_4m", 12, 0, 4194304, true},      {"12r2w_4m_sep", 12, 2, 4194304, false},
    };
    const Case sweep[] = {
        {"17r3w_32k", 17, 3, 32768, true},    {"17r3w_64k", 17, 3, 65536, true},    {"17r3w_128k", 17, 3, 131072, true},
        {"17r3w_192k", 17, 3, 196608, true},  {"17r3w_200000", 17, 3, 200000, true}, {"17r3w_256k", 17, 3, 262144, true},
        {"17r3w_512k", 17, 3, 524288, true},  {"17r3w_1m", 17, 3, 1048576, true},   {"17r3w_4m", 17, 3, 4194304, true},
        {"17r3w_68k", 17, 3, 69632, true},    {"17r3w_100k", 17, 3, 102400, true},
        {"17r3w_sep_32k", 17, 3, 32768, false}, {"17r3w_sep_1m", 17, 3, 1048576, false},
    };
    const Case base[] = {
        {"20r0w", 20, 0, 200000, true},     {"17r3w", 17, 3, 200000, true},   {"17r0w", 17, 0, 200000, true},
        {"14r6w", 14, 6, 200000, true},     {"10r10w", 10, 10, 200000, true}, {"3r17w", 3, 17, 200000, true},
        {"8r2w", 8, 2, 200000, true},       {"12r2w", 12, 2, 200000, true},   {"12r4w", 12, 4, 200000, true},
        {"17r3w_sep", 17, 3, 200000, false}, {"17r3w_a128", 17, 3, 200064, true},
        {"20r0w_256k", 20, 0, 262144, true}, {"17r3w_256k", 17, 3, 262144, true},
        {"20r0w_32k", 20, 0, 32768, true},  {"17r3w_32k", 17, 3, 32768, true}, {"20r8w_32k_sep", 20, 8, 32768, false},
    };
    const int64_t budget = (int64_t)16384 << 20;  // bytes of input-side stripes per launch (~16 GiB)
    uint8_t *pool = nullptr, *sep = nullptr;
    const int64_t pool_bytes = budget + ((int64_t)64 << 20), sep_bytes = (int64_t)8 << 30;
    if (hipMalloc(&pool, pool_bytes) != hipSuccess || hipMalloc(&sep, sep_bytes) != hipSuccess) return 1;
    hipMemset(pool, 0x5A, pool_bytes);
    hipMemset(sep, 0, sep_bytes);
    hipDeviceSynchronize();
    const Case *cases = rs124 ? rs124_cases : pitch_sweep ? sweep : base;
    const size_t ncases = rs124 ? sizeof(rs124_cases) / sizeof(rs124_cases[0])
                          : pitch_sweep ? sizeof(sweep) / sizeof(sweep[0]) : sizeof(base) / sizeof(base[0]);
    for (int round = 0; round < 2; ++round) {
        for (size_t ci = 0; ci < ncases; ++ci) {
            const Case &c = cases[ci];
            const int streams = c.in_place ? c.r + c.w : c.r;
            Layout l{};
            l.pitch = c.pitch;
            l.stripe_bytes = (int64_t)streams * c.pitch;
            l.chunks = (int)(c.pitch / 4096);
            const int64_t stripes = budget / l.stripe_bytes;
            if (c.in_place) {
                l.out_stripe = l.stripe_bytes;
                l.out_pitch = c.pitch;
                l.out_first = (int64_t)c.r * c.pitch;
            } else {  // dense separate output: [stripe][w][pitch]
                l.out_stripe = (int64_t)c.w * c.pitch;
                l.out_pitch = c.pitch;
                l.out_first = 0;
                if (stripes * l.out_stripe > sep_bytes) return 2;
            }
            const float ms = dispatch(c.r, c.w, pool, c.in_place ? pool : sep, l, stripes);
            if (ms < 0) return 3;
            const double bytes = (double)stripes * (c.r + c.w) * l.chunks * 4096.0;
            printf("{\"probe\": \"rw\", \"round\": %d, \"case\": \"%s\", \"reads\": %d, \"writes\": %d, \"pitch\": %lld, "
                   "\"in_place\": %s, \"stripes\": %lld, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n",
                   round, c.name, c.r, c.w, (long long)c.pitch, c.in_place ? "true" : "false", (long long)stripes, ms,
                   bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 8e12);
            fflush(stdout);
        }
    }
    hipFree(pool);
    hipFree(sep);
    return 0;
}
