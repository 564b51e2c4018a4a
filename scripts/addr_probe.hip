// addr_probe.hip -- which address bits make concurrent HBM streams collide, and which
// workgroup order spreads the many-stream RS patterns over the memory system.
//
// Part "bits": K streams read together (one 256-thread workgroup per 4 KiB unit, one
// 16-B NT load per lane per stream, no writes).  Stream i of unit u reads
//   insert(u * 4 KiB, bit b, log2 K) | (i << b)
// i.e. the K addresses of a workgroup differ only in bits b .. b+log2K-1, and the
// streams together cover one contiguous region.  A bit the HBM interleave hashes on
// sends the K streams to different channels/banks; a bit it ignores stacks them on
// the same bank in different rows.  K = 2 (pairs) and K = 8, b = 12 .. 30.
//
// Part "sched": the RS(12,4) decode (12 shards read, 2 written in place) and RS(17,3)
// encode (17 read, 3 written in place) data movement -- XOR folds, NT loads and
// stores, every load of a lane in flight -- at several shard pitches, with the
// workgroup -> (stripe, 4 KiB chunk) order taken from a table:
//   identity     stripe-major, chunks inner (what launch_apply does today);
//   chunkmajor   chunk c of every stripe, then c + 1;
//   stagger G    G stripes interleaved, stripe j of the group starting at chunk j*C/G;
//   random       a seeded permutation of the units;
//   xcdrun R     runs of R consecutive units per XCD (xcd_group 3).
// Interleaved rounds, median launch, algorithmic GB/s and fraction of 8 TB/s.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/addr_probe.hip -o scripts/addr_probe
//   ./scripts/addr_probe bits | pitch | rot | sched
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const gu32x4 *)p); }
__device__ __forceinline__ void stnt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (gu32x4 *)p); }

// ---- part "bits" ---------------------------------------------------------------
template <int K>
__global__ void __launch_bounds__(256) k_bits(const uint8_t *pool, uint32_t *sink, int b) {
    constexpr int LK = K == 2 ? 1 : (K == 4 ? 2 : 3);
    const uint64_t a = (uint64_t)blockIdx.x * 4096u;
    const uint64_t low = a & ((1ull << b) - 1), high = a >> b;
    const uint64_t base = (high << (b + LK)) | low;
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = ldnt(pool + (base | ((uint64_t)i << b)) + threadIdx.x * 16);
    u32x4 acc = x[0];
#pragma unroll
    for (int i = 1; i < K; ++i) acc ^= x[i];
    if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u) sink[threadIdx.x] = acc.z;  // never taken
}

// ---- part "pitch" --------------------------------------------------------------
// K = 8 streams at pitch P (stripe s, stream i, chunk c at s*8P + i*P + c*4 KiB), read
// only, identity order: which pitches 2^a + 2^b make the same-time accesses of the
// streams collide (a bank/channel hash that XORs bit a with bit b cancels such a pitch).
__global__ void __launch_bounds__(256) k_pitch(const uint8_t *pool, uint32_t *sink, int64_t pitch, uint32_t chunks) {
    const uint64_t s = blockIdx.x / chunks, c = blockIdx.x % chunks;
    const uint8_t *base = pool + s * 8 * pitch + c * 4096 + threadIdx.x * 16;
    u32x4 x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = ldnt(base + i * pitch);
    u32x4 acc = x[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) acc ^= x[i];
    if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u) sink[threadIdx.x] = acc.z;  // never taken
}

static int run_pitch(uint8_t *pool, uint32_t *sink) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct R { int a, b; int64_t pitch; uint32_t stripes, chunks; std::vector<float> ms; };
    std::vector<R> rs;
    for (int b = 17; b <= 27; ++b) {
        rs.push_back({-1, b, 1ll << b, 0, 0, {}});
        for (int a = 12; a <= 16; ++a) rs.push_back({a, b, (1ll << b) + (1ll << a), 0, 0, {}});
    }
    for (auto &r : rs) {
        r.chunks = (uint32_t)(r.pitch / 4096);
        r.stripes = (uint32_t)((8ll << 30) / (8 * r.pitch));
    }
    for (int round = 0; round < 5; ++round)
        for (auto &r : rs) {
            auto launch = [&]() {
                hipLaunchKernelGGL(k_pitch, dim3(r.stripes * r.chunks), dim3(256), 0, 0, pool, sink, r.pitch, r.chunks);
            };
            launch();
            (void)hipEventRecord(e0);
            for (int rep = 0; rep < 3; ++rep) launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t = 0;
            (void)hipEventElapsedTime(&t, e0, e1);
            r.ms.push_back(t / 3);
        }
    if (hipGetLastError() != hipSuccess) { printf("{\"error\": \"launch\"}\n"); return 1; }
    for (auto &r : rs) {
        std::sort(r.ms.begin(), r.ms.end());
        const float med = r.ms[r.ms.size() / 2];
        const double bytes = (double)r.stripes * r.chunks * 4096.0 * 8;
        printf("{\"part\": \"pitch\", \"low_bit\": %d, \"high_bit\": %d, \"pitch\": %lld, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n",
               r.a, r.b, (long long)r.pitch, med, bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12);
    }
    fflush(stdout);
    return 0;
}

// ---- part "sched" --------------------------------------------------------------
struct Slots {
    int64_t in_slot[20], out_slot[4];
    int64_t stripe_bytes;
    int chunks;
};

template <int NI, int NO>
__global__ void __launch_bounds__(256) k_sched(uint8_t *pool, const uint32_t *order, Slots s) {
    const uint32_t unit = order[blockIdx.x];
    const int64_t stripe = unit / (uint32_t)s.chunks, chunk = unit % (uint32_t)s.chunks;
    uint8_t *base = pool + stripe * s.stripe_bytes + chunk * 4096 + threadIdx.x * 16;
    u32x4 x[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) x[i] = ldnt(base + s.in_slot[i]);
    u32x4 acc[NO];
#pragma unroll
    for (int r = 0; r < NO; ++r) acc[r] = (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[i % NO] ^= x[i];
#pragma unroll
    for (int r = 0; r < NO; ++r) stnt(base + s.out_slot[r], acc[r]);
}

static std::vector<uint32_t> make_order(const std::string &kind, int arg, uint32_t stripes, uint32_t C) {
    const uint32_t n = stripes * C;
    std::vector<uint32_t> o(n);
    if (kind == "identity") {
        for (uint32_t b = 0; b < n; ++b) o[b] = b;
    } else if (kind == "chunkmajor") {
        for (uint32_t b = 0; b < n; ++b) o[b] = (b % stripes) * C + b / stripes;
    } else if (kind == "stagger") {  // groups of G stripes, interleaved, stripe j starts at chunk j*C/G
        const uint32_t G = (uint32_t)arg;
        for (uint32_t b = 0; b < n; ++b) {
            const uint32_t grp = b / (G * C), j = b % G, k = (b % (G * C)) / G;
            const uint32_t s = grp * G + j;
            if (s >= stripes) { o[b] = b; continue; }  // a ragged last group keeps identity
            o[b] = s * C + (k + j * C / G) % C;
        }
        // ragged tail: make sure it is still a permutation
        const uint32_t full = (stripes / G) * G * C;
        for (uint32_t b = full; b < n; ++b) o[b] = b;
    } else if (kind == "random") {
        for (uint32_t b = 0; b < n; ++b) o[b] = b;
        std::mt19937 g(12345);
        std::shuffle(o.begin(), o.end(), g);
    } else if (kind == "xcdrun") {  // runs of R consecutive units per XCD
        const uint32_t R = (uint32_t)arg, full = (n / (8 * R)) * (8 * R);
        for (uint32_t b = 0; b < n; ++b) {
            if (b >= full) { o[b] = b; continue; }
            const uint32_t xcd = b % 8, j = b / 8;
            o[b] = ((j / R) * 8 + xcd) * R + (j % R);
        }
    }
    return o;
}

// ---- part "rot" ----------------------------------------------------------------
// The RS(12,4) decode / RS(17,3) encode data movement with K consecutive 4 KiB chunks
// per workgroup and the chunk each stream is read at rotated: in phase t stream i reads
// chunk (i + t) mod K, so the same-time accesses of the streams sit at min(K, streams)
// different offsets (K = 1: every stream at one offset, the collision of power-of-two
// pitches).  Every load of a phase in flight, XOR folds, the K x NO output chunks stored
// at the end.  Identity unit order.
template <int NI, int NO, int K>
__global__ void __launch_bounds__(256) k_rot(uint8_t *pool, Slots s) {
    const int64_t groups = s.chunks / K;
    const int64_t stripe = blockIdx.x / groups, g = blockIdx.x % groups;
    uint8_t *base = pool + stripe * s.stripe_bytes + g * (K * 4096) + threadIdx.x * 16;
    u32x4 acc[K][NO];
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int r = 0; r < NO; ++r) acc[k][r] = (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
    for (int t = 0; t < K; ++t) {
        u32x4 x[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) x[i] = ldnt(base + s.in_slot[i] + ((i + t) % K) * 4096);
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[(i + t) % K][i % NO] ^= x[i];
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int r = 0; r < NO; ++r) stnt(base + s.out_slot[r] + k * 4096, acc[k][r]);
}

// The same with one-wave workgroups over 1 KiB chunks (the one-wave kernels' shape): K
// consecutive 1 KiB chunks per workgroup, stream i read at chunk (i + t) mod K in phase t.
template <int NI, int NO, int K>
__global__ void __launch_bounds__(64) k_rot_wave(uint8_t *pool, Slots s) {
    const int64_t groups = s.chunks * 4 / K;  // 1 KiB chunks
    const int64_t stripe = blockIdx.x / groups, g = blockIdx.x % groups;
    uint8_t *base = pool + stripe * s.stripe_bytes + g * (K * 1024) + threadIdx.x * 16;
    u32x4 acc[K][NO];
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int r = 0; r < NO; ++r) acc[k][r] = (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
    for (int t = 0; t < K; ++t) {
        u32x4 x[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) x[i] = ldnt(base + s.in_slot[i] + ((i + t) % K) * 1024);
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[(i + t) % K][i % NO] ^= x[i];
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int r = 0; r < NO; ++r) stnt(base + s.out_slot[r] + k * 1024, acc[k][r]);
}

static int run_rot(uint8_t *pool, int64_t pool_bytes) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct R { const char *name; int ni, no, k; int64_t pitch; Slots s; uint32_t stripes; std::vector<float> ms; bool wave = false; };
    std::vector<R> rs;
    auto add = [&](const char *name, int ni, int no, int64_t pitch, std::vector<int> ks) {
        for (int k : ks) {
            R r{name, ni, no, k, pitch, {}, 0, {}};
            memset(&r.s, 0, sizeof r.s);
            const int nsh = ni == 12 ? 16 : 20;
            for (int i = 0; i < ni; ++i) r.s.in_slot[i] = (ni == 12 ? 2 + i : i) * pitch;
            for (int o = 0; o < no; ++o) r.s.out_slot[o] = (ni == 12 ? o : 17 + o) * pitch;
            r.s.stripe_bytes = nsh * pitch;
            r.s.chunks = (int)(pitch / 4096) / k * k;  // whole chunk groups
            r.stripes = (uint32_t)std::min<int64_t>(pool_bytes / r.s.stripe_bytes, (16ll << 30) / r.s.stripe_bytes);
            rs.push_back(r);
        }
    };
    for (int64_t p : {4ll << 20, (4ll << 20) + 4096, 1ll << 20, (1ll << 20) + 4096, 8ll << 20})
        add("rs124", 12, 2, p, {1, 2, 4, 8, 12, 16});
    const size_t n256 = rs.size();
    for (int64_t p : {4ll << 20, (4ll << 20) + 4096, (1ll << 20) + 4096})
        add("rs124_wave", 12, 2, p, {1, 2, 4, 8, 12, 16});
    for (size_t i = n256; i < rs.size(); ++i) {
        rs[i].wave = true;
        rs[i].s.chunks = (int)(rs[i].pitch / 1024) / rs[i].k * rs[i].k / 4;  // in 4 KiB units (1 KiB chunks / 4)
    }
    add("rs173", 17, 3, 200000, {1, 2, 4, 8});
    add("rs173", 17, 3, 262144, {1, 2, 4, 8});
    for (int round = 0; round < 5; ++round)
        for (auto &r : rs) {
            const dim3 grid(r.wave ? r.stripes * (uint32_t)(r.s.chunks * 4 / r.k) : r.stripes * (uint32_t)(r.s.chunks / r.k));
            auto launch = [&]() {
                if (r.wave) {
#define ROTW(K) \
    if (r.k == K) hipLaunchKernelGGL((k_rot_wave<12, 2, K>), grid, dim3(64), 0, 0, pool, r.s);
                    ROTW(1) ROTW(2) ROTW(4) ROTW(8) ROTW(12) ROTW(16)
#undef ROTW
                    return;
                }
#define ROT(NI, NO, K) \
    if (r.ni == NI && r.k == K) hipLaunchKernelGGL((k_rot<NI, NO, K>), grid, dim3(256), 0, 0, pool, r.s);
                ROT(12, 2, 1) ROT(12, 2, 2) ROT(12, 2, 4) ROT(12, 2, 8) ROT(12, 2, 12) ROT(12, 2, 16)
                ROT(17, 3, 1) ROT(17, 3, 2) ROT(17, 3, 4) ROT(17, 3, 8)
#undef ROT
            };
            launch();
            (void)hipEventRecord(e0);
            for (int rep = 0; rep < 3; ++rep) launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t = 0;
            (void)hipEventElapsedTime(&t, e0, e1);
            r.ms.push_back(t / 3);
        }
    if (hipGetLastError() != hipSuccess) { printf("{\"error\": \"launch\"}\n"); return 1; }
    for (auto &r : rs) {
        std::sort(r.ms.begin(), r.ms.end());
        const float med = r.ms[r.ms.size() / 2];
        const double bytes = (double)r.stripes * r.s.chunks * 4096.0 * (r.ni + r.no);
        printf("{\"part\": \"rot\", \"case\": \"%s\", \"pitch\": %lld, \"K\": %d, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n",
               r.name, (long long)r.pitch, r.k, med, bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12);
    }
    fflush(stdout);
    return 0;
}

struct SchedCase {
    std::string name;
    int ni, no;
    int64_t pitch;
    Slots s;
    uint32_t stripes;
};

static int run_bits(uint8_t *pool, uint32_t *sink) {
    const uint32_t units = (uint32_t)((1ull << 30) / 4096);  // 1 GiB per stream
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct R { int k, b; std::vector<float> ms; };
    std::vector<R> rs;
    for (int k : {2, 8})
        for (int b = 12; b <= 30; ++b) rs.push_back({k, b, {}});
    for (int round = 0; round < 5; ++round)
        for (auto &r : rs) {
            auto launch = [&]() {
                if (r.k == 2) hipLaunchKernelGGL(k_bits<2>, dim3(units), dim3(256), 0, 0, pool, sink, r.b);
                else hipLaunchKernelGGL(k_bits<8>, dim3(units), dim3(256), 0, 0, pool, sink, r.b);
            };
            launch();
            (void)hipEventRecord(e0);
            for (int rep = 0; rep < 3; ++rep) launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t = 0;
            (void)hipEventElapsedTime(&t, e0, e1);
            r.ms.push_back(t / 3);
        }
    if (hipGetLastError() != hipSuccess) { printf("{\"error\": \"launch\"}\n"); return 1; }
    for (auto &r : rs) {
        std::sort(r.ms.begin(), r.ms.end());
        const float med = r.ms[r.ms.size() / 2];
        const double bytes = (double)units * 4096.0 * r.k;
        printf("{\"part\": \"bits\", \"streams\": %d, \"bit\": %d, \"offset_bytes\": %llu, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n",
               r.k, r.b, 1ull << r.b, med, bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12);
        fflush(stdout);
    }
    return 0;
}

static int run_sched(uint8_t *pool, int64_t pool_bytes, int rounds) {
    std::vector<SchedCase> cases;
    auto rs124 = [&](int64_t pitch) {
        SchedCase c;
        c.ni = 12; c.no = 2; c.pitch = pitch;
        memset(&c.s, 0, sizeof c.s);
        for (int i = 0; i < 12; ++i) c.s.in_slot[i] = (2 + i) * pitch;  // data 0,1 erased: shards 2..13 read
        c.s.out_slot[0] = 0; c.s.out_slot[1] = pitch;
        c.s.stripe_bytes = 16 * pitch;
        c.s.chunks = (int)(pitch / 4096);
        c.stripes = (uint32_t)std::min<int64_t>(pool_bytes / c.s.stripe_bytes, (int64_t)(16ll << 30) / c.s.stripe_bytes);
        c.name = "rs124";
        cases.push_back(c);
    };
    auto rs173 = [&](int64_t pitch) {
        SchedCase c;
        c.ni = 17; c.no = 3; c.pitch = pitch;
        memset(&c.s, 0, sizeof c.s);
        for (int i = 0; i < 17; ++i) c.s.in_slot[i] = i * pitch;
        for (int r = 0; r < 3; ++r) c.s.out_slot[r] = (17 + r) * pitch;
        c.s.stripe_bytes = 20 * pitch;
        c.s.chunks = (int)(pitch / 4096);
        c.stripes = (uint32_t)std::min<int64_t>(pool_bytes / c.s.stripe_bytes, (int64_t)(16ll << 30) / c.s.stripe_bytes);
        c.name = "rs173";
        cases.push_back(c);
    };
    for (int64_t p : {1ll << 22, (1ll << 22) + 4096, 1ll << 20, (1ll << 20) + 4096, 3ll << 20, 1ll << 23}) rs124(p);
    for (int64_t p : {200000ll, 262144ll}) rs173(p);

    struct Sched { std::string kind; int arg; };
    std::vector<Sched> scheds = {{"identity", 0}, {"chunkmajor", 0}, {"stagger", 2}, {"stagger", 4}, {"stagger", 8},
                                 {"stagger", 16}, {"random", 0}, {"xcdrun", 32}};
    uint32_t *d_order = nullptr;
    uint32_t max_units = 0;
    for (auto &c : cases) max_units = std::max(max_units, c.stripes * (uint32_t)c.s.chunks);
    if (hipMalloc(&d_order, (size_t)max_units * 4) != hipSuccess) { printf("{\"error\": \"hipMalloc order\"}\n"); return 1; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (auto &c : cases) {
        const uint32_t C = (uint32_t)c.s.chunks, n = c.stripes * C;
        std::vector<std::vector<float>> ms(scheds.size());
        std::vector<std::vector<uint32_t>> orders;
        for (auto &sc : scheds) orders.push_back(make_order(sc.kind, sc.arg, c.stripes, C));
        for (int round = 0; round < rounds; ++round)
            for (size_t i = 0; i < scheds.size(); ++i) {
                (void)hipMemcpy(d_order, orders[i].data(), (size_t)n * 4, hipMemcpyHostToDevice);
                auto launch = [&]() {
                    if (c.ni == 12) hipLaunchKernelGGL((k_sched<12, 2>), dim3(n), dim3(256), 0, 0, pool, d_order, c.s);
                    else hipLaunchKernelGGL((k_sched<17, 3>), dim3(n), dim3(256), 0, 0, pool, d_order, c.s);
                };
                launch();
                (void)hipEventRecord(e0);
                for (int rep = 0; rep < 3; ++rep) launch();
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float t = 0;
                (void)hipEventElapsedTime(&t, e0, e1);
                ms[i].push_back(t / 3);
            }
        if (hipGetLastError() != hipSuccess) { printf("{\"error\": \"launch\"}\n"); return 1; }
        for (size_t i = 0; i < scheds.size(); ++i) {
            std::sort(ms[i].begin(), ms[i].end());
            const float med = ms[i][ms[i].size() / 2];
            const double bytes = (double)n * 4096.0 * (c.ni + c.no);
            printf("{\"part\": \"sched\", \"case\": \"%s\", \"pitch\": %lld, \"stripes\": %u, \"order\": \"%s\", \"arg\": %d, "
                   "\"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n",
                   c.name.c_str(), (long long)c.pitch, c.stripes, scheds[i].kind.c_str(), scheds[i].arg, med,
                   bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12);
        }
        fflush(stdout);
    }
    return 0;
}

int main(int argc, char **argv) {
    const std::string part = argc > 1 ? argv[1] : "bits";
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int64_t pool_bytes = 17ll << 30;
    uint8_t *pool = nullptr;
    uint32_t *sink = nullptr;
    if (hipMalloc(&pool, pool_bytes) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) {
        printf("{\"error\": \"hipMalloc\"}\n");
        return 1;
    }
    (void)hipMemset(pool, 0x3C, pool_bytes);
    (void)hipDeviceSynchronize();
    if (part == "bits") return run_bits(pool, sink);
    if (part == "pitch") return run_pitch(pool, sink);
    if (part == "rot") return run_rot(pool, pool_bytes);
    return run_sched(pool, pool_bytes, rounds);
}
