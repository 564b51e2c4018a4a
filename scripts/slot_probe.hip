// slot_probe.hip -- does WHERE a workgroup's streams sit in the stripe move the HBM rate?
// The headline's data movement (20 sub-chunks read per stripe, 8 written to a separate
// buffer, one 256-thread workgroup per (stripe, 4 KiB chunk), every load of a lane in
// flight, NT loads and stores, XOR only) with the 20 read slots chosen three ways, and the
// RS(17,3) encode's (17 shards read, 3 written in place) at two shard pitches.
// Interleaved rounds, median launch, algorithmic GB/s.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/slot_probe.hip -o scripts/slot_probe && ./scripts/slot_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

struct Slots {
    int n_in, n_out;
    int64_t in_slot[20], out_slot[8];  // byte offsets of the slots inside a stripe
    int64_t stripe_bytes, out_stripe_bytes;
    int chunks;                          // 4 KiB chunks per slot
};

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const gu32x4 *)p); }
__device__ __forceinline__ void stnt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (gu32x4 *)p); }

template <int NI, int NO>
__global__ void __launch_bounds__(256) k_slots(const uint8_t *pool, uint8_t *out, Slots s) {
    const int64_t stripe = blockIdx.x / s.chunks, chunk = blockIdx.x % s.chunks;
    const uint8_t *in = pool + stripe * s.stripe_bytes + chunk * 4096 + threadIdx.x * 16;
    uint8_t *o = out + stripe * s.out_stripe_bytes + chunk * 4096 + threadIdx.x * 16;
    u32x4 x[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) x[i] = ldnt(in + s.in_slot[i]);
    u32x4 acc[NO];
#pragma unroll
    for (int r = 0; r < NO; ++r) acc[r] = (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[i % NO] ^= x[i];
#pragma unroll
    for (int r = 0; r < NO; ++r) stnt(o + s.out_slot[r], acc[r]);
}

struct Case {
    const char *name;
    Slots s;
    int64_t stripes;
    bool inplace;
};

int main() {
    const int64_t B = 32768, P173 = 200000, P256 = 262144;
    std::vector<Case> cases;
    auto clay = [&](const char *name, std::vector<int> slots) {
        Case c{name, {}, 1 << 15, false};
        c.s.n_in = 20;
        c.s.n_out = 8;
        for (int i = 0; i < 20; ++i) c.s.in_slot[i] = slots[i] * B;
        for (int r = 0; r < 8; ++r) c.s.out_slot[r] = r * B;
        c.s.stripe_bytes = 48 * B;
        c.s.out_stripe_bytes = 8 * B;
        c.s.chunks = 8;
        cases.push_back(c);
    };
    std::vector<int> contiguous, helper_e1, spread;
    for (int i = 0; i < 20; ++i) contiguous.push_back(i);
    for (int z = 4; z < 8; ++z)  // Clay(4,2), erased node 1: helper planes 4..7, nodes != 1
        for (int nd = 0; nd < 6; ++nd)
            if (nd != 1) helper_e1.push_back(z * 6 + nd);
    for (int i = 0; i < 20; ++i) spread.push_back((i * 12) % 48 + (i * 12) / 48);  // every 12th slot, wrapped
    clay("clay42 slots 0-19", contiguous);
    clay("clay42 helper slots of node 1 (the bench)", helper_e1);
    clay("clay42 slots spread over the stripe", spread);
    auto rs = [&](const char *name, int64_t pitch, bool inplace) {
        Case c{name, {}, (int64_t)(16.0 * (1 << 30) / (20 * pitch)), inplace};
        c.s.n_in = 17;
        c.s.n_out = 3;
        for (int i = 0; i < 17; ++i) c.s.in_slot[i] = i * pitch;
        for (int r = 0; r < 3; ++r) c.s.out_slot[r] = inplace ? (17 + r) * pitch : r * pitch;
        c.s.stripe_bytes = 20 * pitch;
        c.s.out_stripe_bytes = inplace ? 20 * pitch : 3 * pitch;
        c.s.chunks = (int)(pitch / 4096);  // whole chunks only (the 200,000-B tail is left out)
        cases.push_back(c);
    };
    rs("rs173 200,000-B shards in place", P173, true);
    rs("rs173 200,000-B shards, separate outputs", P173, false);
    rs("rs173 256 KiB shards in place", P256, true);
    rs("rs173 256 KiB shards, separate outputs", P256, false);
    // LRC(12 data, 4 XOR local parities), 64 KiB blocks [d d d p] x 4: the encode reads the twelve
    // data blocks and writes the four parities in place; the block-2 repair reads blocks 0, 1, 3
    // of its group and writes one block to a separate buffer
    const int64_t P64 = 65536;
    {
        Case c{"lrc encode 64 KiB blocks in place", {}, 1 << 15, true};
        c.s.n_in = 12;
        c.s.n_out = 4;
        for (int i = 0; i < 12; ++i) c.s.in_slot[i] = (int64_t)((i / 3) * 4 + i % 3) * P64;
        for (int r = 0; r < 4; ++r) c.s.out_slot[r] = (int64_t)(r * 4 + 3) * P64;
        c.s.stripe_bytes = c.s.out_stripe_bytes = 16 * P64;
        c.s.chunks = 16;
        cases.push_back(c);
    }
    {
        Case c{"lrc repair of block 2, 64 KiB blocks", {}, 1 << 15, false};
        c.s.n_in = 3;
        c.s.n_out = 1;
        const int slots[3] = {0, 1, 3};
        for (int i = 0; i < 3; ++i) c.s.in_slot[i] = slots[i] * P64;
        c.s.out_slot[0] = 0;
        c.s.stripe_bytes = 16 * P64;
        c.s.out_stripe_bytes = P64;
        c.s.chunks = 16;
        cases.push_back(c);
    }

    int64_t pool_bytes = 0, out_bytes = 0;
    for (auto &c : cases) {
        pool_bytes = std::max(pool_bytes, c.stripes * c.s.stripe_bytes);
        out_bytes = std::max(out_bytes, c.stripes * c.s.out_stripe_bytes);
    }
    uint8_t *pool = nullptr, *out = nullptr;
    if (hipMalloc(&pool, pool_bytes) != hipSuccess || hipMalloc(&out, out_bytes) != hipSuccess) {
        printf("{\"error\": \"hipMalloc\"}\n");
        return 1;
    }
    (void)hipMemset(pool, 0x3C, pool_bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<std::vector<float>> ms(cases.size());
    auto launch = [&](const Case &c) {
        const dim3 grid((unsigned)(c.stripes * c.s.chunks));
        uint8_t *dst = c.inplace ? pool : out;
        if (c.s.n_in == 20) hipLaunchKernelGGL((k_slots<20, 8>), grid, dim3(256), 0, 0, pool, dst, c.s);
        else if (c.s.n_in == 12) hipLaunchKernelGGL((k_slots<12, 4>), grid, dim3(256), 0, 0, pool, dst, c.s);
        else if (c.s.n_in == 3) hipLaunchKernelGGL((k_slots<3, 1>), grid, dim3(256), 0, 0, pool, dst, c.s);
        else hipLaunchKernelGGL((k_slots<17, 3>), grid, dim3(256), 0, 0, pool, dst, c.s);
    };
    for (int round = 0; round < 5; ++round)
        for (size_t i = 0; i < cases.size(); ++i) {
            launch(cases[i]);
            (void)hipEventRecord(e0);
            for (int rep = 0; rep < 4; ++rep) launch(cases[i]);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t = 0;
            (void)hipEventElapsedTime(&t, e0, e1);
            ms[i].push_back(t / 4);
        }
    if (hipGetLastError() != hipSuccess) {
        printf("{\"error\": \"launch\"}\n");
        return 1;
    }
    for (size_t i = 0; i < cases.size(); ++i) {
        std::sort(ms[i].begin(), ms[i].end());
        const float med = ms[i][ms[i].size() / 2];
        const Case &c = cases[i];
        const double bytes = (double)c.stripes * c.s.chunks * 4096.0 * (c.s.n_in + c.s.n_out);
        printf("{\"case\": \"%s\", \"stripes\": %lld, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n", c.name,
               (long long)c.stripes, med, bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12);
    }
    return 0;
}
