// percall_sizes.cpp -- per-call RS(12,4) encodeParity / decodeMissing {0,1} on host
// shards of 64 KiB .. 8 MiB, through the gather path (used slots memcpy'd into pinned
// staging, one kernel reading it over PCIe: ecx_tune host_gather_kib >= the shard) and
// through the per-slot path (one runtime H2D copy per shard from pageable memory, the
// kernel, one D2H copy per output).  Prints one JSON line per (case, size, path): median
// microseconds per call and algorithmic GB/s ((12 + outputs) x L per call).
//
//   hipcc -O2 -std=c++17 -I include scripts/percall_sizes.cpp -L repair-pipelining_amd -lecx \
//         -Wl,-rpath,'$ORIGIN/../repair-pipelining_amd' -o scripts/percall_sizes
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <random>
#include <vector>

#include "ecx.h"
#include "ecx_tune.h"

static double median_us(const std::function<int()> &call, int reps) {
    if (call() != 0) return -1.0;
    std::vector<double> t;
    for (int i = 0; i < reps; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        if (call() != 0) return -1.0;
        t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    std::mt19937 rng(5);
    ecx_rs *rs = nullptr;
    if (ecx_rs_create(12, 4, &rs)) return 1;
    for (int L : {64 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20}) {
        std::vector<std::vector<uint8_t>> sh(16, std::vector<uint8_t>(L));
        for (auto &s : sh)
            for (auto &c : s) c = (uint8_t)rng();
        std::vector<uint8_t *> p(16);
        for (int i = 0; i < 16; ++i) p[i] = sh[i].data();
        uint8_t present[16];
        for (int i = 0; i < 16; ++i) present[i] = i >= 2;
        const int reps = L >= (2 << 20) ? 15 : 40;
        for (int gather : {0, 1}) {
            ecx_tune("host_gather_kib", gather ? (L >> 10) : (L >> 10) - 1);
            const double enc = median_us([&] { return ecx_rs_encode_parity(rs, p.data(), 16, L, 0, L); }, reps);
            const double dec = median_us([&] { return ecx_rs_decode_missing(rs, p.data(), present, 16, L, 0, L); }, reps);
            printf("{\"case\": \"RS(12,4) encodeParity\", \"shard_bytes\": %d, \"path\": \"%s\", \"us_per_call\": %.1f, "
                   "\"GBps\": %.2f}\n", L, gather ? "gather" : "per-slot", enc, 16.0 * L / enc / 1e3);
            printf("{\"case\": \"RS(12,4) decodeMissing {0,1}\", \"shard_bytes\": %d, \"path\": \"%s\", \"us_per_call\": %.1f, "
                   "\"GBps\": %.2f}\n", L, gather ? "gather" : "per-slot", dec, 14.0 * L / dec / 1e3);
            fflush(stdout);
        }
    }
    ecx_tune("host_gather_kib", 512);
    ecx_rs_destroy(rs);
    return 0;
}
