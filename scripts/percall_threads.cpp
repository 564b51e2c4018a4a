// percall_threads.cpp -- per-call host entry points called from several threads at once,
// as the reference's node processes do (one Redis handler thread per node object,
// ClayCodeNode.kt:38-40): RS(4,2) encodeParity and Clay(4,2) performCoding repair on
// 32 KiB buffers, every thread with its own buffers, for 1..16 threads, with one shared
// context per device (ecx_tune host_contexts 0: calls serialised) and with a context
// leased per call (1: calls on separate streams).  Rounds interleave the two modes.
// One JSON line per (case, threads, mode): aggregate calls per second.
//
//   hipcc -O2 -std=c++17 -I include scripts/percall_threads.cpp -L repair-pipelining_amd -lecx \
//         -Wl,-rpath,'$ORIGIN/../repair-pipelining_amd' -o scripts/percall_threads
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <random>
#include <thread>
#include <vector>

#include "ecx.h"
#include "ecx_tune.h"

struct Buffers {
    std::vector<std::vector<uint8_t>> shards, cin, cout;
    std::vector<uint8_t *> sp, op;
    std::vector<const uint8_t *> ip;
};

int main() {
    const int L = 32768, erased = 1, calls = 300, rounds = 3;
    ecx_rs *rs = nullptr;
    ecx_clay *clay = nullptr;
    if (ecx_rs_create(4, 2, &rs) || ecx_clay_create(4, 2, &erased, 1, &clay)) return 1;
    std::mt19937 rng(11);
    const int max_threads = 16;
    std::vector<Buffers> b(max_threads);
    for (auto &x : b) {
        x.shards.assign(6, std::vector<uint8_t>(L));
        x.cin.assign(48, std::vector<uint8_t>(L));
        x.cout.assign(8, std::vector<uint8_t>(L));
        for (auto &v : x.shards) for (auto &c : v) c = (uint8_t)rng();
        for (auto &v : x.cin) for (auto &c : v) c = (uint8_t)rng();
        for (auto &v : x.shards) x.sp.push_back(v.data());
        for (int i = 0; i < 48; ++i) x.ip.push_back(i % 6 == erased ? nullptr : x.cin[i].data());
        for (auto &v : x.cout) x.op.push_back(v.data());
    }
    const char *names[2] = {"RS(4,2) encodeParity, 32 KiB shards", "Clay(4,2) performCoding repair e=1, B=32 KiB"};
    auto one = [&](int which, Buffers &x) {
        return which == 0 ? ecx_rs_encode_parity(rs, x.sp.data(), 6, L, 0, L)
                          : ecx_clay_perform_coding(clay, x.ip.data(), x.op.data(), L);
    };
    for (int which = 0; which < 2; ++which) {
        for (int T : {1, 2, 4, 8, 16}) {
            std::vector<double> best(2, 0.0);
            for (int r = 0; r < rounds; ++r) {
                for (int mode = 0; mode < 2; ++mode) {
                    ecx_tune("host_contexts", mode);
                    for (int t = 0; t < T; ++t)
                        if (one(which, b[t])) return 2;  // warm (contexts, plans, staging)
                    std::atomic<int> bad{0};
                    const auto t0 = std::chrono::steady_clock::now();
                    std::vector<std::thread> th;
                    for (int t = 0; t < T; ++t)
                        th.emplace_back([&, t] {
                            for (int i = 0; i < calls; ++i)
                                if (one(which, b[t])) bad++;
                        });
                    for (auto &x : th) x.join();
                    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    if (bad) return 3;
                    best[mode] = std::max(best[mode], T * calls / s);
                }
            }
            for (int mode = 0; mode < 2; ++mode)
                printf("{\"case\": \"%s\", \"threads\": %d, \"host_contexts\": %d, \"calls_per_s\": %.0f, "
                       "\"us_per_call_per_thread\": %.1f}\n",
                       names[which], T, mode, best[mode], 1e6 * T / best[mode]);
            fflush(stdout);
        }
    }
    ecx_tune("host_contexts", 1);
    ecx_clay_destroy(clay);
    ecx_rs_destroy(rs);
    return 0;
}
