// percall_threshold.cpp -- TEST-SIDE measurement of the per-call CPU/GPU crossover (SURVEY.md 8(b)
// group 1; ecx_tune "host_exec_kib"), run on the GPU box by tests/test_percall.py.  For each
// drop-in site's call shape and byte count it times, on one thread, the median microseconds per
// call of (a) libecx on the device (host_exec_kib 0), (b) libecx's host executor (host_exec_kib
// large), (c) libecx's default, and (d) the oracle (the restated reference loop, liborc.so: the
// baseline the drop-in is compared with), and checks that all outputs agree byte for byte.
// One JSON line per (case, bytes).  With `--threads T`: the same sites from T caller threads at
// once, sizes 2 KiB - 4 MiB (or up to an optional third argument; concurrent_main below).
//
//   case "rs31_single"  LRC chain word: RS(3,1) encodeParitySingle (NodeHelper.kt:89)
//   case "rs22_pair"    Clay pair transform: RS(2,2) decodeMissing, 2 of 4 present (ClayCodeNode.kt:125-132)
//   case "rs42_encode"  SampleEncoder: RS(4,2) encodeParity (SampleEncoder.java:83)
//   case "clay42"       Clay(4,2) performCoding, node 1 erased (ClayCodeHelper.kt:90, ClayCodeRunner)
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ecx.h"
#include "../../include/ecx_tune.h"
#include "../../oracle/ecx_oracle.h"

namespace {
std::mt19937 rng(7);

double median_us(const std::function<int()> &call, int reps) {
    for (int i = 0; i < 3; ++i)
        if (call() < 0) return -1.0;
    std::vector<double> t;
    for (int i = 0; i < reps; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        if (call() < 0) return -1.0;
        t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

struct Bufs {
    std::vector<std::vector<uint8_t>> v;
    std::vector<uint8_t *> p;
    Bufs(int n, int len) : v((size_t)n, std::vector<uint8_t>((size_t)len)), p((size_t)n) {
        for (int i = 0; i < n; ++i) {
            for (auto &c : v[(size_t)i]) c = (uint8_t)rng();
            p[(size_t)i] = v[(size_t)i].data();
        }
    }
};

void emit(const char *cas, int bytes, double dev, double hx, double def, double orc, bool same) {
    std::printf("{\"case\": \"%s\", \"bytes\": %d, \"device_us\": %.2f, \"host_exec_us\": %.2f, \"default_us\": %.2f, "
                "\"oracle_us\": %.2f, \"outputs_agree\": %s}\n",
                cas, bytes, dev, hx, def, orc, same ? "true" : "false");
    std::fflush(stdout);
}
}  // namespace

// ---- concurrent callers: the reference's drop-in sites run on one handler
// thread per node object (ClayCodeNode.kt:38-40, :125-132, :271-274), so the per-call threshold is
// measured with T caller threads at once, each on its own buffers: for each size, the aggregate
// calls per second with every call on the device (host_exec_kib 0: leased per-call contexts,
// separate streams) and on the host executor (host_exec_kib 1 GiB: the calling thread's core).
// One JSON line per (case, threads, bytes); "crossover" rows name the smallest size at which the
// device path's aggregate rate beats the host executor's.
struct Site {
    const char *name;
    int in_slots, out_slots;
    std::function<int(uint8_t *const *, uint8_t *const *, int)> call;  // (inputs, outputs, bytes)
};

double aggregate_calls_per_s(const Site &site, int threads, int bytes, double seconds,
                             std::vector<Bufs> &ins, std::vector<Bufs> &outs) {
    std::vector<std::thread> th;
    std::vector<long> done((size_t)threads, 0);
    std::atomic<int> ready{0}, bad{0};
    std::atomic<bool> go{false};
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<double> el((size_t)threads, 0.0);
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            if (site.call(ins[(size_t)t].p.data(), outs[(size_t)t].p.data(), bytes) < 0) bad.fetch_add(1);  // warm
            ready.fetch_add(1);
            while (!go.load()) std::this_thread::yield();
            const auto s0 = std::chrono::steady_clock::now();
            long n = 0;
            double e = 0.0;
            do {
                if (site.call(ins[(size_t)t].p.data(), outs[(size_t)t].p.data(), bytes) < 0) bad.fetch_add(1);
                ++n;
                e = std::chrono::duration<double>(std::chrono::steady_clock::now() - s0).count();
            } while (e < seconds);
            done[(size_t)t] = n;
            el[(size_t)t] = e;
        });
    while (ready.load() < threads) std::this_thread::yield();
    go.store(true);
    for (auto &x : th) x.join();
    (void)t0;
    if (bad.load()) return -1.0;
    double rate = 0.0;
    for (int t = 0; t < threads; ++t) rate += (double)done[(size_t)t] / el[(size_t)t];
    return rate;
}

int concurrent_main(int threads, int max_bytes) {
    int default_kib = 0;
    ecx_tune_value("host_exec_kib", &default_kib);
    const int erased = 1;
    ecx_rs *rs = nullptr;
    ecx_clay *clay = nullptr;
    if (ecx_rs_create(2, 2, &rs) || ecx_clay_create(4, 2, &erased, 1, &clay)) return 1;
    const uint8_t present[4] = {1, 0, 1, 0};
    std::vector<Site> sites = {
        // RS(2,2) decodeMissing of the pair transform: 2 shards read, 2 rebuilt in place
        {"rs22_pair", 4, 0,
         [&](uint8_t *const *in, uint8_t *const *, int L) { return ecx_rs_decode_missing(rs, in, present, 4, L, 0, L); }},
        // Clay(4,2) performCoding of node 1: 40 present sub-chunks in (20 used), 8 repaired out
        {"clay42", 48, 8,
         [&](uint8_t *const *in, uint8_t *const *out, int B) {
             const uint8_t *ip[48];
             for (int i = 0; i < 48; ++i) ip[i] = (i % 6) == erased ? nullptr : in[i];
             return ecx_clay_perform_coding(clay, ip, out, B);
         }},
    };
    const std::vector<int> sizes = {2048, 4096, 8192, 16384, 32768, 65536, 131072, 262144, 524288, 1 << 20,
                                    2 << 20, 4 << 20};
    for (const Site &site : sites) {
        int crossover = -1;
        for (int L : sizes) {
            if (L > max_bytes) break;
            std::vector<Bufs> ins, outs;
            for (int t = 0; t < threads; ++t) {
                ins.emplace_back(site.in_slots, L);
                outs.emplace_back(std::max(1, site.out_slots), L);
            }
            // the two paths give the same bytes (thread 0's buffers, one call each)
            Bufs a(site.in_slots, L), ao(std::max(1, site.out_slots), L);
            std::vector<std::vector<uint8_t>> b = a.v, bo = ao.v;
            std::vector<uint8_t *> pb((size_t)site.in_slots), pbo(bo.size());
            for (size_t i = 0; i < b.size(); ++i) pb[i] = b[i].data();
            for (size_t i = 0; i < bo.size(); ++i) pbo[i] = bo[i].data();
            ecx_tune("host_exec_kib", 0);
            const int s1 = site.call(a.p.data(), ao.p.data(), L);
            ecx_tune("host_exec_kib", 1 << 20);
            const int s2 = site.call(pb.data(), pbo.data(), L);
            const bool same = s1 >= 0 && s2 >= 0 && a.v == b && ao.v == bo;
            const double secs = 0.25;
            ecx_tune("host_exec_kib", 0);
            const double dev = aggregate_calls_per_s(site, threads, L, secs, ins, outs);
            ecx_tune("host_exec_kib", 1 << 20);
            const double host = aggregate_calls_per_s(site, threads, L, secs, ins, outs);
            ecx_tune("host_exec_kib", default_kib);
            if (crossover < 0 && dev > host) crossover = L;
            std::printf("{\"case\": \"%s\", \"threads\": %d, \"bytes\": %d, \"device_calls_per_s\": %.1f, "
                        "\"host_exec_calls_per_s\": %.1f, \"device_us_per_call\": %.2f, \"host_exec_us_per_call\": %.2f, "
                        "\"outputs_agree\": %s}\n",
                        site.name, threads, L, dev, host, dev > 0 ? threads * 1e6 / dev : -1.0,
                        host > 0 ? threads * 1e6 / host : -1.0, same ? "true" : "false");
            std::fflush(stdout);
        }
        std::printf("{\"case\": \"%s\", \"threads\": %d, \"crossover_bytes\": %d}\n", site.name, threads, crossover);
        std::fflush(stdout);
    }
    ecx_rs_destroy(rs);
    ecx_clay_destroy(clay);
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 3 && std::strcmp(argv[1], "--threads") == 0)
        return concurrent_main(std::atoi(argv[2]), argc >= 4 ? std::atoi(argv[3]) : (4 << 20));
    int default_kib = 0;
    ecx_tune_value("host_exec_kib", &default_kib);
    auto with_kib = [&](int kib, const std::function<int()> &f, int reps) {
        ecx_tune("host_exec_kib", kib);
        const double t = median_us(f, reps);
        ecx_tune("host_exec_kib", default_kib);
        return t;
    };
    const std::vector<int> sizes = {34, 256, 1024, 2174, 4096, 8192, 16384, 32768, 65536, 104449};
    // ---- RS(3,1) encodeParitySingle (accumulates: output ^= c * shard)
    {
        ecx_rs *rs = nullptr;
        orc_rs *orc = nullptr;
        if (ecx_rs_create(3, 1, &rs) || orc_rs_create(3, 1, &orc)) return 1;
        for (int L : sizes) {
            Bufs in(1, L), out(4, L);
            const int reps = L <= 4096 ? 400 : 100;
            auto call = [&](int which) {
                return [&, which] {
                    return ecx_rs_encode_parity_single(rs, in.p[0], out.p[(size_t)which], 1, 0, 0, L);
                };
            };
            const double dev = with_kib(0, call(0), reps);
            const double hx = with_kib(1 << 20, call(1), reps);
            const double def = median_us(call(2), reps);
            const double orct = median_us([&] { return orc_rs_encode_parity_single(orc, in.p[0], out.p[3], 1, 0, 0, L); },
                                          reps);
            // every path XOR-accumulated the same product an odd/even number of times: compare
            // one fresh application of each path
            std::vector<uint8_t> a((size_t)L, 0), b((size_t)L, 0), c((size_t)L, 0);
            ecx_tune("host_exec_kib", 0);
            ecx_rs_encode_parity_single(rs, in.p[0], a.data(), 1, 0, 0, L);
            ecx_tune("host_exec_kib", 1 << 20);
            ecx_rs_encode_parity_single(rs, in.p[0], b.data(), 1, 0, 0, L);
            ecx_tune("host_exec_kib", default_kib);
            orc_rs_encode_parity_single(orc, in.p[0], c.data(), 1, 0, 0, L);
            emit("rs31_single", L, dev, hx, def, orct, a == c && b == c);
        }
        ecx_rs_destroy(rs);
        orc_rs_free(orc);
    }
    // ---- RS(2,2) decodeMissing of the pair transform: shards 1 and 3 missing
    {
        ecx_rs *rs = nullptr;
        orc_rs *orc = nullptr;
        if (ecx_rs_create(2, 2, &rs) || orc_rs_create(2, 2, &orc)) return 1;
        const uint8_t present[4] = {1, 0, 1, 0};
        for (int L : sizes) {
            Bufs sh(4, L);
            const int reps = L <= 4096 ? 400 : 100;
            auto call = [&] { return ecx_rs_decode_missing(rs, sh.p.data(), present, 4, L, 0, L); };
            const double dev = with_kib(0, call, reps);
            const double hx = with_kib(1 << 20, call, reps);
            const double def = median_us(call, reps);
            const double orct = median_us([&] { return orc_rs_decode_missing(orc, sh.p.data(), present, 4, L, 0, L); }, reps);
            Bufs a(4, L);
            std::vector<std::vector<uint8_t>> b = a.v, c = a.v;
            std::vector<uint8_t *> pb(4), pc(4);
            for (int i = 0; i < 4; ++i) {
                pb[(size_t)i] = b[(size_t)i].data();
                pc[(size_t)i] = c[(size_t)i].data();
            }
            ecx_tune("host_exec_kib", 0);
            ecx_rs_decode_missing(rs, a.p.data(), present, 4, L, 0, L);
            ecx_tune("host_exec_kib", 1 << 20);
            ecx_rs_decode_missing(rs, pb.data(), present, 4, L, 0, L);
            ecx_tune("host_exec_kib", default_kib);
            orc_rs_decode_missing(orc, pc.data(), present, 4, L, 0, L);
            emit("rs22_pair", L, dev, hx, def, orct, a.v == c && b == c);
        }
        ecx_rs_destroy(rs);
        orc_rs_free(orc);
    }
    // ---- RS(4,2) encodeParity
    {
        ecx_rs *rs = nullptr;
        orc_rs *orc = nullptr;
        if (ecx_rs_create(4, 2, &rs) || orc_rs_create(4, 2, &orc)) return 1;
        for (int L : {2174, 8192, 32768, 104449}) {
            Bufs sh(6, L);
            const int reps = L <= 8192 ? 300 : 60;
            auto call = [&] { return ecx_rs_encode_parity(rs, sh.p.data(), 6, L, 0, L); };
            const double dev = with_kib(0, call, reps);
            const double hx = with_kib(1 << 20, call, reps);
            const double def = median_us(call, reps);
            Bufs o(6, L);
            for (int i = 0; i < 4; ++i) o.v[(size_t)i] = sh.v[(size_t)i];
            const double orct = median_us([&] { return orc_rs_encode_parity(orc, o.p.data(), 6, L, 0, L); }, reps);
            emit("rs42_encode", L, dev, hx, def, orct, sh.v == o.v);
        }
        ecx_rs_destroy(rs);
        orc_rs_free(orc);
    }
    // ---- Clay(4,2) performCoding, node 1 erased
    {
        const int e[1] = {1};
        ecx_clay *clay = nullptr;
        orc_clay *orc = nullptr;
        if (ecx_clay_create(4, 2, e, 1, &clay) || orc_clay_create(4, 2, e, 1, &orc)) return 1;
        for (int B : {512, 2174, 8192, 32768}) {
            Bufs in(48, B), out(8, B), ref(8, B);
            std::vector<const uint8_t *> ip(48);
            std::vector<uint8_t *> iq(48);
            for (int i = 0; i < 48; ++i) {
                ip[(size_t)i] = (i % 6) == 1 ? nullptr : in.p[(size_t)i];
                iq[(size_t)i] = (i % 6) == 1 ? nullptr : in.p[(size_t)i];
            }
            const int reps = B <= 8192 ? 200 : 60;
            auto call = [&] { return ecx_clay_perform_coding(clay, ip.data(), out.p.data(), B); };
            const double dev = with_kib(0, call, reps);
            const double hx = with_kib(1 << 20, call, reps);
            const double def = median_us(call, reps);
            const double orct = median_us([&] { return orc_clay_perform_coding(orc, iq.data(), ref.p.data(), B); }, reps);
            emit("clay42", B, dev, hx, def, orct, out.v == ref.v);
        }
        ecx_clay_destroy(clay);
        orc_clay_free(orc);
    }
    return 0;
}
