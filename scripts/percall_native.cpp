// percall_native.cpp -- per-call latency of the host-buffer entry points called from
// native code, as a JNI shim would call them (no Python marshalling): RS(4,2)
// encodeParity / decodeMissing and Clay(4,2) performCoding repair, with the gather
// path's H2D/D2H copies (host_zero_copy 0) and with zero-copy kernels (1).
// One JSON line per case: median microseconds per call over 300 calls.
//
//   hipcc -O2 -std=c++17 -I include scripts/percall_native.cpp -L repair-pipelining_amd -lecx \
//         -Wl,-rpath,'$ORIGIN/../repair-pipelining_amd' -o scripts/percall_native
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <functional>
#include <random>
#include <vector>

#include <hip/hip_runtime.h>

#include "ecx.h"
#include "ecx_tune.h"

static double median_us(const std::function<int()> &call, int reps = 300) {
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
    // PERCALL_SCHED=spin|yield|blocking: the HIP device scheduling flag, set before any
    // HIP call (how the host thread waits in hipStreamSynchronize); unset = the default.
    if (const char *m = std::getenv("PERCALL_SCHED")) {
        const std::string s = m;
        const unsigned f = s == "spin" ? hipDeviceScheduleSpin : s == "yield" ? hipDeviceScheduleYield
                         : s == "blocking" ? hipDeviceScheduleBlockingSync : hipDeviceScheduleAuto;
        if (hipSetDeviceFlags(f) != hipSuccess) return 2;
    }
    std::mt19937 rng(7);
    auto fill = [&](std::vector<uint8_t> &v) {
        for (auto &b : v) b = (uint8_t)rng();
    };
    ecx_rs *rs = nullptr;
    ecx_clay *clay = nullptr;
    const int erased = 1;
    if (ecx_rs_create(4, 2, &rs) || ecx_clay_create(4, 2, &erased, 1, &clay)) return 1;
    for (int zc : {0, 1}) {
        ecx_tune("host_zero_copy", zc);
        for (int L : {4096, 32768}) {
            std::vector<std::vector<uint8_t>> sh(6, std::vector<uint8_t>(L));
            for (auto &s : sh) fill(s);
            std::vector<uint8_t *> p(6);
            for (int i = 0; i < 6; ++i) p[i] = sh[i].data();
            const uint8_t present[6] = {1, 0, 1, 1, 1, 1};
            const double enc = median_us([&] { return ecx_rs_encode_parity(rs, p.data(), 6, L, 0, L); });
            const double dec = median_us([&] { return ecx_rs_decode_missing(rs, p.data(), present, 6, L, 0, L); });
            printf("{\"case\": \"RS(4,2) encodeParity, %d B shards\", \"host_zero_copy\": %d, \"us_per_call\": %.1f}\n",
                   L, zc, enc);
            printf("{\"case\": \"RS(4,2) decodeMissing (1 data shard), %d B shards\", \"host_zero_copy\": %d, "
                   "\"us_per_call\": %.1f}\n", L, zc, dec);
            std::vector<std::vector<uint8_t>> in(48, std::vector<uint8_t>(L)), out(8, std::vector<uint8_t>(L));
            std::vector<const uint8_t *> ip(48);
            std::vector<uint8_t *> op(8);
            for (int i = 0; i < 48; ++i) {
                fill(in[i]);
                ip[i] = (i % 6 == erased) ? nullptr : in[i].data();
            }
            for (int j = 0; j < 8; ++j) op[j] = out[j].data();
            const double clay_us = median_us([&] { return ecx_clay_perform_coding(clay, ip.data(), op.data(), L); });
            printf("{\"case\": \"Clay(4,2) performCoding repair e=1, B=%d\", \"host_zero_copy\": %d, "
                   "\"us_per_call\": %.1f}\n", L, zc, clay_us);
            fflush(stdout);
        }
    }
    ecx_tune("host_zero_copy", 1);
    // The CodingLoop operator API (EcxCodingLoop.codeSomeShards): the matrix comes with
    // every call; with and without the plan cache.
    {
        uint8_t mat[6 * 4];
        ecx_rs_matrix(rs, mat);
        for (int cache : {0, 256}) {
            ecx_tune("plan_cache", cache);
            for (int L : {4096, 32768}) {
                std::vector<std::vector<uint8_t>> sh(6, std::vector<uint8_t>(L));
                for (auto &s : sh) fill(s);
                std::vector<const uint8_t *> ip(4);
                std::vector<uint8_t *> op(2);
                for (int i = 0; i < 4; ++i) ip[i] = sh[i].data();
                for (int o = 0; o < 2; ++o) op[o] = sh[4 + o].data();
                const double us = median_us([&] { return ecx_code_some_shards(mat + 16, ip.data(), 4, op.data(), 2, 0, L); });
                printf("{\"case\": \"CodingLoop.codeSomeShards RS(4,2) parity, %d B shards\", \"plan_cache\": %d, "
                       "\"us_per_call\": %.1f}\n", L, cache, us);
                // one helper's hop of the pipelined chain (ClayCodeNode.kt:182-186): decodeMissingSingle
                const uint8_t present[6] = {0, 1, 1, 1, 1, 1};
                uint8_t *acc[1] = {sh[0].data()};
                const double us2 = median_us([&] {
                    return ecx_rs_decode_missing_single(rs, sh[2].data(), 2, 1, present, acc, 1, 0, L, 0);
                });
                printf("{\"case\": \"decodeMissingSingle RS(4,2), one helper, accumulate, %d B shards\", "
                       "\"plan_cache\": %d, \"us_per_call\": %.1f}\n", L, cache, us2);
                fflush(stdout);
            }
        }
        ecx_tune("plan_cache", 256);
    }
    // The LRC chain hop (NodeHelper.kt:86-97): the reference calls
    // LRCErasureCode.encodeParitySingle (RS(3,1), ReedSolomon.java:110-118) once per 34-B
    // word, 1024 words per 34,816-B block (PipelineUtil.kt:10-11).  The same partial sums
    // for the whole block: one host call over 34,816 B, or one device-resident
    // ecx_rs_encode_partial_batch (block already in HBM; includes the stream sync).
    {
        ecx_rs *rs31 = nullptr;
        if (ecx_rs_create(3, 1, &rs31)) return 1;
        const int W = 34, NW = 1024, BLK = W * NW;
        std::vector<uint8_t> block(BLK), acc(BLK);
        fill(block);
        const double word = median_us([&] { return ecx_rs_encode_parity_single(rs31, block.data(), acc.data(), 1, 0, 0, W); });
        const double blk = median_us([&] { return ecx_rs_encode_parity_single(rs31, block.data(), acc.data(), 1, 0, 0, BLK); });
        uint8_t *d_in = nullptr, *d_acc = nullptr;
        if (hipMalloc(&d_in, BLK) != hipSuccess || hipMalloc(&d_acc, BLK) != hipSuccess) return 1;
        if (hipMemcpy(d_in, block.data(), BLK, hipMemcpyHostToDevice) != hipSuccess) return 1;
        const double dev = median_us([&] {
            int st = ecx_rs_encode_partial_batch(rs31, 1, d_in, BLK, d_acc, BLK, BLK, 1, BLK, 0, nullptr);
            return st ? st : ecx_synchronize(nullptr);
        });
        printf("{\"case\": \"LRC chain hop, encodeParitySingle per 34-B word (NodeHelper.kt:89)\", \"us_per_call\": %.1f, "
               "\"calls_per_block\": %d, \"us_per_block\": %.1f}\n", word, NW, word * NW);
        printf("{\"case\": \"LRC chain hop, one encodeParitySingle over the 34,816-B block (host buffers)\", "
               "\"us_per_call\": %.1f, \"calls_per_block\": 1, \"us_per_block\": %.1f}\n", blk, blk);
        printf("{\"case\": \"LRC chain hop, ecx_rs_encode_partial_batch over the block in HBM (+ sync)\", "
               "\"us_per_call\": %.1f, \"calls_per_block\": 1, \"us_per_block\": %.1f}\n", dev, dev);
        fflush(stdout);
        (void)hipFree(d_in);
        (void)hipFree(d_acc);
        ecx_rs_destroy(rs31);
    }
    // Large per-call buffers (the byte[][] API on BASELINE config 5's shape): RS(12,4)
    // encodeParity and a 2-erasure decodeMissing over 16 x L host shards; algorithmic
    // GB/s = (12 read + 4 or 2 written) x L per call.
    {
        ecx_rs *rs124 = nullptr;
        if (ecx_rs_create(12, 4, &rs124)) return 1;
        for (int L : {1 << 20, 4 << 20}) {
            std::vector<std::vector<uint8_t>> sh(16, std::vector<uint8_t>(L));
            for (auto &s : sh) fill(s);
            std::vector<uint8_t *> p(16);
            for (int i = 0; i < 16; ++i) p[i] = sh[i].data();
            uint8_t present[16];
            for (int i = 0; i < 16; ++i) present[i] = i >= 2;
            const double enc = median_us([&] { return ecx_rs_encode_parity(rs124, p.data(), 16, L, 0, L); }, 20);
            const double dec = median_us([&] { return ecx_rs_decode_missing(rs124, p.data(), present, 16, L, 0, L); }, 20);
            printf("{\"case\": \"RS(12,4) encodeParity, %d B shards (host)\", \"us_per_call\": %.1f, \"GBps\": %.2f}\n", L,
                   enc, 16.0 * L / enc / 1e3);
            printf("{\"case\": \"RS(12,4) decodeMissing {0,1}, %d B shards (host)\", \"us_per_call\": %.1f, \"GBps\": %.2f}\n", L,
                   dec, 14.0 * L / dec / 1e3);
            fflush(stdout);
        }
        ecx_rs_destroy(rs124);
    }
    ecx_clay_destroy(clay);
    ecx_rs_destroy(rs);
    return 0;
}
