// host_exec_check.cpp -- host-only check of the per-call executor (repair-pipelining_amd/csrc/
// host_exec.cpp) at every instruction-set level this CPU has (AVX-512BW + GFNI, AVX2, scalar),
// built with AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_native.py:
//   * every product c * x (c, x in 0..255) through a one-coefficient map equals Field::mul
//     (the GF2P8AFFINEQB bit matrix and the nibble tables of every c);
//   * random maps (1..20 inputs, 1..8 outputs, zero and one coefficients included) over byte
//     counts around every vector and block boundary (1, 34, 63..65, 2174, 4095..4097, 10000) at
//     odd offsets equal a dense table-row application, and bytes outside the range are untouched;
//   * outputs aliasing inputs (x ^= c * y, decodeMissing in place) give the pre-update result,
//     and so do outputs overlapping an input at a shifted address;
//   * host_exec_all_zero is true exactly when every output row is zero over the range.
// Exit status 0 = all good.
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../repair-pipelining_amd/csrc/host_exec.hpp"

using namespace ecx;

namespace {
int failures = 0;
std::mt19937_64 rng(2025);

void expect(bool ok, const char *what, int level) {
    if (!ok) {
        std::fprintf(stderr, "FAIL (isa %d): %s\n", level, what);
        ++failures;
    }
}

LinearMap random_map(int n_out, int n_in) {
    LinearMap m;
    m.n_out = n_out;
    m.n_in = n_in;
    m.a.resize((size_t)n_out * n_in);
    for (auto &c : m.a) {
        const int r = (int)(rng() % 10);
        c = r == 0 ? 0 : (r == 1 ? 1 : (uint8_t)rng());
    }
    for (int j = 0; j < n_in; ++j) m.in_slot.push_back(j);
    for (int o = 0; o < n_out; ++o) m.out_slot.push_back(n_in + o);
    return m;
}

void check_level(int level) {
    const Field &f = Field::get();
    // every product
    {
        LinearMap m;
        m.n_out = 1;
        m.n_in = 1;
        m.a = {0};
        m.in_slot = {0};
        m.out_slot = {1};
        std::vector<uint8_t> x(256), y(256);
        for (int v = 0; v < 256; ++v) x[v] = (uint8_t)v;
        for (int c = 0; c < 256; ++c) {
            m.a[0] = (uint8_t)c;
            const uint8_t *ins[2] = {x.data(), nullptr};
            uint8_t *outs[2] = {nullptr, y.data()};
            host_exec_apply(m, ins, outs, 0, 256);
            bool ok = true;
            for (int v = 0; v < 256; ++v) ok = ok && y[v] == f.mul((uint8_t)c, (uint8_t)v);
            expect(ok, "c * x for every c, x", level);
        }
    }
    // random maps, sizes, offsets
    for (int64_t len : {1, 2, 34, 63, 64, 65, 127, 2174, 4095, 4096, 4097, 8192, 10000}) {
        for (int trial = 0; trial < 4; ++trial) {
            const int n_in = 1 + (int)(rng() % 20), n_out = 1 + (int)(rng() % 8);
            const LinearMap m = random_map(n_out, n_in);
            const int64_t off = (int64_t)(rng() % 7), pad = 5;
            std::vector<std::vector<uint8_t>> buf((size_t)(n_in + n_out), std::vector<uint8_t>((size_t)(off + len + pad)));
            for (auto &b : buf)
                for (auto &v : b) v = (uint8_t)rng();
            std::vector<std::vector<uint8_t>> want = buf;
            for (int o = 0; o < n_out; ++o)
                for (int64_t i = 0; i < len; ++i) {
                    uint8_t v = 0;
                    for (int j = 0; j < n_in; ++j) v ^= f.mul(m.at(o, j), buf[(size_t)j][(size_t)(off + i)]);
                    want[(size_t)(n_in + o)][(size_t)(off + i)] = v;
                }
            std::vector<const uint8_t *> ins;
            std::vector<uint8_t *> outs;
            for (auto &b : buf) {
                ins.push_back(b.data());
                outs.push_back(b.data());
            }
            host_exec_apply(m, ins.data(), outs.data(), off, len);
            expect(buf == want, "random map vs dense application (range and the bytes around it)", level);
            // all_zero: the check map [M | I] over (inputs, the outputs just written) is zero
            LinearMap chk;
            chk.n_out = n_out;
            chk.n_in = n_in + n_out;
            chk.a.assign((size_t)chk.n_out * chk.n_in, 0);
            for (int o = 0; o < n_out; ++o) {
                for (int j = 0; j < n_in; ++j) chk.a[(size_t)o * chk.n_in + j] = m.at(o, j);
                chk.a[(size_t)o * chk.n_in + n_in + o] = 1;
                chk.out_slot.push_back(o);
            }
            for (int j = 0; j < chk.n_in; ++j) chk.in_slot.push_back(j);
            expect(host_exec_all_zero(chk, ins.data(), off, len), "check map of a valid result is all zero", level);
            buf[(size_t)(n_in + n_out - 1)][(size_t)(off + len - 1)] ^= 0x10;
            expect(!host_exec_all_zero(chk, ins.data(), off, len), "one flipped byte makes it non-zero", level);
        }
    }
    // the one-coefficient form (encodeParitySingle / code_single), assign and accumulate
    for (int64_t len : {1, 34, 1023, 1024, 1025, 5000}) {
        std::vector<uint8_t> y((size_t)len), x((size_t)len);
        for (auto &v : y) v = (uint8_t)rng();
        for (auto &v : x) v = (uint8_t)rng();
        for (int acc = 0; acc < 2; ++acc) {
            const uint8_t c = (uint8_t)(rng() | 2);
            std::vector<uint8_t> want = x;
            for (int64_t i = 0; i < len; ++i)
                want[(size_t)i] = (uint8_t)((acc ? x[(size_t)i] : 0) ^ f.mul(c, y[(size_t)i]));
            host_exec_scale(c, y.data(), x.data(), len, acc != 0);
            expect(x == want, "host_exec_scale", level);
        }
        std::vector<uint8_t> want = y;  // in place: y = 3 * y
        for (auto &v : want) v = f.mul(3, v);
        host_exec_scale(3, y.data(), y.data(), len, false);
        expect(y == want, "host_exec_scale in place", level);
    }
    // aliasing: x ^= c * y (code_single's accumulate row [c, 1] over {y, x} written to x)
    for (int64_t len : {33, 4096, 9000}) {
        LinearMap m;
        m.n_out = 1;
        m.n_in = 2;
        m.a = {0x8E, 1};
        m.in_slot = {0, 1};
        m.out_slot = {1};
        std::vector<uint8_t> y((size_t)len), x((size_t)len);
        for (auto &v : y) v = (uint8_t)rng();
        for (auto &v : x) v = (uint8_t)rng();
        std::vector<uint8_t> want = x;
        for (int64_t i = 0; i < len; ++i) want[(size_t)i] ^= f.mul(0x8E, y[(size_t)i]);
        const uint8_t *ins[2] = {y.data(), x.data()};
        uint8_t *outs[2] = {nullptr, x.data()};
        host_exec_apply(m, ins, outs, 0, len);
        expect(x == want, "output aliasing an input", level);
    }
    // shifted overlap (round-5 advice): the output starts d bytes after (or before) an input
    // inside one buffer, across 4 KiB blocks; the result is the map of the ORIGINAL input bytes
    for (int64_t len : {100, 4096, 9000}) {
        for (int64_t d : {-4097, -1, 1, 17, 4096, 5000}) {
            if (d >= len || -d >= len) continue;
            LinearMap m;
            m.n_out = 1;
            m.n_in = 2;
            m.a = {0x53, 0xC1};
            m.in_slot = {0, 1};
            m.out_slot = {2};
            std::vector<uint8_t> arena((size_t)(3 * len + 8192)), other((size_t)len);
            for (auto &v : arena) v = (uint8_t)rng();
            for (auto &v : other) v = (uint8_t)rng();
            uint8_t *in0 = arena.data() + len + 4096, *out = in0 + d;
            const std::vector<uint8_t> orig(in0, in0 + len);
            std::vector<uint8_t> want((size_t)len);
            for (int64_t i = 0; i < len; ++i)
                want[(size_t)i] = (uint8_t)(f.mul(0x53, orig[(size_t)i]) ^ f.mul(0xC1, other[(size_t)i]));
            const uint8_t *ins[3] = {in0, other.data(), nullptr};
            uint8_t *outs[3] = {nullptr, nullptr, out};
            host_exec_apply(m, ins, outs, 0, len);
            expect(std::memcmp(out, want.data(), (size_t)len) == 0, "output overlapping an input at a shift", level);
            // the one-coefficient form over the same kind of overlap
            for (auto &v : arena) v = (uint8_t)rng();
            const std::vector<uint8_t> orig2(in0, in0 + len);
            host_exec_scale(0x1D, in0, out, len, false);
            bool ok = true;
            for (int64_t i = 0; i < len; ++i) ok = ok && out[i] == f.mul(0x1D, orig2[(size_t)i]);
            expect(ok, "host_exec_scale with a shifted overlap", level);
        }
    }
}
}  // namespace

int main() {
    int ran = 0;
    for (int level : {2, 1, 0}) {
        if (host_exec_force_isa(level) != level) {
            std::printf("isa %d: not on this CPU, skipped\n", level);
            continue;
        }
        check_level(level);
        ++ran;
    }
    host_exec_force_isa(-1);
    if (failures) return 1;
    std::printf("host_exec_check: ok (%d instruction-set levels)\n", ran);
    return 0;
}
