// planner_check.cpp -- host-only check of the planner (gf.cpp, codes.cpp), built
// with AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_native.py.
//
// Round trips through the composed maps with a dense host application:
//   * RS(k,m): encode_map, then decode_map for every erasure pattern of up to m
//     shards (k,m small) or sampled patterns, rebuilds the erased shards;
//   * Clay(k,m) (+ shortened Clay(10,4)): the encode map (erased = parity
//     column), then the repair map of every single node and of sampled node
//     pairs, rebuilds the erased sub-chunks of a random codeword;
//   * LRC: encode, then every one-block-per-group erasure;
//   * Matrix::inverse throws "singular" with ECX_E_SINGULAR.
// Exit status 0 = all good; failures print and exit 1.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../repair-pipelining_amd/csrc/codes.hpp"

using namespace ecx;

namespace {
int failures = 0;
std::mt19937_64 rng(12345);

void expect(bool ok, const char *what) {
    if (!ok) {
        std::fprintf(stderr, "FAIL: %s\n", what);
        ++failures;
    }
}

// out[slot] = sum_j a[o][j] * in[in_slot[j]] over `len` bytes, slots index `bufs`.
void apply(const LinearMap &m, std::vector<std::vector<uint8_t>> &bufs, size_t len) {
    const Field &f = Field::get();
    std::vector<std::vector<uint8_t>> res(m.n_out, std::vector<uint8_t>(len, 0));
    for (int o = 0; o < m.n_out; ++o)
        for (int j = 0; j < m.n_in; ++j) {
            const uint8_t c = m.at(o, j);
            if (!c) continue;
            const std::vector<uint8_t> &x = bufs.at((size_t)m.in_slot[j]);
            for (size_t i = 0; i < len; ++i) res[o][i] ^= f.mul(c, x[i]);
        }
    for (int o = 0; o < m.n_out; ++o) bufs.at((size_t)m.out_slot[o]) = res[o];
}

std::vector<uint8_t> random_bytes(size_t n) {
    std::vector<uint8_t> v(n);
    for (auto &b : v) b = (uint8_t)rng();
    return v;
}

void check_rs(int k, int m, int samples) {
    RsCode rs(k, m);
    const size_t len = 33;
    std::vector<std::vector<uint8_t>> sh(k + m);
    for (int i = 0; i < k; ++i) sh[i] = random_bytes(len);
    for (int i = k; i < k + m; ++i) sh[i].assign(len, 0);
    apply(rs.encode_map(), sh, len);
    const auto orig = sh;
    for (int s = 0; s < samples; ++s) {
        std::vector<bool> present(k + m, true);
        const int ne = 1 + (int)(rng() % m);
        for (int e = 0; e < ne; ++e) present[rng() % (k + m)] = false;
        auto work = orig;
        for (int i = 0; i < k + m; ++i)
            if (!present[i]) work[i].assign(len, 0xEE);
        apply(rs.decode_map(present), work, len);
        expect(work == orig, "RS decode_map round trip");
    }
}

void check_clay(int k, int m, int v, const std::vector<std::vector<int>> &patterns) {
    const int n_real = k + m;
    std::vector<int> parity;
    for (int i = k; i < n_real; ++i) parity.push_back(i);
    ClayPlanner enc(k, m, parity, v);
    const int alpha = enc.alpha(), slots = n_real * alpha;
    const size_t len = 17;
    std::vector<bool> present(slots, true);
    for (int z = 0; z < alpha; ++z)
        for (int p : parity) present[(size_t)z * n_real + p] = false;
    // encode: data sub-chunks -> parity sub-chunks (outputs are z*|E| + j)
    std::vector<std::vector<uint8_t>> stripe(slots);
    for (int s = 0; s < slots; ++s) stripe[s] = present[s] ? random_bytes(len) : std::vector<uint8_t>(len, 0);
    LinearMap em = enc.perform_coding_map(present);
    {
        std::vector<std::vector<uint8_t>> ins = stripe;  // in slots index the stripe
        std::vector<std::vector<uint8_t>> outs(parity.size() * alpha, std::vector<uint8_t>(len, 0));
        const Field &f = Field::get();
        for (int o = 0; o < em.n_out; ++o)
            for (int j = 0; j < em.n_in; ++j)
                if (em.at(o, j))
                    for (size_t i = 0; i < len; ++i) outs[em.out_slot[o]][i] ^= f.mul(em.at(o, j), ins[em.in_slot[j]][i]);
        for (int z = 0; z < alpha; ++z)
            for (size_t j = 0; j < parity.size(); ++j) stripe[(size_t)z * n_real + parity[j]] = outs[z * parity.size() + j];
    }
    for (const std::vector<int> &er : patterns) {
        ClayPlanner rep(k, m, er, v);
        std::vector<bool> pres(slots, true);
        for (int z = 0; z < alpha; ++z)
            for (int e : er) pres[(size_t)z * n_real + e] = false;
        LinearMap rm = rep.perform_coding_map(pres);
        const Field &f = Field::get();
        std::vector<std::vector<uint8_t>> outs(er.size() * alpha, std::vector<uint8_t>(len, 0));
        for (int o = 0; o < rm.n_out; ++o)
            for (int j = 0; j < rm.n_in; ++j)
                if (rm.at(o, j)) {
                    expect(pres[rm.in_slot[j]], "repair map reads an erased sub-chunk");
                    for (size_t i = 0; i < len; ++i) outs[rm.out_slot[o]][i] ^= f.mul(rm.at(o, j), stripe[rm.in_slot[j]][i]);
                }
        bool ok = true;
        for (int z = 0; z < alpha; ++z)
            for (size_t j = 0; j < er.size(); ++j) ok &= outs[z * er.size() + j] == stripe[(size_t)z * n_real + er[j]];
        expect(ok, "Clay repair map round trip");
    }
}

void check_lrc() {
    LrcCode lrc;
    const size_t len = 23;
    std::vector<std::vector<uint8_t>> b(LrcCode::kN);
    for (int i = 0; i < LrcCode::kN; ++i) b[i] = (i % 4 == 3) ? std::vector<uint8_t>(len, 0) : random_bytes(len);
    apply(lrc.encode_map(), b, len);
    const auto orig = b;
    for (int a = 0; a < 4; ++a)
        for (int c = 0; c < 4; ++c) {
            std::vector<bool> present(LrcCode::kN, true);
            present[a] = false;          // group 0
            present[8 + c] = false;      // group 2
            auto work = orig;
            work[a].assign(len, 1);
            work[8 + c].assign(len, 2);
            apply(lrc.decode_map(present), work, len);
            expect(work == orig, "LRC decode round trip");
        }
    std::vector<bool> two(LrcCode::kN, true);
    two[0] = two[1] = false;
    bool threw = false;
    try {
        lrc.decode_map(two);
    } catch (const Error &e) {
        threw = e.code == ECX_E_NOT_ENOUGH_SHARDS;
    }
    expect(threw, "LRC two missing in a group must throw NOT_ENOUGH_SHARDS");
}

void check_singular() {
    Matrix mtx(2, 2);
    mtx.at(0, 0) = mtx.at(0, 1) = mtx.at(1, 0) = mtx.at(1, 1) = 1;
    bool threw = false;
    try {
        (void)mtx.inverse();
    } catch (const Error &e) {
        threw = e.code == ECX_E_SINGULAR;
    }
    expect(threw, "singular matrix must throw ECX_E_SINGULAR");
}
}  // namespace

int main() {
    check_singular();
    check_rs(4, 2, 40);
    check_rs(12, 4, 60);
    check_rs(3, 1, 8);
    check_rs(2, 2, 12);
    check_clay(4, 2, 0, {{0}, {1}, {2}, {3}, {4}, {5}, {0, 1}, {1, 4}, {2, 5}});
    check_clay(6, 3, 0, {{0}, {4}, {8}, {1, 7}, {0, 3, 6}});
    check_clay(10, 4, 2, {{3}, {0}, {13}, {2, 11}});
    check_lrc();
    std::printf("planner_check: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
