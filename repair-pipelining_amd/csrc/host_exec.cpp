// host_exec.cpp -- the per-call executor below the CPU/GPU size threshold (SURVEY.md 8(b) group 1).
//
// The reference's drop-in sites call the codec at fine grain: one encodeParitySingle per 34-B
// word (NodeHelper.kt:89, 1,024 calls per block), one RS(2,2) decodeMissing per Clay sub-chunk
// pair of 2,174 B (ClayCodeNode.kt:125-132, ClayCodeHelper.kt:90).  A call that small is all
// latency on the GPU -- staging, a launch and a synchronise, 19-52 us -- against well under a
// microsecond of arithmetic, so per-call entry points whose byte count is at most the
// threshold (ecx_tune "host_exec_kib", default 8 KiB; profiles/r05_percall_threshold.jsonl)
// apply the map here, on the calling thread; everything above it, and every batch entry
// point, runs the HIP kernels.  It is not a fallback: with no HIP device the call fails (ECX_E_DEVICE) as
// the GPU path would, and "host_exec_kib" 0 sends every call to the device.
//
// Arithmetic: c * x over GF(2^8) (0x11D) is linear over GF(2), so it is one GF2P8AFFINEQB with
// the 8x8 bit matrix of c (64 bytes per instruction, AVX-512 + GFNI), or two 16-entry nibble
// lookups with VPSHUFB (AVX2: c*x = T_lo[x & 15] ^ T_hi[x >> 4]), or the 256-byte product row
// (scalar tails).  Outputs are computed per block into a scratch area before any is stored, so
// outputs may alias inputs (decodeMissing in place, the accumulate rows of code_single).
// Plain C++ (no HIP headers): compiled by the host compiler (Makefile), so its target-attribute
// SIMD functions and CPU-feature checks never reach the device compilation.
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cstring>

#include "host_exec.hpp"

namespace ecx {
namespace {

constexpr int64_t kBlock = 4096;  // bytes of every row per pass (scratch: n_out x kBlock)

// The bit matrix of x -> c*x for GF2P8AFFINEQB: result bit i = parity(byte (7 - i) of A & x),
// so byte (7 - i) holds, at bit j, bit i of c * 2^j.
uint64_t affine_of(uint8_t c) {
    const Field &f = Field::get();
    uint8_t col[8];
    for (int j = 0; j < 8; ++j) col[j] = f.mul(c, (uint8_t)(1u << j));
    uint64_t a = 0;
    for (int i = 0; i < 8; ++i) {
        uint8_t row = 0;
        for (int j = 0; j < 8; ++j) row |= (uint8_t)(((col[j] >> i) & 1u) << j);
        a |= (uint64_t)row << (8 * (7 - i));
    }
    return a;
}

std::atomic<int> g_force_isa{-1};  // host_exec_force_isa (tests); read by every calling thread

int isa_level() {  // 2: AVX-512BW + GFNI, 1: AVX2, 0: scalar
    const int forced = g_force_isa.load(std::memory_order_relaxed);
    if (forced >= 0) return forced;
    static const int v = [] {
        __builtin_cpu_init();
        if (__builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("gfni")) return 2;
        if (__builtin_cpu_supports("avx2")) return 1;
        return 0;
    }();
    return v;
}

// Per-coefficient tables, built once: the GFNI bit matrix and the two AVX2 nibble tables of every c.
struct CoefTables {
    uint64_t affine[256];
    alignas(16) uint8_t lo[256][16], hi[256][16];
    CoefTables() {
        const Field &f = Field::get();
        for (int c = 0; c < 256; ++c) {
            affine[c] = affine_of((uint8_t)c);
            for (int v = 0; v < 16; ++v) {
                lo[c][v] = f.mul((uint8_t)c, (uint8_t)v);
                hi[c][v] = f.mul((uint8_t)c, (uint8_t)(v << 4));
            }
        }
    }
};
const CoefTables &tables() {
    static const CoefTables t;
    return t;
}

struct Coef {
    const uint8_t *in;  // input row at the block's first byte
    uint8_t c;
    uint64_t affine;          // GFNI matrix of c
    const uint8_t *lo, *hi;   // nibble tables of c (AVX2)
};

__attribute__((target("avx512f,avx512bw,gfni"))) void row_gfni(const Coef *cf, int n, uint8_t *acc, int64_t len) {
    int64_t b = 0;
    for (; b + 64 <= len; b += 64) {
        __m512i s = _mm512_setzero_si512();
        for (int k = 0; k < n; ++k) {
            const __m512i x = _mm512_loadu_si512((const void *)(cf[k].in + b));
            s = _mm512_xor_si512(s, cf[k].c == 1 ? x
                                                 : _mm512_gf2p8affine_epi64_epi8(
                                                       x, _mm512_set1_epi64((long long)cf[k].affine), 0));
        }
        _mm512_storeu_si512((void *)(acc + b), s);
    }
    if (b < len) {
        const __mmask64 m = len - b == 64 ? ~0ull : ((1ull << (len - b)) - 1);
        __m512i s = _mm512_setzero_si512();
        for (int k = 0; k < n; ++k) {
            const __m512i x = _mm512_maskz_loadu_epi8(m, cf[k].in + b);
            s = _mm512_xor_si512(s, cf[k].c == 1 ? x
                                                 : _mm512_gf2p8affine_epi64_epi8(
                                                       x, _mm512_set1_epi64((long long)cf[k].affine), 0));
        }
        _mm512_mask_storeu_epi8(acc + b, m, s);
    }
}

__attribute__((target("avx2"))) void row_avx2(const Coef *cf, int n, uint8_t *acc, int64_t len) {
    const __m256i nib = _mm256_set1_epi8(0x0F);
    int64_t b = 0;
    for (; b + 32 <= len; b += 32) {
        __m256i s = _mm256_setzero_si256();
        for (int k = 0; k < n; ++k) {
            const __m256i x = _mm256_loadu_si256((const __m256i *)(cf[k].in + b));
            if (cf[k].c == 1) {
                s = _mm256_xor_si256(s, x);
                continue;
            }
            const __m256i tl = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i *)cf[k].lo));
            const __m256i th = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i *)cf[k].hi));
            const __m256i l = _mm256_shuffle_epi8(tl, _mm256_and_si256(x, nib));
            const __m256i h = _mm256_shuffle_epi8(th, _mm256_and_si256(_mm256_srli_epi16(x, 4), nib));
            s = _mm256_xor_si256(s, _mm256_xor_si256(l, h));
        }
        _mm256_storeu_si256((__m256i *)(acc + b), s);
    }
    const Field &f = Field::get();
    for (; b < len; ++b) {
        uint8_t v = 0;
        for (int k = 0; k < n; ++k) v ^= f.row(cf[k].c)[cf[k].in[b]];
        acc[b] = v;
    }
}

void row_scalar(const Coef *cf, int n, uint8_t *acc, int64_t len) {
    const Field &f = Field::get();
    std::memset(acc, 0, (size_t)len);
    for (int k = 0; k < n; ++k) {
        const uint8_t *row = f.row(cf[k].c), *in = cf[k].in;
        for (int64_t b = 0; b < len; ++b) acc[b] ^= row[in[b]];
    }
}

// out rows (or, with `zero`, only whether every row is zero) of map `m` over [offset, offset+len)
bool apply_rows(const LinearMap &m, const uint8_t *const *inputs, uint8_t *const *outputs, int64_t offset,
                int64_t len, bool zero) {
    const CoefTables &t = tables();
    const int level = isa_level();
    thread_local std::vector<Coef> coefs;    // row o's coefficients: coefs[first[o] .. first[o + 1])
    thread_local std::vector<int> first;
    thread_local std::vector<uint8_t> scratch;
    coefs.clear();
    first.assign((size_t)m.n_out + 1, 0);
    for (int o = 0; o < m.n_out; ++o) {
        first[(size_t)o] = (int)coefs.size();
        for (int j = 0; j < m.n_in; ++j) {
            const uint8_t c = m.at(o, j);
            if (c) coefs.push_back({inputs[m.in_slot[j]] + offset, c, t.affine[c], t.lo[c], t.hi[c]});
        }
    }
    first[(size_t)m.n_out] = (int)coefs.size();
    const int64_t blk = std::min<int64_t>(len, kBlock);
    if (scratch.size() < (size_t)(m.n_out * blk)) scratch.resize((size_t)(m.n_out * blk));
    for (int64_t b0 = 0; b0 < len; b0 += kBlock) {
        const int64_t w = std::min<int64_t>(kBlock, len - b0);
        for (int o = 0; o < m.n_out; ++o) {
            Coef *r = coefs.data() + first[(size_t)o];
            const int n = first[(size_t)o + 1] - first[(size_t)o];
            uint8_t *acc = scratch.data() + (size_t)o * blk;
            if (n == 0) {
                std::memset(acc, 0, (size_t)w);
                continue;
            }
            if (level == 2) row_gfni(r, n, acc, w);
            else if (level == 1) row_avx2(r, n, acc, w);
            else row_scalar(r, n, acc, w);
            for (int k = 0; k < n; ++k) r[k].in += w;
        }
        if (zero) {
            for (int o = 0; o < m.n_out; ++o) {
                const uint8_t *acc = scratch.data() + (size_t)o * blk;
                for (int64_t i = 0; i < w; ++i)
                    if (acc[i]) return false;
            }
            continue;
        }
        // every row of this block is computed before any is stored: outputs may alias inputs
        for (int o = 0; o < m.n_out; ++o)
            std::memcpy(outputs[m.out_slot[o]] + offset + b0, scratch.data() + (size_t)o * blk, (size_t)w);
    }
    return true;
}

}  // namespace

namespace {
// [a, a + n) and [b, b + n) share a byte but start at different addresses
bool shifted_overlap(const uint8_t *a, const uint8_t *b, int64_t n) {
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    return x != y && x < y + (uintptr_t)n && y < x + (uintptr_t)n;
}
}  // namespace

void host_exec_apply(const LinearMap &m, const uint8_t *const *inputs, uint8_t *const *outputs, int64_t offset,
                     int64_t byte_count) {
    for (int slot : m.out_slot)
        if (!outputs[slot]) throw Error(ECX_E_NULL, "output buffer is null");
    // Block by block every row is computed before any is stored, so an output may BE an input
    // (the same address).  An output that overlaps an input at a shifted address would overwrite
    // input bytes a later block still reads: such inputs are read from a copy taken first, as the
    // device path stages every input before it writes anything.
    int max_in = 0;
    for (int slot : m.in_slot) max_in = std::max(max_in, slot);
    thread_local std::vector<const uint8_t *> ins;
    thread_local std::vector<uint8_t> copies;
    ins.assign(inputs, inputs + max_in + 1);
    std::vector<int> shifted;
    for (int j = 0; j < m.n_in; ++j) {
        const int slot = m.in_slot[j];
        if (!inputs[slot]) continue;
        for (int slot_o : m.out_slot)
            if (shifted_overlap(inputs[slot] + offset, outputs[slot_o] + offset, byte_count)) {
                if (std::find(shifted.begin(), shifted.end(), slot) == shifted.end()) shifted.push_back(slot);
                break;
            }
    }
    if (!shifted.empty()) {
        copies.resize(shifted.size() * (size_t)byte_count);
        for (size_t i = 0; i < shifted.size(); ++i) {
            uint8_t *c = copies.data() + i * (size_t)byte_count;
            std::memcpy(c, inputs[shifted[i]] + offset, (size_t)byte_count);
            ins[(size_t)shifted[i]] = c - offset;  // read back at + offset
        }
    }
    (void)apply_rows(m, ins.data(), outputs, offset, byte_count, false);
}

bool host_exec_all_zero(const LinearMap &m, const uint8_t *const *inputs, int64_t offset, int64_t byte_count) {
    return apply_rows(m, inputs, nullptr, offset, byte_count, true);
}

void host_exec_scale(uint8_t c, const uint8_t *in, uint8_t *out, int64_t n, bool accumulate) {
    const CoefTables &t = tables();
    const int level = isa_level();
    // out (=|^=) c * in, in blocks through a small stack buffer: out may be in (the same
    // address); an input overlapping out at a shifted address is copied first
    thread_local std::vector<uint8_t> copy;
    if (shifted_overlap(in, out, n)) {
        copy.assign(in, in + n);
        in = copy.data();
    }
    uint8_t acc[1024];
    Coef k[2] = {{in, c, t.affine[c], t.lo[c], t.hi[c]}, {out, 1, t.affine[1], t.lo[1], t.hi[1]}};
    const int terms = accumulate ? 2 : 1;
    for (int64_t b0 = 0; b0 < n; b0 += (int64_t)sizeof(acc)) {
        const int64_t w = std::min<int64_t>((int64_t)sizeof(acc), n - b0);
        if (level == 2) row_gfni(k, terms, acc, w);
        else if (level == 1) row_avx2(k, terms, acc, w);
        else row_scalar(k, terms, acc, w);
        std::memcpy(out + b0, acc, (size_t)w);
        k[0].in += w;
        k[1].in += w;
    }
}

int host_exec_isa() { return isa_level(); }

int host_exec_force_isa(int level) {
    g_force_isa.store(-1);
    const int have = isa_level();
    if (level > have) return -1;
    g_force_isa.store(level);
    return level;
}

}  // namespace ecx
