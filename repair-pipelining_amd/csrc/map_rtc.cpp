// map_rtc.cpp -- generation, hiprtc compilation and launch of the bit-plane kernel for
// one composed map (map_rtc.hpp).
#include "map_rtc.hpp"

#include <algorithm>
#include <map>
#include <mutex>
#include <sstream>
#include <vector>

#include "clay_rtc.hpp"
#include "engine.hpp"

namespace ecx {

namespace {

int popc(unsigned v) { return __builtin_popcount(v); }

// The used columns of the map: inputs with at least one non-zero coefficient.
std::vector<int> used_columns(const LinearMap &m) {
    std::vector<int> cols;
    for (int j = 0; j < m.n_in; ++j) {
        bool any = false;
        for (int o = 0; o < m.n_out && !any; ++o) any = m.at(o, j) != 0;
        if (any) cols.push_back(j);
    }
    return cols;
}

// One input's share of every row, in planes: output plane i of row r takes the XOR of
// the input planes in plane_sets(c_r)[i].  Each such set is split into its low nibble
// (planes 0-3) and high nibble (4-7); every nibble subset of two or more planes that
// some target needs is materialised once (built from its largest already available
// subset), and every target is then one x3(acc, lo, hi) -- or a plain XOR / copy when a
// nibble is empty or the row is still unwritten.
void emit_input(std::ostringstream &o, const LinearMap &m, int j, const std::string &x, std::vector<bool> &fresh) {
    struct Target {
        int row, plane;
        unsigned lo, hi;
    };
    std::vector<Target> targets;
    for (int r = 0; r < m.n_out; ++r) {
        const uint8_t c = m.at(r, j);
        if (!c) continue;
        const auto sets = plane_sets(c);
        for (int i = 0; i < 8; ++i) {
            unsigned mask = 0;
            for (int p : sets[i]) mask |= 1u << p;
            targets.push_back({r, i, mask & 0xFu, mask >> 4});
        }
    }
    for (int half = 0; half < 2; ++half) {
        const char pre = half ? 'h' : 'l';
        auto single = [&](int k) { return x + "[" + std::to_string(k + 4 * half) + "]"; };
        std::vector<unsigned> need;
        for (const Target &t : targets) {
            const unsigned v = half ? t.hi : t.lo;
            if (popc(v) >= 2 && std::find(need.begin(), need.end(), v) == need.end()) need.push_back(v);
        }
        std::stable_sort(need.begin(), need.end(), [](unsigned a, unsigned b) { return popc(a) < popc(b); });
        std::vector<unsigned> have;  // materialised subsets (plus the singles, implicitly)
        for (unsigned v : need) {
            unsigned best = 0;
            for (unsigned h : have)
                if ((h & ~v) == 0 && popc(h) > popc(best)) best = h;
            std::vector<int> rest;
            std::string cur;
            if (best) {
                cur = std::string(1, pre) + std::to_string(best);
                for (int k = 0; k < 4; ++k)
                    if ((v & ~best) >> k & 1u) rest.push_back(k);
            } else {
                for (int k = 0; k < 4; ++k)
                    if (v >> k & 1u) rest.push_back(k);
                cur = single(rest[0]);
                rest.erase(rest.begin());
            }
            size_t k = 0;
            for (; k + 1 < rest.size(); k += 2) cur = "x3(" + cur + ", " + single(rest[k]) + ", " + single(rest[k + 1]) + ")";
            if (k < rest.size()) cur = "(" + cur + " ^ " + single(rest[k]) + ")";
            o << "    const u32 " << pre << v << " = " << cur << ";\n";
            have.push_back(v);
        }
    }
    auto term = [&](unsigned v, int half) -> std::string {
        if (!v) return "";
        if (popc(v) == 1) return x + "[" + std::to_string(__builtin_ctz(v) + 4 * half) + "]";
        return std::string(1, half ? 'h' : 'l') + std::to_string(v);
    };
    for (const Target &t : targets) {
        const std::string a = term(t.lo, 0), b = term(t.hi, 1);
        const std::string d = "acc" + std::to_string(t.row) + "[" + std::to_string(t.plane) + "]";
        if (a.empty() && b.empty()) {
            if (fresh[t.row]) o << "    " << d << " = 0u;\n";
            continue;
        }
        if (fresh[t.row]) {
            if (!a.empty() && !b.empty()) o << "    " << d << " = " << a << " ^ " << b << ";\n";
            else o << "    " << d << " = " << (a.empty() ? b : a) << ";\n";
        } else {
            if (!a.empty() && !b.empty()) o << "    " << d << " = x3(" << d << ", " << a << ", " << b << ");\n";
            else o << "    " << d << " ^= " << (a.empty() ? b : a) << ";\n";
        }
    }
    for (const Target &t : targets) fresh[t.row] = false;
}

}  // namespace

bool map_planes_supported(const LinearMap &m, std::string *why) {
    auto no = [&](const char *w) {
        if (why) *why = w;
        return false;
    };
    if (m.n_out < 1 || m.n_out > kPlanesMaxRows) return no("k_map_planes keeps every row in registers: 1..16 rows");
    if (m.nnz() > kPlanesMaxNnz) return no("k_map_planes: too many coefficients for straight-line code");
    if ((int)m.in_slot.size() != m.n_in || (int)m.out_slot.size() != m.n_out) return no("malformed map");
    return true;
}

std::string map_planes_source(const LinearMap &m, const PlanesShape &shape, bool accumulate) {
    std::string why;
    if (!map_planes_supported(m, &why)) throw Error(ECX_E_ILLEGAL_ARGUMENT, why);
    const std::vector<int> cols = used_columns(m);
    const int R = m.n_out, n = (int)cols.size();
    std::ostringstream o;
    o << "// k_map_planes: generated by map_rtc.cpp for a " << R << " x " << m.n_in << " map (" << m.nnz()
      << " coefficients over " << n << " used inputs)" << (accumulate ? ", accumulating" : "") << "\n";
    o << rtc_prelude();
    o << "extern \"C\" __global__ void __launch_bounds__(" << kPlanesThreads << ", " << shape.waves << ")\n"
      << "k_map_planes(const unsigned char *in, long long iss, long long isl, unsigned char *out, long long oss,\n"
      << "             long long osl, long long n_chunks) {\n"
      << "    const u32 b = blockIdx.x;\n"
      << "    const long long c = (long long)(b % (u32)n_chunks), s = (long long)(b / (u32)n_chunks);\n"
      << "    const u64 ib = uniform64((u64)(in + s * iss + c * 4096));\n"
      << "    unsigned char *const ob = (unsigned char *)uniform64((u64)(out + s * oss + c * 4096));\n"
      << "    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)ib, 0, 0x7FFFFFFF, 0x00020000);\n"
      << "    const u32 voff = threadIdx.x * 16u, sl = (u32)isl;\n"
      << "    const u32 m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);\n"
      << "    auto ld = [&](u32 so, u32 (&x)[8]) {\n"
      << "        const auto v0 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, (int)so, " << (shape.nt_loads ? 2 : 0)
      << ");\n"
      << "        const auto v1 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(voff + 2048u), (int)so, "
      << (shape.nt_loads ? 2 : 0) << ");\n"
      << "        x[0] = v0[0]; x[1] = v0[1]; x[2] = v0[2]; x[3] = v0[3];\n"
      << "        x[4] = v1[0]; x[5] = v1[1]; x[6] = v1[2]; x[7] = v1[3];\n"
      << "    };\n"
      << "    auto st = [&](long long slot, u32 (&x)[8]) {\n"
      << "        unsigned char *q = ob + slot * osl + voff;\n";
    if (accumulate)
        o << "        const u32x4 p0 = *(const gu32x4 *)q, p1 = *(const gu32x4 *)(q + 2048);\n"
          << "        x[0] ^= p0[0]; x[1] ^= p0[1]; x[2] ^= p0[2]; x[3] ^= p0[3];\n"
          << "        x[4] ^= p1[0]; x[5] ^= p1[1]; x[6] ^= p1[2]; x[7] ^= p1[3];\n";
    o << "        __builtin_nontemporal_store((u32x4){x[0], x[1], x[2], x[3]}, (gu32x4 *)q);\n"
      << "        __builtin_nontemporal_store((u32x4){x[4], x[5], x[6], x[7]}, (gu32x4 *)(q + 2048));\n"
      << "    };\n";
    for (int r = 0; r < R; ++r) o << "    u32 acc" << r << "[8];\n";
    // Loads run `lookahead` inputs ahead of the one being computed; an empty asm with a
    // memory clobber after each input keeps the scheduler from hoisting every load to
    // the top (the Clay kernel spilled that way, clay_rtc.cpp).
    const int L = std::max(0, std::min(shape.lookahead, 15));
    auto emit_load = [&](int it) {
        o << "    u32 in" << it << "[8];\n    ld(" << m.in_slot[cols[it]] << "u * sl, in" << it << ");\n";
    };
    for (int it = 0; it < std::min(L, n); ++it) emit_load(it);
    std::vector<bool> fresh(R, true);
    for (int it = 0; it < n; ++it) {
        if (it + L < n) emit_load(it + L);
        const std::string x = "in" + std::to_string(it);
        o << "    {  // input column " << cols[it] << " (slot " << m.in_slot[cols[it]] << ")\n"
          << "    tr(" << x << ", m4, m2, m1);\n";
        emit_input(o, m, cols[it], x, fresh);
        o << "    }\n    asm volatile(\"\" ::: \"memory\");\n";
    }
    for (int r = 0; r < R; ++r) {
        if (fresh[r]) {  // a row no input reaches: zeros (or nothing to add)
            if (accumulate) continue;
            o << "    for (int i = 0; i < 8; ++i) acc" << r << "[i] = 0u;\n";
        } else {
            o << "    untr(acc" << r << ", m4, m2, m1);\n";
        }
        o << "    st(" << m.out_slot[r] << "ll, acc" << r << ");\n";
    }
    o << "}\n";
    return o.str();
}

// ---------------------------------------------------------------- the kernel object
struct MapPlanes::Impl {
    std::mutex mu;
    struct Loaded {
        hipModule_t mod = nullptr;
        hipFunction_t fn = nullptr;
    };
    std::map<std::string, std::string> source;                  // shape key -> source
    std::map<std::string, std::vector<char>> code;              // arch + source -> code object (compiled once)
    std::map<std::pair<std::string, int>, Loaded> dev;          // (source, device) -> module
    std::map<std::pair<std::string, int>, std::string> failed;  // (source, device) -> why (deterministic: not retried)
};

MapPlanes::MapPlanes(LinearMap m) : map_(std::move(m)), impl_(new Impl) {
    std::string why;
    if (!map_planes_supported(map_, &why)) throw Error(ECX_E_ILLEGAL_ARGUMENT, why);
}

MapPlanes::~MapPlanes() {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return;
    for (auto &kv : impl_->dev) {
        (void)hipSetDevice(kv.first.second);
        (void)hipModuleUnload(kv.second.mod);
    }
    (void)hipSetDevice(cur);
}

namespace {
PlanesShape planes_current_shape() {
    const Tuning t = tuning();  // one snapshot
    PlanesShape sh;
    sh.lookahead = t.planes_lookahead;
    sh.waves = t.planes_waves;
    return sh;
}
}  // namespace

bool MapPlanes::load(const PlanesShape &sh, bool accumulate, hipFunction_t *fn, std::string *why) {
    int d = 0;
    check_hip(hipGetDevice(&d), "hipGetDevice");
    std::lock_guard<std::mutex> lk(impl_->mu);
    const std::string key = std::to_string(sh.lookahead) + "/" + std::to_string(sh.waves) + "/" +
                            std::to_string((int)sh.nt_loads) + "/" + std::to_string((int)accumulate);
    auto si = impl_->source.find(key);
    if (si == impl_->source.end()) si = impl_->source.emplace(key, map_planes_source(map_, sh, accumulate)).first;
    const std::string &src = si->second;
    const std::pair<std::string, int> dk{src, d};
    auto di = impl_->dev.find(dk);
    if (di == impl_->dev.end()) {
        auto f = impl_->failed.find(dk);
        if (f != impl_->failed.end()) {
            if (why) *why = f->second;
            return false;
        }
        Impl::Loaded n;
        bool deterministic = true;  // as ClayRtc::prepare: load errors are retried, compile errors not
        try {
            const std::string arch = rtc_offload_arch();
            auto ci = impl_->code.find(arch + "\n" + src);
            if (ci == impl_->code.end()) ci = impl_->code.emplace(arch + "\n" + src, rtc_compile(src, arch)).first;
            const hipError_t le = hipModuleLoadData(&n.mod, ci->second.data());
            deterministic = le != hipErrorOutOfMemory;
            check_hip(le, "hipModuleLoadData(k_map_planes)");
            check_hip(hipModuleGetFunction(&n.fn, n.mod, kernel_name()), "hipModuleGetFunction(k_map_planes)");
        } catch (const Error &e) {
            if (n.mod) (void)hipModuleUnload(n.mod);
            if (deterministic) impl_->failed[dk] = e.what();
            if (why) *why = e.what();
            return false;
        }
        di = impl_->dev.emplace(dk, n).first;
    }
    if (fn) *fn = di->second.fn;
    return true;
}

bool MapPlanes::available(bool accumulate, std::string *why) {
    return load(planes_current_shape(), accumulate, nullptr, why);
}

void MapPlanes::launch(const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride, uint8_t *out,
                       int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes, int64_t nchunks,
                       bool accumulate, hipStream_t stream) {
    if (nstripes <= 0 || nchunks <= 0) return;
    hipFunction_t fn = nullptr;
    std::string why;
    if (!load(planes_current_shape(), accumulate, &fn, &why)) throw Error(ECX_E_DEVICE, why);
    const int64_t max_blocks = (int64_t)1 << 30;
    const int64_t stripes_per_launch = std::max<int64_t>(1, max_blocks / nchunks);
    set_last_kernel(kernel_name());
    for (int64_t s0 = 0; s0 < nstripes; s0 += stripes_per_launch) {
        const int64_t ns = std::min(stripes_per_launch, nstripes - s0);
        const uint8_t *pin = in + s0 * in_stripe_stride;
        uint8_t *pout = out + s0 * out_stripe_stride;
        long long iss = in_stripe_stride, isl = in_slot_stride, oss = out_stripe_stride, osl = out_slot_stride;
        long long nc = nchunks;
        void *args[] = {&pin, &iss, &isl, &pout, &oss, &osl, &nc};
        check_hip(hipModuleLaunchKernel(fn, (unsigned)(ns * nchunks), 1, 1, kPlanesThreads, 1, 1, 0, stream, args,
                                        nullptr),
                  "k_map_planes launch");
    }
}

}  // namespace ecx
