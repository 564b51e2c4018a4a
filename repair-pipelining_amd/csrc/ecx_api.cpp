// ecx_api.cpp -- the C ABI (include/ecx.h).  Translates planner/HIP errors into
// ecx_status codes; every arithmetic entry point executes on the HIP device.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <unordered_map>
#include <mutex>
#include <string>
#include <tuple>

#include "clay_rtc.hpp"
#include "map_rtc.hpp"
#include "engine.hpp"
#include "host_pipe.hpp"

using namespace ecx;

struct ecx_map {
    explicit ecx_map(LinearMap m) : cm(std::move(m)) {}
    CompiledMap cm;
};

struct ecx_rs {
    explicit ecx_rs(int k, int m) : code(k, m) {}
    RsCode code;
    bool shared = false;  // owned by the process-wide codec registry (ecx_rs_create)
    std::mutex mu;
    std::unique_ptr<ecx_map> enc, check;
    std::map<std::string, std::unique_ptr<ecx_map>> dec, partial;  // plans live as long as the codec
};

struct ecx_clay {
    ecx_clay(int k, int m, std::vector<int> e, int v = 0, bool is_test = false) : pl(k, m, std::move(e), v, is_test) {}
    ClayPlanner pl;
    bool shared = false;  // owned by the process-wide codec registry (ecx_clay_create)
    std::mutex mu;
    std::map<std::string, std::unique_ptr<ecx_map>> maps;
    // Single-node repair as the per-helper-plane kernel (clay_rtc.hpp), built on first use.
    std::unique_ptr<ClayRtc> rtc;
    int rtc_state = 0;  // 0 = not tried, 1 = available, -1 = not representable
    std::string rtc_why;
};

namespace {

thread_local std::string g_last_error;

// roctx ranges around the entry points (ecx_tune "roctx", or ECX_ROCTX=1 in the
// environment): `rocprofv3 --marker-trace` then shows which call issued which kernels.
// The marker library is opened on first use; without it the ranges are no-ops.
struct Roctx {
    int (*push)(const char *) = nullptr;
    int (*pop)() = nullptr;
};
const Roctx &roctx_lib() {
    static const Roctx r = [] {
        Roctx x;
        void *h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            x.push = reinterpret_cast<int (*)(const char *)>(dlsym(h, "roctxRangePushA"));
            x.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
            if (!x.push || !x.pop) x = Roctx{};
        }
        return x;
    }();
    return r;
}
std::atomic<int> g_roctx{[] {
    const char *e = std::getenv("ECX_ROCTX");
    return e && e[0] == '1' ? 1 : 0;
}()};

struct Range {
    const Roctx *lib = nullptr;
    explicit Range(const char *name) {
        if (g_roctx.load(std::memory_order_relaxed) && roctx_lib().push) {
            lib = &roctx_lib();
            lib->push(name);
        }
    }
    ~Range() {
        if (lib) lib->pop();
    }
};

template <class F>
int guarded(const char *name, F &&f) {
    Range range(name);
    try {
        return f();
    } catch (const Error &e) {
        g_last_error = e.what();
        return e.code;
    } catch (const std::bad_alloc &) {
        g_last_error = "out of memory";
        return ECX_E_NOMEM;
    } catch (const std::exception &e) {
        g_last_error = e.what();
        return ECX_E_ILLEGAL_ARGUMENT;
    }
}

std::string key_of(const std::vector<bool> &v, int extra = 0) {
    std::string s(v.size() + 8, '\0');
    for (size_t i = 0; i < v.size(); ++i) s[i] = v[i] ? '1' : '0';
    std::memcpy(&s[v.size()], &extra, sizeof(int));
    return s;
}

// ReedSolomon.checkBuffersAndSizes, ReedSolomon.java:338-363.
void check_buffers(const RsCode &c, uint8_t *const *shards, int shard_count, int shard_length, int offset,
                   int byte_count) {
    if (shard_count != c.n()) throw Error(ECX_E_ILLEGAL_ARGUMENT, "wrong number of shards: " + std::to_string(shard_count));
    if (!shards) throw Error(ECX_E_NULL, "shards is null");
    for (int i = 0; i < shard_count; ++i)
        if (!shards[i]) throw Error(ECX_E_NULL, "shard " + std::to_string(i) + " is null");
    if (offset < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "offset is negative: " + std::to_string(offset));
    if (byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "byteCount is negative: " + std::to_string(byte_count));
    if ((long long)shard_length < (long long)offset + byte_count)
        throw Error(ECX_E_ILLEGAL_ARGUMENT, "buffers to small: " + std::to_string(byte_count) + std::to_string(offset));
}

LinearMap dense_map(const uint8_t *m, int n_out, int n_in) {
    LinearMap lm;
    lm.n_out = n_out;
    lm.n_in = n_in;
    lm.a.assign(m, m + (size_t)n_out * n_in);
    for (int j = 0; j < n_in; ++j) lm.in_slot.push_back(j);
    for (int o = 0; o < n_out; ++o) lm.out_slot.push_back(o);
    return lm;
}

// The CodingLoop entry points receive their matrix with every call: the reference
// passes the codec's parity rows or decode rows each time (ReedSolomon.java:105-107,
// :262-264).  Compiling a plan costs the planner, a device upload and, when the plan
// is dropped, a hipFree that synchronises the device, so plans are cached by the
// map's content (least recently used first out; ecx_tune "plan_cache" sets the size,
// 0 compiles every call).
std::shared_ptr<CompiledMap> cached_plan(LinearMap lm) {
    const size_t cap = (size_t)tuning().plan_cache;
    if (cap == 0) return std::make_shared<CompiledMap>(std::move(lm));
    std::string key(sizeof(int) * (2 + lm.in_slot.size() + lm.out_slot.size()) + lm.a.size(), '\0');
    char *k = &key[0];
    std::memcpy(k, &lm.n_out, sizeof(int));
    std::memcpy(k + sizeof(int), &lm.n_in, sizeof(int));
    k += 2 * sizeof(int);
    std::memcpy(k, lm.in_slot.data(), lm.in_slot.size() * sizeof(int));
    k += lm.in_slot.size() * sizeof(int);
    std::memcpy(k, lm.out_slot.data(), lm.out_slot.size() * sizeof(int));
    k += lm.out_slot.size() * sizeof(int);
    std::memcpy(k, lm.a.data(), lm.a.size());
    using Entry = std::pair<std::string, std::shared_ptr<CompiledMap>>;
    static std::mutex mu;
    static std::list<Entry> lru;  // front = most recently used
    static std::unordered_map<std::string, std::list<Entry>::iterator> index;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = index.find(key);
        if (it != index.end()) {
            lru.splice(lru.begin(), lru, it->second);
            return it->second->second;
        }
    }
    auto plan = std::make_shared<CompiledMap>(std::move(lm));  // compiled outside the lock
    std::lock_guard<std::mutex> lk(mu);
    auto it = index.find(key);
    if (it != index.end()) return it->second->second;  // another thread compiled it first
    lru.emplace_front(key, plan);
    index[key] = lru.begin();
    while (lru.size() > cap) {
        index.erase(lru.back().first);
        lru.pop_back();  // the plan is freed when its last in-flight user drops it
    }
    return plan;
}

std::vector<bool> present_vec(const uint8_t *p, int n) {
    std::vector<bool> v(n);
    for (int i = 0; i < n; ++i) v[i] = p[i] != 0;
    return v;
}

ecx_map *rs_decode_map(ecx_rs *rs, const std::vector<bool> &present) {
    std::lock_guard<std::mutex> lk(rs->mu);
    auto &slot = rs->dec[key_of(present)];
    if (!slot) slot = std::make_unique<ecx_map>(rs->code.decode_map(present));
    return slot.get();
}

// isParityCorrect's map (ReedSolomon.java:129-178): row p = parityRows[p] over the data
// shards plus 1 x parity shard p, i.e. the syndrome, all zero exactly when the parity is right.
ecx_map *rs_check_map(ecx_rs *rs) {
    const RsCode &c = rs->code;
    std::lock_guard<std::mutex> lk(rs->mu);
    if (!rs->check) {
        LinearMap lm;
        lm.n_out = c.m();
        lm.n_in = c.n();
        lm.a.assign((size_t)c.m() * c.n(), 0);
        for (int p = 0; p < c.m(); ++p) {
            std::memcpy(&lm.a[(size_t)p * c.n()], c.parity_row(p), (size_t)c.k());
            lm.a[(size_t)p * c.n() + c.k() + p] = 1;
            lm.out_slot.push_back(p);
        }
        for (int j = 0; j < c.n(); ++j) lm.in_slot.push_back(j);
        rs->check = std::make_unique<ecx_map>(lm.pruned());
    }
    return rs->check.get();
}

ecx_map *clay_standard_map(ecx_clay *c) {
    const int n = c->pl.n_real(), a = c->pl.alpha();
    std::vector<bool> present((size_t)n * a, true);
    for (int z = 0; z < a; ++z)
        for (int e : c->pl.erased())
            if (e >= 0 && e < n) present[(size_t)z * n + e] = false;
    std::lock_guard<std::mutex> lk(c->mu);
    auto &slot = c->maps[key_of(present, -1)];
    if (!slot) slot = std::make_unique<ecx_map>(c->pl.perform_coding_map(present));
    return slot.get();
}

}  // namespace

namespace {
// Process-wide codec registry: equal codecs are one reference-counted object.
// ecx_*_create takes a reference, ecx_*_destroy drops it.  A codec nobody references
// stays registered, idle, so that the next create of the same codec (the reference builds
// one per file or repair) finds its compiled plans and generated kernels; at most
// kCodecIdleMax idle codecs are kept, least recently released first out, and an evicted
// codec frees its device state.  Past kCodecRegistryMax registered codecs, creates return
// private objects that destroy frees at once.
constexpr size_t kCodecRegistryMax = 4096;
constexpr size_t kCodecIdleMax = 64;

template <typename T, typename Key>
struct Registry {
    std::mutex mu;
    std::map<Key, std::unique_ptr<T>> reg;
    std::map<const T *, Key> key_of;
    std::list<const T *> idle;  // front = most recently released
    std::map<const T *, typename std::list<const T *>::iterator> idle_pos;
    std::map<const T *, int> refs;
    std::map<const T *, std::unique_ptr<T>> priv;  // private objects (registry full): freed by destroy

    template <typename Make>
    T *get(const Key &key, Make make) {
        std::lock_guard<std::mutex> lk(mu);
        auto it = reg.find(key);
        if (it != reg.end()) {
            T *obj = it->second.get();
            auto ip = idle_pos.find(obj);
            if (ip != idle_pos.end()) {
                idle.erase(ip->second);
                idle_pos.erase(ip);
            }
            ++refs[obj];
            return obj;
        }
        std::unique_ptr<T> obj(make());  // may throw (invalid geometry): nothing registered
        if (reg.size() >= kCodecRegistryMax) {
            T *p = obj.get();
            priv.emplace(p, std::move(obj));
            return p;
        }
        obj->shared = true;
        T *p = obj.get();
        reg.emplace(key, std::move(obj));
        key_of.emplace(p, key);
        refs[p] = 1;
        return p;
    }

    // Drops one reference; frees a private object, parks a shared one as idle.  A pointer
    // the registry does not hold a live reference for (a second destroy) is ignored, never
    // dereferenced.
    void release(T *obj) {
        if (!obj) return;
        std::vector<std::unique_ptr<T>> evicted;  // destroyed outside the lock (hipFree syncs)
        {
            std::lock_guard<std::mutex> lk(mu);
            auto pv = priv.find(obj);
            if (pv != priv.end()) {
                evicted.push_back(std::move(pv->second));
                priv.erase(pv);
                return;
            }
            auto r = refs.find(obj);
            if (r == refs.end() || r->second <= 0) return;  // not a live reference: ignore
            if (--r->second > 0) return;
            idle.push_front(obj);
            idle_pos[obj] = idle.begin();
            while (idle.size() > kCodecIdleMax) {
                const T *victim = idle.back();
                idle.pop_back();
                idle_pos.erase(victim);
                refs.erase(victim);
                auto k = key_of.find(victim);
                auto e = reg.find(k->second);
                evicted.push_back(std::move(e->second));
                reg.erase(e);
                key_of.erase(k);
            }
        }
    }

    void stats(int *live, int *idle_n) {
        std::lock_guard<std::mutex> lk(mu);
        if (live) *live = (int)(reg.size() - idle.size());
        if (idle_n) *idle_n = (int)idle.size();
    }
};

Registry<ecx_rs, std::pair<int, int>> &rs_registry() {
    static Registry<ecx_rs, std::pair<int, int>> r;
    return r;
}
Registry<ecx_clay, std::tuple<int, int, int, std::vector<int>, int>> &clay_registry() {
    static Registry<ecx_clay, std::tuple<int, int, int, std::vector<int>, int>> r;
    return r;
}
}  // namespace

extern "C" {

const char *ecx_status_string(int s) {
    switch (s) {
    case ECX_OK: return "ok";
    case ECX_E_ILLEGAL_ARGUMENT: return "IllegalArgumentException";
    case ECX_E_NOT_ENOUGH_SHARDS: return "Not enough shards present";
    case ECX_E_SINGULAR: return "Matrix is singular";
    case ECX_E_TOO_MANY_SHARDS: return "too many shards - max is 256";
    case ECX_E_INDEX: return "ArrayIndexOutOfBoundsException";
    case ECX_E_NULL: return "NullPointerException";
    case ECX_E_NOMEM: return "out of memory";
    case ECX_E_DEVICE: return "HIP device error";
    default: return "unknown status";
    }
}

const char *ecx_last_error(void) { return g_last_error.c_str(); }
int ecx_version(void) { return 106; }  // 1.06: round-5 ABI (check batches device and host, multi-GPU host batches, per-call executor)

// ---------------------------------------------------------------- device
int ecx_device_count(int *count) {
    return guarded(__func__, [&]() -> int {
        int n = 0;
        check_hip(hipGetDeviceCount(&n), "hipGetDeviceCount");
        *count = n;
        return ECX_OK;
    });
}

int ecx_set_device(int device) {
    return guarded(__func__, [&]() -> int {
        check_hip(hipSetDevice(device), "hipSetDevice");
        return ECX_OK;
    });
}

int ecx_synchronize(void *stream) {
    return guarded(__func__, [&]() -> int {
        check_hip(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
        return ECX_OK;
    });
}

// ---------------------------------------------------------------- Galois / Matrix
int ecx_gf_multiply(int a, int b) { return Field::get().mul((uint8_t)a, (uint8_t)b); }

int ecx_gf_divide(int a, int b) {
    return guarded(__func__, [&]() -> int { return (int)Field::get().div((uint8_t)a, (uint8_t)b); });
}

int ecx_gf_exp(int a, int n) {
    return guarded(__func__, [&]() -> int {
        if (n < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative exponent");
        return (int)Field::get().pow((uint8_t)a, n);
    });
}

int ecx_gf_tables(int16_t *log_table, uint8_t *exp_table, uint8_t *mul_table) {
    const Field &f = Field::get();
    if (log_table)
        for (int i = 0; i < 256; ++i) log_table[i] = f.log((uint8_t)i);
    if (exp_table)
        for (int i = 0; i < 510; ++i) exp_table[i] = f.exp(i);
    if (mul_table)
        for (int a = 0; a < 256; ++a) std::memcpy(mul_table + 256 * a, f.row((uint8_t)a), 256);
    return ECX_OK;
}

int ecx_matrix_times(const uint8_t *a, int ar, int ac, const uint8_t *b, int br, int bc, uint8_t *out) {
    return guarded(__func__, [&]() -> int {
        Matrix A(ar, ac), B(br, bc);
        std::memcpy(A.row(0), a, (size_t)ar * ac);
        std::memcpy(B.row(0), b, (size_t)br * bc);
        Matrix C = A * B;
        std::memcpy(out, C.row(0), (size_t)ar * bc);
        return ECX_OK;
    });
}

int ecx_matrix_invert(const uint8_t *m, int n, uint8_t *out) {
    return guarded(__func__, [&]() -> int {
        Matrix A(n, n);
        std::memcpy(A.row(0), m, (size_t)n * n);
        Matrix I = A.inverse();
        std::memcpy(out, I.row(0), (size_t)n * n);
        return ECX_OK;
    });
}

// ---------------------------------------------------------------- CodingLoop
int ecx_code_some_shards(const uint8_t *matrix_rows, const uint8_t *const *inputs, int input_count,
                         uint8_t *const *outputs, int output_count, int offset, int byte_count) {
    return guarded(__func__, [&]() -> int {
        if (input_count <= 0 || output_count < 0 || offset < 0 || byte_count < 0)
            throw Error(ECX_E_ILLEGAL_ARGUMENT, "invalid counts");
        const std::shared_ptr<CompiledMap> cm = cached_plan(dense_map(matrix_rows, output_count, input_count).pruned());
        run_host(*cm, inputs, outputs, offset, byte_count);
        // Rows with every coefficient zero have no entries but are still written (as zeros) by the kernel.
        return ECX_OK;
    });
}

int ecx_check_some_shards(const uint8_t *matrix_rows, const uint8_t *const *inputs, int input_count,
                          const uint8_t *const *to_check, int check_count, int offset, int byte_count,
                          uint8_t *temp_buffer) {
    (void)temp_buffer;
    return guarded(__func__, [&]() -> int {
        if (input_count <= 0 || check_count < 0 || offset < 0 || byte_count < 0)
            throw Error(ECX_E_ILLEGAL_ARGUMENT, "invalid counts");
        // row o: sum_i M[o][i]*in[i] + 1*to_check[o] == 0  <=>  to_check[o] is correct
        const int w = input_count + check_count;
        LinearMap lm;
        lm.n_out = check_count;
        lm.n_in = w;
        lm.a.assign((size_t)check_count * w, 0);
        for (int o = 0; o < check_count; ++o) {
            std::memcpy(&lm.a[(size_t)o * w], matrix_rows + (size_t)o * input_count, (size_t)input_count);
            lm.a[(size_t)o * w + input_count + o] = 1;
            lm.out_slot.push_back(o);
        }
        for (int j = 0; j < w; ++j) lm.in_slot.push_back(j);
        std::vector<const uint8_t *> ptrs(inputs, inputs + input_count);
        ptrs.insert(ptrs.end(), to_check, to_check + check_count);
        const std::shared_ptr<CompiledMap> cm = cached_plan(lm.pruned());
        return run_host_all_zero(*cm, ptrs.data(), offset, byte_count) ? 1 : 0;
    });
}

int ecx_code_single(const uint8_t *matrix_rows, int row_length, const uint8_t *input, int index, uint8_t *output,
                    int output_index, int offset, int byte_count, int is_first_time) {
    return guarded(__func__, [&]() -> int {
        if (index < 0 || index >= row_length || output_index < 0) throw Error(ECX_E_INDEX, "matrix index");
        if (offset < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "invalid counts");
        const uint8_t c = matrix_rows[(size_t)output_index * row_length + index];
        if (host_exec_wanted(byte_count)) {  // below the per-call crossover: no plan, no device round trip
            if (!input || !output) throw Error(ECX_E_NULL, "null buffer");
            host_exec_scale(c, input + offset, output + offset, byte_count, !is_first_time);
            return ECX_OK;
        }
        const uint8_t row[2] = {c, (uint8_t)(is_first_time ? 0 : 1)};
        const std::shared_ptr<CompiledMap> cm = cached_plan(dense_map(row, 1, 2));
        const uint8_t *ins[2] = {input, output};
        uint8_t *outs[1] = {output};
        run_host(*cm, ins, outs, offset, byte_count);
        return ECX_OK;
    });
}

// ---------------------------------------------------------------- ReedSolomon
// Codec objects are immutable after creation apart from their lock-protected plan caches,
// so equal codecs are one object: the reference builds a ReedSolomon (or a Clay decoding
// step) per file or repair (SampleEncoder.java:83, ClayCode.java:43-51), and sharing keeps
// the compiled, device-resident plans -- and the hiprtc-compiled Clay kernels -- of every
// earlier call instead of rebuilding them per object.  Shared codecs are reference-
// counted; up to kCodecIdleMax unreferenced ones stay cached (Registry above).
int ecx_rs_create(int data_shards, int parity_shards, ecx_rs **out) {
    return guarded(__func__, [&]() -> int {
        *out = nullptr;
        *out = rs_registry().get(std::make_pair(data_shards, parity_shards),
                                 [&] { return new ecx_rs(data_shards, parity_shards); });
        return ECX_OK;
    });
}

void ecx_rs_destroy(ecx_rs *rs) { rs_registry().release(rs); }

int ecx_rs_matrix(const ecx_rs *rs, uint8_t *out) {
    const Matrix &m = rs->code.matrix();
    std::memcpy(out, m.row(0), (size_t)m.rows() * m.cols());
    return ECX_OK;
}

int ecx_rs_shape(const ecx_rs *rs, int *data_shards, int *parity_shards) {
    if (!rs) return ECX_E_NULL;
    if (data_shards) *data_shards = rs->code.k();
    if (parity_shards) *parity_shards = rs->code.m();
    return ECX_OK;
}

int ecx_rs_encode_map(ecx_rs *rs, const ecx_map **out) {
    return guarded(__func__, [&]() -> int {
        std::lock_guard<std::mutex> lk(rs->mu);
        if (!rs->enc) rs->enc = std::make_unique<ecx_map>(rs->code.encode_map());
        *out = rs->enc.get();
        return ECX_OK;
    });
}

int ecx_rs_decode_map(ecx_rs *rs, const uint8_t *shard_present, const ecx_map **out) {
    return guarded(__func__, [&]() -> int {
        std::vector<bool> present = present_vec(shard_present, rs->code.n());
        int np = 0;
        for (bool b : present) np += b;
        if (np < rs->code.k()) throw Error(ECX_E_NOT_ENOUGH_SHARDS, "Not enough shards present");
        *out = rs_decode_map(rs, present);
        return ECX_OK;
    });
}

int ecx_rs_encode_parity_batch(ecx_rs *rs, uint8_t *base, int64_t stripe_stride, int64_t shard_stride,
                               int64_t nstripes, int64_t offset, int64_t byte_count, void *stream) {
    return guarded(__func__, [&]() -> int {
        if (nstripes < 0 || offset < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (!base) throw Error(ECX_E_NULL, "null device pointer");
        const ecx_map *m = nullptr;
        const int st = ecx_rs_encode_map(rs, &m);
        if (st) return st;
        launch_apply(const_cast<ecx_map *>(m)->cm, base + offset, stripe_stride, shard_stride, base + offset,
                     stripe_stride, shard_stride, nstripes, byte_count, (hipStream_t)stream);
        return ECX_OK;
    });
}

int ecx_rs_decode_missing_batch(ecx_rs *rs, const uint8_t *shard_present, uint8_t *base, int64_t stripe_stride,
                                int64_t shard_stride, int64_t nstripes, int64_t offset, int64_t byte_count,
                                void *stream) {
    return guarded(__func__, [&]() -> int {
        if (nstripes < 0 || offset < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (!base) throw Error(ECX_E_NULL, "null device pointer");
        const ecx_map *m = nullptr;
        const int st = ecx_rs_decode_map(rs, shard_present, &m);  // Not enough shards -> -2
        if (st) return st;
        if (m->cm.map().n_out == 0) return ECX_OK;  // all present (ReedSolomon.java:216-218)
        launch_apply(const_cast<ecx_map *>(m)->cm, base + offset, stripe_stride, shard_stride, base + offset,
                     stripe_stride, shard_stride, nstripes, byte_count, (hipStream_t)stream);
        return ECX_OK;
    });
}

namespace {
// The plain layout's pitch (scripts/rs_layout_contract.py): the smallest
// ODD multiple of 4 KiB at or above the shard.  4 KiB-aligned shards run full-chunk kernels only,
// and an odd count keeps the streams off the power-of-two boundaries whose address bits the HBM
// interleave does not spread (section 4, "Where the streams collide": 4 MiB + 4 KiB, not 4 MiB).
int64_t recommended_pitch(int64_t byte_count) {
    constexpr int64_t kStep = 4 << 10;
    int64_t c = (byte_count + kStep - 1) / kStep;
    if (c % 2 == 0 && c > 0) ++c;
    return c * kStep;
}

// The blocked layout's block: the largest power of two with n blocks
// (one per shard of a stripe) within 1 MiB, 4 KiB..1 MiB -- 32 KiB for RS(17,3) (0.76 of HBM),
// 64 KiB for RS(12,4) (0.816); one block of byte_count bytes for smaller shards.
int64_t recommended_block(int n, int64_t byte_count) {
    int64_t b = 1 << 20;
    while (b > (4 << 10) && b * n > (1 << 20)) b >>= 1;
    return byte_count >= b ? b : byte_count;
}

int64_t resolve_block(int n, int64_t byte_count, int64_t block_bytes) {
    if (block_bytes < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative block size");
    return block_bytes == 0 ? recommended_block(n, byte_count) : block_bytes;
}

// The two passes of a blocked batch (ecx.h), each in place: the full blocks as nstripes * full
// "stripes" of n block-sized slots, then the tails as nstripes stripes of n tail-sized slots.
// pass(offset, stripe_stride, slot_bytes, units) runs the map over one of them.
// (a std::function: this file's helpers sit inside the extern "C" block, where templates cannot)
void blocked_passes(int n, int64_t nstripes, int64_t byte_count, int64_t block,
                    const std::function<void(int64_t, int64_t, int64_t, int64_t)> &pass) {
    if (nstripes == 0 || byte_count == 0) return;
    const int64_t full = byte_count / block, tail = byte_count % block;
    int64_t stride = 0, units = 0, body = 0;
    if (__builtin_mul_overflow((int64_t)n, block, &stride) || __builtin_mul_overflow(nstripes, full, &units) ||
        __builtin_mul_overflow(units, stride, &body))
        throw Error(ECX_E_ILLEGAL_ARGUMENT, "blocked batch extent overflows");
    if (full > 0) pass((int64_t)0, stride, block, units);
    if (tail > 0) pass(body, (int64_t)n * tail, tail, nstripes);
}

void launch_blocked(CompiledMap &cm, uint8_t *base, int n, int64_t nstripes, int64_t byte_count, int64_t block,
                    hipStream_t stream) {
    blocked_passes(n, nstripes, byte_count, block, [&](int64_t off, int64_t ss, int64_t len, int64_t units) {
        launch_apply(cm, base + off, ss, len, base + off, ss, len, units, len, stream);
    });
}

// The same two passes from host memory: two pipelined host batches (host_pipe.cpp), the second
// after the first has drained (each is synchronous).  With a device list (ndev > 0) each pass is
// split over the entries like any host batch: the full blocks as nstripes * full small stripes,
// the tails by stripes (by byte ranges where there are fewer stripes than entries).
void host_blocked(CompiledMap &cm, uint8_t *base, int n, int64_t nstripes, int64_t byte_count, int64_t block,
                  const int *devices = nullptr, int ndev = 0) {
    const bool multi = ndev != 0 || devices;
    if (multi) for_device_ranges(devices, ndev, 0, [](int64_t, int64_t) {});  // the list, even for an empty batch
    blocked_passes(n, nstripes, byte_count, block, [&](int64_t off, int64_t ss, int64_t len, int64_t units) {
        if (multi) run_host_batch_devices(cm, base + off, ss, len, base + off, ss, len, units, len, devices, ndev);
        else run_host_batch(cm, base + off, ss, len, base + off, ss, len, units, len);
    });
}
}  // namespace

int ecx_rs_blocked_layout(int data_shards, int parity_shards, int64_t byte_count, int64_t *layout) {
    return guarded(__func__, [&]() -> int {
        if (!layout) throw Error(ECX_E_NULL, "null layout");
        if (byte_count < 0 || data_shards <= 0 || parity_shards <= 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "bad shape");
        if (data_shards + parity_shards > 256) throw Error(ECX_E_TOO_MANY_SHARDS, "too many shards - max is 256");
        const int64_t b = recommended_block(data_shards + parity_shards, byte_count);
        layout[0] = b;
        layout[1] = b ? byte_count / b : 0;
        layout[2] = b ? byte_count % b : 0;
        return ECX_OK;
    });
}

int ecx_rs_recommended_pitch(int data_shards, int parity_shards, int64_t byte_count, int64_t *pitch) {
    return guarded(__func__, [&]() -> int {
        if (!pitch) throw Error(ECX_E_NULL, "null pitch");
        if (byte_count < 0 || data_shards <= 0 || parity_shards <= 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "bad shape");
        if (data_shards + parity_shards > 256) throw Error(ECX_E_TOO_MANY_SHARDS, "too many shards - max is 256");
        *pitch = recommended_pitch(byte_count);
        return ECX_OK;
    });
}

int ecx_rs_encode_parity_blocked_batch(ecx_rs *rs, uint8_t *base, int64_t nstripes, int64_t byte_count,
                                       int64_t block_bytes, void *stream) {
    return guarded(__func__, [&]() -> int {
        if (nstripes < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (!base) throw Error(ECX_E_NULL, "null device pointer");
        const ecx_map *m = nullptr;
        const int st = ecx_rs_encode_map(rs, &m);
        if (st) return st;
        const int64_t block = resolve_block(rs->code.n(), byte_count, block_bytes);
        launch_blocked(const_cast<ecx_map *>(m)->cm, base, rs->code.n(), nstripes, byte_count, block,
                       (hipStream_t)stream);
        return ECX_OK;
    });
}

int ecx_rs_decode_missing_blocked_batch(ecx_rs *rs, const uint8_t *shard_present, uint8_t *base, int64_t nstripes,
                                        int64_t byte_count, int64_t block_bytes, void *stream) {
    return guarded(__func__, [&]() -> int {
        if (nstripes < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (!base) throw Error(ECX_E_NULL, "null device pointer");
        const ecx_map *m = nullptr;
        const int st = ecx_rs_decode_map(rs, shard_present, &m);  // Not enough shards -> -2
        if (st) return st;
        const int64_t block = resolve_block(rs->code.n(), byte_count, block_bytes);
        if (m->cm.map().n_out == 0) return ECX_OK;  // all present (ReedSolomon.java:216-218)
        launch_blocked(const_cast<ecx_map *>(m)->cm, base, rs->code.n(), nstripes, byte_count, block,
                       (hipStream_t)stream);
        return ECX_OK;
    });
}

int ecx_rs_encode_parity_blocked_batch_host(ecx_rs *rs, uint8_t *base, int64_t nstripes, int64_t byte_count,
                                            int64_t block_bytes) {
    return guarded(__func__, [&]() -> int {
        if (!rs) throw Error(ECX_E_NULL, "null codec");
        if (nstripes < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (nstripes > 0 && !base) throw Error(ECX_E_NULL, "null host pointer");
        const ecx_map *m = nullptr;
        const int st = ecx_rs_encode_map(rs, &m);
        if (st) return st;
        const int64_t block = resolve_block(rs->code.n(), byte_count, block_bytes);
        host_blocked(const_cast<ecx_map *>(m)->cm, base, rs->code.n(), nstripes, byte_count, block);
        return ECX_OK;
    });
}

int ecx_rs_decode_missing_blocked_batch_host(ecx_rs *rs, const uint8_t *shard_present, uint8_t *base,
                                             int64_t nstripes, int64_t byte_count, int64_t block_bytes) {
    return guarded(__func__, [&]() -> int {
        if (!rs) throw Error(ECX_E_NULL, "null codec");
        if (nstripes < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (nstripes > 0 && !base) throw Error(ECX_E_NULL, "null host pointer");
        const ecx_map *m = nullptr;
        const int st = ecx_rs_decode_map(rs, shard_present, &m);  // Not enough shards -> -2
        if (st) return st;
        const int64_t block = resolve_block(rs->code.n(), byte_count, block_bytes);
        if (m->cm.map().n_out == 0) return ECX_OK;  // all present (ReedSolomon.java:216-218)
        host_blocked(const_cast<ecx_map *>(m)->cm, base, rs->code.n(), nstripes, byte_count, block);
        return ECX_OK;
    });
}

int ecx_rs_encode_parity_blocked_batch_host_devices(ecx_rs *rs, uint8_t *base, int64_t nstripes, int64_t byte_count,
                                                    int64_t block_bytes, const int *devices, int ndev) {
    return guarded(__func__, [&]() -> int {
        if (!rs) throw Error(ECX_E_NULL, "null codec");
        if (!devices) throw Error(ECX_E_NULL, "null device list");
        if (ndev <= 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "empty device list");
        if (nstripes < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (nstripes > 0 && !base) throw Error(ECX_E_NULL, "null host pointer");
        const ecx_map *m = nullptr;
        const int st = ecx_rs_encode_map(rs, &m);
        if (st) return st;
        const int64_t block = resolve_block(rs->code.n(), byte_count, block_bytes);
        host_blocked(const_cast<ecx_map *>(m)->cm, base, rs->code.n(), nstripes, byte_count, block, devices, ndev);
        return ECX_OK;
    });
}

int ecx_rs_decode_missing_blocked_batch_host_devices(ecx_rs *rs, const uint8_t *shard_present, uint8_t *base,
                                                     int64_t nstripes, int64_t byte_count, int64_t block_bytes,
                                                     const int *devices, int ndev) {
    return guarded(__func__, [&]() -> int {
        if (!rs) throw Error(ECX_E_NULL, "null codec");
        if (!devices) throw Error(ECX_E_NULL, "null device list");
        if (ndev <= 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "empty device list");
        if (nstripes < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (nstripes > 0 && !base) throw Error(ECX_E_NULL, "null host pointer");
        const ecx_map *m = nullptr;
        const int st = ecx_rs_decode_map(rs, shard_present, &m);  // Not enough shards -> -2
        if (st) return st;
        const int64_t block = resolve_block(rs->code.n(), byte_count, block_bytes);
        // all present (ReedSolomon.java:216-218): nothing to touch, the device list still checked
        host_blocked(const_cast<ecx_map *>(m)->cm, base, rs->code.n(), m->cm.map().n_out == 0 ? 0 : nstripes,
                     byte_count, block, devices, ndev);
        return ECX_OK;
    });
}

int ecx_rs_encode_parity(ecx_rs *rs, uint8_t *const *shards, int shard_count, int shard_length, int offset,
                         int byte_count) {
    return guarded(__func__, [&]() -> int {
        check_buffers(rs->code, shards, shard_count, shard_length, offset, byte_count);
        const ecx_map *m = nullptr;
        int st = ecx_rs_encode_map(rs, &m);
        if (st) return st;
        run_host(const_cast<ecx_map *>(m)->cm, shards, shards, offset, byte_count);
        return ECX_OK;
    });
}

int ecx_rs_encode_parity_single(ecx_rs *rs, const uint8_t *shard, uint8_t *output, int input_index,
                                int output_index, int offset, int byte_count) {
    return guarded(__func__, [&]() -> int {
        const RsCode &c = rs->code;
        if (output_index < 0 || output_index >= c.m() || input_index < 0 || input_index >= c.k())
            throw Error(ECX_E_INDEX, "parity row / column index");
        if (offset < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "invalid counts");
        if (host_exec_wanted(byte_count)) {  // below the per-call crossover: no plan, no device round trip
            if (!shard || !output) throw Error(ECX_E_NULL, "null buffer");
            host_exec_scale(c.parity_row(output_index)[input_index], shard + offset, output + offset, byte_count, true);
            return ECX_OK;
        }
        const uint8_t row[2] = {c.parity_row(output_index)[input_index], 1};
        const std::shared_ptr<CompiledMap> cm = cached_plan(dense_map(row, 1, 2));
        const uint8_t *ins[2] = {shard, output};
        uint8_t *outs[1] = {output};
        run_host(*cm, ins, outs, offset, byte_count);
        return ECX_OK;
    });
}

int ecx_rs_is_parity_correct(ecx_rs *rs, uint8_t *const *shards, int shard_count, int shard_length, int first_byte,
                             int byte_count, uint8_t *temp_buffer, int temp_length) {
    return guarded(__func__, [&]() -> int {
        check_buffers(rs->code, shards, shard_count, shard_length, first_byte, byte_count);
        if (temp_buffer && (long long)temp_length < (long long)first_byte + byte_count)
            throw Error(ECX_E_ILLEGAL_ARGUMENT, "tempBuffer is not big enough");
        return run_host_all_zero(rs_check_map(rs)->cm, shards, first_byte, byte_count) ? 1 : 0;
    });
}

int ecx_rs_is_parity_correct_batch(ecx_rs *rs, const uint8_t *base, int64_t stripe_stride, int64_t shard_stride,
                                   int64_t nstripes, int64_t offset, int64_t byte_count, uint8_t *verdict,
                                   void *stream) {
    return guarded(__func__, [&]() -> int {
        if (!rs) throw Error(ECX_E_NULL, "null codec");
        if (nstripes < 0 || offset < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (nstripes == 0) return ECX_OK;
        if (!base || !verdict) throw Error(ECX_E_NULL, "null device pointer");
        launch_check(rs_check_map(rs)->cm, base + offset, stripe_stride, shard_stride, verdict, nstripes, byte_count,
                     (hipStream_t)stream);
        return ECX_OK;
    });
}

int ecx_rs_decode_missing(ecx_rs *rs, uint8_t *const *shards, const uint8_t *shard_present, int shard_count,
                          int shard_length, int offset, int byte_count) {
    return guarded(__func__, [&]() -> int {
        check_buffers(rs->code, shards, shard_count, shard_length, offset, byte_count);
        std::vector<bool> present = present_vec(shard_present, rs->code.n());
        int np = 0;
        for (bool b : present) np += b;
        if (np == rs->code.n()) return ECX_OK;
        if (np < rs->code.k()) throw Error(ECX_E_NOT_ENOUGH_SHARDS, "Not enough shards present");
        ecx_map *m = rs_decode_map(rs, present);
        run_host(m->cm, shards, shards, offset, byte_count);
        return ECX_OK;
    });
}

int ecx_rs_decode_missing_single(ecx_rs *rs, const uint8_t *shard, int shard_index, int index,
                                 const uint8_t *shard_present, uint8_t *const *outputs, int output_count, int offset,
                                 int byte_count, int is_first) {
    (void)shard_index;
    return guarded(__func__, [&]() -> int {
        const RsCode &c = rs->code;
        std::vector<bool> present = present_vec(shard_present, c.n());
        int np = 0;
        for (bool b : present) np += b;
        // fewer than k present leaves zero rows in the sub-matrix: "Matrix is singular"
        if (np < c.k()) throw Error(ECX_E_SINGULAR, "Matrix is singular");
        const Matrix dec = c.data_decoder(present, nullptr);
        std::vector<int> missing;
        for (int i = 0; i < c.k(); ++i)
            if (!present[i]) missing.push_back(i);
        if (output_count > c.m() || (int)missing.size() > c.m()) throw Error(ECX_E_INDEX, "matrixRows index");
        if (output_count > (int)missing.size()) throw Error(ECX_E_NULL, "no decode row for this output (no missing data shard)");
        if (index < 0 || index >= c.k()) throw Error(ECX_E_INDEX, "matrix column index");
        if (offset < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "invalid counts");
        if (output_count == 0) return ECX_OK;
        // row j: out_j (=|^=) D^-1[missing_j][index] * shard
        const int w = 1 + output_count;
        LinearMap lm;
        lm.n_out = output_count;
        lm.n_in = w;
        lm.a.assign((size_t)output_count * w, 0);
        for (int j = 0; j < output_count; ++j) {
            lm.a[(size_t)j * w] = dec.at(missing[j], index);
            if (!is_first) lm.a[(size_t)j * w + 1 + j] = 1;
            lm.out_slot.push_back(j);
        }
        for (int j = 0; j < w; ++j) lm.in_slot.push_back(j);
        std::vector<const uint8_t *> ins(1, shard);
        ins.insert(ins.end(), outputs, outputs + output_count);
        const std::shared_ptr<CompiledMap> cm = cached_plan(lm.pruned());
        run_host(*cm, ins.data(), outputs, offset, byte_count);
        return ECX_OK;
    });
}

// ---------------------------------------------------------------- maps
int ecx_map_create(const uint8_t *matrix, int n_out, int n_in, const int *in_slot, const int *out_slot,
                   ecx_map **out) {
    return guarded(__func__, [&]() -> int {
        *out = nullptr;
        if (n_out < 0 || n_in <= 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "map shape");
        LinearMap lm = dense_map(matrix, n_out, n_in);
        if (in_slot) lm.in_slot.assign(in_slot, in_slot + n_in);
        if (out_slot) lm.out_slot.assign(out_slot, out_slot + n_out);
        for (int s : lm.in_slot)
            if (s < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative slot");
        for (int s : lm.out_slot)
            if (s < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative slot");
        *out = new ecx_map(lm.pruned());
        return ECX_OK;
    });
}

void ecx_map_destroy(ecx_map *map) { delete map; }

int ecx_map_info(const ecx_map *map, int *n_out, int *n_in, int *nnz) {
    const LinearMap &m = map->cm.map();
    if (n_out) *n_out = m.n_out;
    if (n_in) *n_in = m.n_in;
    if (nnz) *nnz = m.nnz();
    return ECX_OK;
}

int ecx_map_matrix(const ecx_map *map, uint8_t *matrix, int *in_slot, int *out_slot) {
    const LinearMap &m = map->cm.map();
    if (matrix) std::memcpy(matrix, m.a.data(), m.a.size());
    if (in_slot) std::copy(m.in_slot.begin(), m.in_slot.end(), in_slot);
    if (out_slot) std::copy(m.out_slot.begin(), m.out_slot.end(), out_slot);
    return ECX_OK;
}

int ecx_map_slot_extent(const ecx_map *map, int *max_in_slot, int *max_out_slot) {
    return guarded(__func__, [&]() -> int {
        if (!map) throw Error(ECX_E_NULL, "null map");
        const LinearMap &m = map->cm.map();
        int mi = -1, mo = -1;
        for (int s : m.in_slot) mi = std::max(mi, s);
        for (int s : m.out_slot) mo = std::max(mo, s);
        if (max_in_slot) *max_in_slot = mi;
        if (max_out_slot) *max_out_slot = mo;
        return ECX_OK;
    });
}

int ecx_map_apply_batch(const ecx_map *map, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                        uint8_t *out, int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes,
                        int64_t byte_count, void *stream) {
    return guarded(__func__, [&]() -> int {
        if (nstripes < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (!in || !out) throw Error(ECX_E_NULL, "null device pointer");
        launch_apply(const_cast<ecx_map *>(map)->cm, in, in_stripe_stride, in_slot_stride, out, out_stripe_stride,
                     out_slot_stride, nstripes, byte_count, (hipStream_t)stream);
        return ECX_OK;
    });
}

int ecx_map_accumulate_batch(const ecx_map *map, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                             uint8_t *out, int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes,
                             int64_t byte_count, void *stream) {
    return guarded(__func__, [&]() -> int {
        if (nstripes < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (!in || !out) throw Error(ECX_E_NULL, "null device pointer");
        launch_apply(const_cast<ecx_map *>(map)->cm, in, in_stripe_stride, in_slot_stride, out, out_stripe_stride,
                     out_slot_stride, nstripes, byte_count, (hipStream_t)stream, true);
        return ECX_OK;
    });
}

// ---------------------------------------------------------------- batched partial sums
namespace {
// One-input map: row o = coefficient of `column` in row o of `m` (0 if absent).
ecx_map *single_input_map(const LinearMap &m, int column_slot, std::vector<int> out_slots) {
    LinearMap lm;
    lm.n_in = 1;
    lm.in_slot.push_back(0);
    lm.n_out = m.n_out;
    lm.out_slot = std::move(out_slots);
    int col = -1;
    for (int j = 0; j < m.n_in; ++j)
        if (m.in_slot[j] == column_slot) col = j;
    for (int o = 0; o < m.n_out; ++o) lm.a.push_back(col < 0 ? 0 : m.at(o, col));
    return new ecx_map(lm);
}
}  // namespace

int ecx_rs_decode_partial_batch(ecx_rs *rs, const uint8_t *shard_present, int shard_index, const uint8_t *in,
                                int64_t in_stripe_stride, uint8_t *acc, int64_t acc_stripe_stride,
                                int64_t acc_row_stride, int64_t nstripes, int64_t byte_count, int is_first,
                                void *stream) {
    return guarded(__func__, [&]() -> int {
        const RsCode &c = rs->code;
        if (shard_index < 0 || shard_index >= c.n()) throw Error(ECX_E_INDEX, "shard index");
        std::vector<bool> present = present_vec(shard_present, c.n());
        int np = 0;
        for (bool b : present) np += b;
        if (np < c.k()) throw Error(ECX_E_NOT_ENOUGH_SHARDS, "Not enough shards present");
        if (np == c.n()) return ECX_OK;
        ecx_map *full = rs_decode_map(rs, present);  // rows: the missing shards, data AND parity
        ecx_map *part;
        {
            std::lock_guard<std::mutex> lk(rs->mu);
            auto &slot = rs->partial[key_of(present, shard_index)];
            if (!slot) {
                std::vector<int> rows;
                for (int o = 0; o < full->cm.map().n_out; ++o) rows.push_back(o);
                slot.reset(single_input_map(full->cm.map(), shard_index, rows));
            }
            part = slot.get();
        }
        launch_apply(part->cm, in, in_stripe_stride, 0, acc, acc_stripe_stride, acc_row_stride, nstripes, byte_count,
                     (hipStream_t)stream, !is_first);
        return ECX_OK;
    });
}

int ecx_rs_encode_partial_batch(ecx_rs *rs, int input_index, const uint8_t *in, int64_t in_stripe_stride,
                                uint8_t *acc, int64_t acc_stripe_stride, int64_t acc_row_stride, int64_t nstripes,
                                int64_t byte_count, int is_first, void *stream) {
    return guarded(__func__, [&]() -> int {
        const RsCode &c = rs->code;
        if (input_index < 0 || input_index >= c.k()) throw Error(ECX_E_INDEX, "data shard index");
        ecx_map *part;
        {
            std::lock_guard<std::mutex> lk(rs->mu);
            auto &slot = rs->partial[key_of({}, -1 - input_index)];
            if (!slot) {
                LinearMap lm;
                lm.n_in = 1;
                lm.in_slot.push_back(0);
                lm.n_out = c.m();
                for (int p = 0; p < c.m(); ++p) {
                    lm.a.push_back(c.parity_row(p)[input_index]);
                    lm.out_slot.push_back(p);
                }
                slot = std::make_unique<ecx_map>(lm);
            }
            part = slot.get();
        }
        launch_apply(part->cm, in, in_stripe_stride, 0, acc, acc_stripe_stride, acc_row_stride, nstripes, byte_count,
                     (hipStream_t)stream, !is_first);
        return ECX_OK;
    });
}

// ---------------------------------------------------------------- Clay
int ecx_clay_create(int data_units, int parity_units, const int *erased, int n_erased, ecx_clay **out) {
    return ecx_clay_create_shortened(data_units, parity_units, 0, erased, n_erased, out);
}

int ecx_clay_create_shortened(int data_units, int parity_units, int virtual_units, const int *erased, int n_erased,
                              ecx_clay **out) {
    return ecx_clay_create_ex(data_units, parity_units, virtual_units, erased, n_erased, 0, out);
}

int ecx_clay_create_ex(int data_units, int parity_units, int virtual_units, const int *erased, int n_erased, int flags,
                       ecx_clay **out) {
    return guarded(__func__, [&]() -> int {
        if (!out) throw Error(ECX_E_NULL, "null out");
        *out = nullptr;
        if (n_erased < 0 || virtual_units < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "n_erased / virtual_units");
        if (flags & ~ECX_CLAY_IS_TEST) throw Error(ECX_E_ILLEGAL_ARGUMENT, "unknown Clay flags");
        if (n_erased > 0 && !erased) throw Error(ECX_E_NULL, "null erased list");
        const std::vector<int> e(erased, erased + n_erased);  // order matters (the reference's erasedIndexes)
        const bool is_test = (flags & ECX_CLAY_IS_TEST) != 0;
        *out = clay_registry().get(std::make_tuple(data_units, parity_units, virtual_units, e, flags),
                                   [&] { return new ecx_clay(data_units, parity_units, e, virtual_units, is_test); });
        return ECX_OK;
    });
}

void ecx_clay_destroy(ecx_clay *clay) { clay_registry().release(clay); }

int ecx_codec_stats(int *rs_live, int *rs_idle, int *clay_live, int *clay_idle) {
    rs_registry().stats(rs_live, rs_idle);
    clay_registry().stats(clay_live, clay_idle);
    return ECX_OK;
}

int ecx_clay_geometry(const ecx_clay *clay, int *q, int *t, int *alpha) {
    if (q) *q = clay->pl.q();
    if (t) *t = clay->pl.t();
    if (alpha) *alpha = clay->pl.alpha();
    return ECX_OK;
}

int ecx_clay_shape(const ecx_clay *clay, int *nodes, int *n_erased, int *alpha) {
    if (!clay) return ECX_E_NULL;
    if (nodes) *nodes = clay->pl.n_real();
    if (n_erased) *n_erased = (int)clay->pl.erased().size();
    if (alpha) *alpha = clay->pl.alpha();
    return ECX_OK;
}

int ecx_clay_helper_planes(const ecx_clay *clay, int erased_index, int *out) {
    return guarded(__func__, [&]() -> int {
        std::vector<int> h = clay->pl.helper_planes(erased_index);
        std::copy(h.begin(), h.end(), out);
        return (int)h.size();
    });
}

int ecx_clay_perform_coding(ecx_clay *clay, const uint8_t *const *inputs, uint8_t *const *outputs, int buf_size) {
    return guarded(__func__, [&]() -> int {
        if (clay->pl.erased().empty()) return ECX_OK;
        if (buf_size < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "buf_size");
        const int w = clay->pl.n_real() * clay->pl.alpha();
        std::vector<bool> present(w);
        for (int j = 0; j < w; ++j) present[j] = inputs[j] != nullptr;
        ecx_map *m;
        {
            std::lock_guard<std::mutex> lk(clay->mu);
            auto &slot = clay->maps[key_of(present, -1)];
            if (!slot) slot = std::make_unique<ecx_map>(clay->pl.perform_coding_map(present));
            m = slot.get();
        }
        run_host(m->cm, inputs, outputs, 0, buf_size);
        return ECX_OK;
    });
}

int ecx_clay_decode_single_helper(ecx_clay *clay, const uint8_t *const *helper_coupled, int helper_i,
                                  uint8_t *const *outputs, int erased_index, int buf_size) {
    return guarded(__func__, [&]() -> int {
        if (buf_size < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "buf_size");
        const int nh = (int)clay->pl.helper_planes(erased_index).size();
        const int w = nh * clay->pl.n_real();
        std::vector<bool> present(w);
        for (int j = 0; j < w; ++j) present[j] = helper_coupled[j] != nullptr;
        ecx_map *m;
        {
            std::lock_guard<std::mutex> lk(clay->mu);
            auto &slot = clay->maps[key_of(present, helper_i * 4096 + erased_index)];
            if (!slot) slot = std::make_unique<ecx_map>(clay->pl.decode_single_helper_map(present, helper_i, erased_index, nullptr));
            m = slot.get();
        }
        run_host(m->cm, helper_coupled, outputs, 0, buf_size);
        return ECX_OK;
    });
}

int ecx_clay_map(ecx_clay *clay, const ecx_map **out) {
    return guarded(__func__, [&]() -> int {
        *out = clay_standard_map(clay);
        return ECX_OK;
    });
}

namespace {
// The per-helper-plane repair kernel of a single-erasure step, or nullptr when the
// step's repair has no such program (ClayPlanner::repair_program throws; the reason is
// kept for ecx_clay_rtc_compile_check).
ClayRtc *clay_rtc(ecx_clay *clay) {
    std::lock_guard<std::mutex> lk(clay->mu);
    if (clay->rtc_state == 0) {
        try {
            if (clay->pl.erased().size() != 1) throw Error(ECX_E_ILLEGAL_ARGUMENT, "not a single-node repair");
            clay->rtc.reset(new ClayRtc(clay->pl.repair_program(clay->pl.erased()[0])));
            clay->rtc_state = 1;
        } catch (const Error &e) {
            clay->rtc_state = -1;
            clay->rtc_why = e.what();
        }
    }
    return clay->rtc_state == 1 ? clay->rtc.get() : nullptr;
}
}  // namespace

int ecx_clay_perform_coding_batch(ecx_clay *clay, const uint8_t *in, int64_t in_stripe_stride, int64_t in_sub_stride,
                                  uint8_t *out, int64_t out_stripe_stride, int64_t out_sub_stride, int64_t nstripes,
                                  int64_t buf_size, void *stream) {
    return guarded(__func__, [&]() -> int {
        if (clay->pl.erased().empty()) return ECX_OK;
        if (nstripes < 0 || buf_size < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (!in || !out) throw Error(ECX_E_NULL, "null device pointer");
        ecx_map *m = clay_standard_map(clay);
        // Single-node repair: the per-helper-plane kernel (clay_rtc.hpp) for the whole
        // 4 KiB chunks of 16-B-aligned layouts whose slot offsets fit 31 bits; the
        // composed-map kernel takes any tail and every other layout.
        int64_t done = 0;
        const char *rtc_kernel = nullptr;
        // auto (1): repairs whose composed map spans several 8-row tiles (alpha > 8), where
        // the composed kernel is bound by vector issue (Clay(10,4): 0.61 -> 0.70 of HBM);
        // Clay(4,2)'s single-tile map is memory-bound and stays on the composed kernel
        // (0.83 there vs 0.63 per plane: profiles/r02_clay_rtc_ab.jsonl).
        const int rtc_mode = tuning().clay_rtc;
        const bool rtc_want = rtc_mode == 2 || (rtc_mode == 1 && m->cm.n_tiles() > 1);
        if (rtc_want && buf_size >= kChunkBytes && ((uintptr_t)in % 16) == 0 && ((uintptr_t)out % 16) == 0 &&
            in_stripe_stride % 16 == 0 && in_sub_stride % 16 == 0 && out_stripe_stride % 16 == 0 &&
            out_sub_stride % 16 == 0 && in_sub_stride >= 0 && out_sub_stride >= 0) {
            if (ClayRtc *r = clay_rtc(clay)) {
                // auto: a generated kernel that cannot be compiled or loaded here (no
                // hiprtc, another target) falls back to the composed map; forced (2) throws
                RtcShape sh = rtc_current_shape();
                // slot offsets beyond 31 bits (1 MiB sub-chunks of Clay(10,4)): the plane-group
                // kernel with 64-bit load addresses; the per-plane kernel has no such form
                const bool narrow = (int64_t)r->program().max_in_slot * in_sub_stride + kChunkBytes <= 0x7FFFFFFF;
                if (!narrow) sh.wide = 1;
                if ((narrow || (clay_grp_supported(r->program()) && sh.group)) &&
                    (rtc_mode == 2 || r->available(sh, (hipStream_t)stream))) {
                    done = buf_size / kChunkBytes * kChunkBytes;
                    r->launch(sh, in, in_stripe_stride, in_sub_stride, out, out_stripe_stride, out_sub_stride,
                              nstripes, done / kChunkBytes, (hipStream_t)stream);
                    rtc_kernel = r->kernel_name(sh);
                    int dev = 0;
                    check_hip(hipGetDevice(&dev), "hipGetDevice");
                    note_device_launch(dev, (hipStream_t)stream, nstripes * done * (int64_t)(r->program().max_in_slot + 1));
                }
            }
        }
        if (done < buf_size)
            launch_apply(m->cm, in + done, in_stripe_stride, in_sub_stride, out + done, out_stripe_stride,
                         out_sub_stride, nstripes, buf_size - done, (hipStream_t)stream);
        if (rtc_kernel) set_last_kernel(rtc_kernel);
        return ECX_OK;
    });
}

int ecx_clay_rtc_compile_check(ecx_clay *clay) {
    return guarded(__func__, [&]() -> int {
        ClayRtc *r = clay_rtc(clay);
        if (!r) throw Error(ECX_E_ILLEGAL_ARGUMENT, "no per-helper-plane program: " + clay->rtc_why);
        return (int)rtc_compile_check(clay_rtc_selected_source(r->program(), rtc_current_shape()));
    });
}

int ecx_clay_rtc_source(ecx_clay *clay, char *buf, int len) {
    return guarded(__func__, [&]() -> int {
        ClayRtc *r = clay_rtc(clay);
        if (!r) throw Error(ECX_E_ILLEGAL_ARGUMENT, "no per-helper-plane program: " + clay->rtc_why);
        const std::string src = clay_rtc_selected_source(r->program(), rtc_current_shape());
        if (buf && len > (int)src.size()) std::memcpy(buf, src.c_str(), src.size() + 1);
        return (int)src.size();
    });
}

int ecx_map_planes_compile_check(const ecx_map *map, int accumulate) {
    return guarded(__func__, [&]() -> int {
        PlanesShape sh;
        const Tuning tu = tuning();
        sh.lookahead = tu.planes_lookahead;
        sh.waves = tu.planes_waves;
        return (int)rtc_compile_check(map_planes_source(map->cm.map(), sh, accumulate != 0));
    });
}

int ecx_map_planes_source(const ecx_map *map, int accumulate, char *buf, int len) {
    return guarded(__func__, [&]() -> int {
        PlanesShape sh;
        const Tuning tu = tuning();
        sh.lookahead = tu.planes_lookahead;
        sh.waves = tu.planes_waves;
        const std::string src = map_planes_source(map->cm.map(), sh, accumulate != 0);
        if (buf && len > (int)src.size()) std::memcpy(buf, src.c_str(), src.size() + 1);
        return (int)src.size();
    });
}

// ---------------------------------------------------------------- LRC
namespace {
struct LrcCache {
    std::mutex mu;
    LrcCode code;
    std::unique_ptr<ecx_map> enc;
    std::map<uint32_t, std::unique_ptr<ecx_map>> dec;  // present mask -> map
};
LrcCache *lrc_cache() {
    static LrcCache c;
    return &c;
}
}  // namespace

int ecx_lrc_map(const uint8_t *block_present, const ecx_map **out) {
    return guarded(__func__, [&]() -> int {
        if (!out) throw Error(ECX_E_NULL, "null out pointer");
        LrcCache &c = *lrc_cache();
        std::lock_guard<std::mutex> lk(c.mu);
        if (!block_present) {
            if (!c.enc) c.enc = std::make_unique<ecx_map>(c.code.encode_map());
            *out = c.enc.get();
            return ECX_OK;
        }
        uint32_t mask = 0;
        std::vector<bool> present(LrcCode::kN);
        for (int i = 0; i < LrcCode::kN; ++i) {
            present[i] = block_present[i] != 0;
            mask |= present[i] ? (1u << i) : 0u;
        }
        auto &slot = c.dec[mask];
        if (!slot) slot = std::make_unique<ecx_map>(c.code.decode_map(present));
        *out = slot.get();
        return ECX_OK;
    });
}

int ecx_lrc_encode_batch(uint8_t *stripes, int64_t stripe_stride, int64_t block_stride, int64_t nstripes,
                         int64_t block_size, void *stream) {
    const ecx_map *m = nullptr;
    int st = ecx_lrc_map(nullptr, &m);
    if (st) return st;
    return ecx_map_apply_batch(m, stripes, stripe_stride, block_stride, stripes, stripe_stride, block_stride, nstripes,
                               block_size, stream);
}

int ecx_lrc_decode_batch(uint8_t *stripes, int64_t stripe_stride, int64_t block_stride, const uint8_t *block_present,
                         int64_t nstripes, int64_t block_size, void *stream) {
    if (!block_present) return ECX_E_NULL;
    const ecx_map *m = nullptr;
    int st = ecx_lrc_map(block_present, &m);
    if (st) return st;
    if (m->cm.map().n_out == 0) return ECX_OK;  // nothing missing
    return ecx_map_apply_batch(m, stripes, stripe_stride, block_stride, stripes, stripe_stride, block_stride, nstripes,
                               block_size, stream);
}

// ---------------------------------------------------------------- host-memory batches (f1)
int ecx_map_apply_batch_host(const ecx_map *map, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                             uint8_t *out, int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes,
                             int64_t byte_count) {
    return guarded(__func__, [&]() -> int {
        if (nstripes < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (!in || !out) throw Error(ECX_E_NULL, "null host pointer");
        run_host_batch(const_cast<ecx_map *>(map)->cm, in, in_stripe_stride, in_slot_stride, out, out_stripe_stride,
                       out_slot_stride, nstripes, byte_count);
        return ECX_OK;
    });
}

int ecx_clay_perform_coding_batch_host(ecx_clay *clay, const uint8_t *in, int64_t in_stripe_stride,
                                       int64_t in_sub_stride, uint8_t *out, int64_t out_stripe_stride,
                                       int64_t out_sub_stride, int64_t nstripes, int64_t buf_size) {
    return guarded(__func__, [&]() -> int {
        if (clay->pl.erased().empty()) return ECX_OK;
        if (nstripes < 0 || buf_size < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (!in || !out) throw Error(ECX_E_NULL, "null host pointer");
        ecx_map *m = clay_standard_map(clay);
        run_host_batch(m->cm, in, in_stripe_stride, in_sub_stride, out, out_stripe_stride, out_sub_stride, nstripes,
                       buf_size);
        return ECX_OK;
    });
}

int ecx_map_apply_batch_host_devices(const ecx_map *map, const uint8_t *in, int64_t in_stripe_stride,
                                     int64_t in_slot_stride, uint8_t *out, int64_t out_stripe_stride,
                                     int64_t out_slot_stride, int64_t nstripes, int64_t byte_count,
                                     const int *devices, int ndev) {
    return guarded(__func__, [&]() -> int {
        if (!map) throw Error(ECX_E_NULL, "null map");
        if (nstripes < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (!in || !out) throw Error(ECX_E_NULL, "null host pointer");
        run_host_batch_devices(const_cast<ecx_map *>(map)->cm, in, in_stripe_stride, in_slot_stride, out,
                               out_stripe_stride, out_slot_stride, nstripes, byte_count, devices, ndev);
        return ECX_OK;
    });
}

int ecx_clay_perform_coding_batch_host_devices(ecx_clay *clay, const uint8_t *in, int64_t in_stripe_stride,
                                               int64_t in_sub_stride, uint8_t *out, int64_t out_stripe_stride,
                                               int64_t out_sub_stride, int64_t nstripes, int64_t buf_size,
                                               const int *devices, int ndev) {
    return guarded(__func__, [&]() -> int {
        if (!clay) throw Error(ECX_E_NULL, "null decoding step");
        if (!devices) throw Error(ECX_E_NULL, "null device list");
        if (ndev <= 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "empty device list");
        if (clay->pl.erased().empty()) return ECX_OK;
        if (nstripes < 0 || buf_size < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (!in || !out) throw Error(ECX_E_NULL, "null host pointer");
        run_host_batch_devices(clay_standard_map(clay)->cm, in, in_stripe_stride, in_sub_stride, out,
                               out_stripe_stride, out_sub_stride, nstripes, buf_size, devices, ndev);
        return ECX_OK;
    });
}

namespace {
int rs_check_host(const char *fn, ecx_rs *rs, const uint8_t *base, int64_t stripe_stride, int64_t shard_stride,
                  int64_t nstripes, int64_t offset, int64_t byte_count, uint8_t *verdict, const int *devices,
                  int ndev, bool multi) {
    return guarded(fn, [&]() -> int {
        if (!rs) throw Error(ECX_E_NULL, "null codec");
        if (nstripes < 0 || offset < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        if (stripe_stride < 0 || shard_stride < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative stride");
        if (nstripes > 0 && (!base || !verdict)) throw Error(ECX_E_NULL, "null host pointer");
        CompiledMap &cm = rs_check_map(rs)->cm;
        const uint8_t *in = nstripes > 0 ? base + offset : base;
        if (multi) run_host_check_batch_devices(cm, in, stripe_stride, shard_stride, nstripes, byte_count, verdict,
                                                devices, ndev);
        else run_host_check_batch(cm, in, stripe_stride, shard_stride, nstripes, byte_count, verdict);
        return ECX_OK;
    });
}
}  // namespace

int ecx_rs_is_parity_correct_batch_host(ecx_rs *rs, const uint8_t *base, int64_t stripe_stride,
                                        int64_t shard_stride, int64_t nstripes, int64_t offset,
                                        int64_t byte_count, uint8_t *verdict) {
    return rs_check_host(__func__, rs, base, stripe_stride, shard_stride, nstripes, offset, byte_count, verdict,
                         nullptr, 0, false);
}

int ecx_rs_is_parity_correct_batch_host_devices(ecx_rs *rs, const uint8_t *base, int64_t stripe_stride,
                                                int64_t shard_stride, int64_t nstripes, int64_t offset,
                                                int64_t byte_count, uint8_t *verdict, const int *devices,
                                                int ndev) {
    return rs_check_host(__func__, rs, base, stripe_stride, shard_stride, nstripes, offset, byte_count, verdict,
                         devices, ndev, true);
}

int ecx_host_alloc(int64_t nbytes, void **out) {
    return guarded(__func__, [&]() -> int {
        if (!out) throw Error(ECX_E_NULL, "null out pointer");
        if (nbytes < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative size");
        *out = nullptr;
        check_hip(hipHostMalloc(out, (size_t)std::max<int64_t>(nbytes, 1), hipHostMallocDefault), "hipHostMalloc");
        return ECX_OK;
    });
}

int ecx_host_free(void *ptr) {
    return guarded(__func__, [&]() -> int {
        if (ptr) check_hip(hipHostFree(ptr), "hipHostFree");
        return ECX_OK;
    });
}

int ecx_host_register(void *ptr, int64_t nbytes) {
    return guarded(__func__, [&]() -> int {
        if (!ptr) throw Error(ECX_E_NULL, "null pointer");
        if (nbytes <= 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "non-positive size");
        check_hip(hipHostRegister(ptr, (size_t)nbytes, hipHostRegisterDefault), "hipHostRegister");
        return ECX_OK;
    });
}

int ecx_host_unregister(void *ptr) {
    return guarded(__func__, [&]() -> int {
        if (!ptr) throw Error(ECX_E_NULL, "null pointer");
        check_hip(hipHostUnregister(ptr), "hipHostUnregister");
        return ECX_OK;
    });
}

// ---------------------------------------------------------------- tuning hook (include/ecx_tune.h)
namespace {
bool diagnostic_builds_allowed() {
    const char *v = std::getenv("ECX_DIAGNOSTIC");
    return v && std::strcmp(v, "1") == 0;
}

// Knobs of the measured-and-rejected kernels and builds: accepted by
// the diagnostic library only (`make DIAG=1`, libecx_diag.so).
bool lab_key(const std::string &k) {
    return k == "bitslice" || k == "lds_lut" || k == "wave_groups" || k == "rtc_units" || k == "rtc_persist" ||
           k == "rtc_diag" || k == "occ_lds" || k == "units";
}

// Deployment knobs (host pipeline, per-call plan cache, markers, the layout selection's on/off):
// what a production caller may set.  Every other key changes a kernel's launch shape -- results
// are identical, only speed differs -- and is accepted only by the diagnostic library or when the
// process opted in with ECX_SHAPE_KNOBS=1 in its environment (read once, at the first ecx_tune), so
// one library loaded into a JVM cannot reshape every other caller's launches.
bool deployment_key(const std::string &k) {
    return k == "host_chunk_kib" || k == "host_buffers" || k == "host_gather_kib" || k == "host_zero_copy" ||
           k == "host_contexts" || k == "host_exec_kib" || k == "roctx" || k == "plan_cache" || k == "layout_select";
}

bool shape_knobs_enabled() {
    static const bool on = [] {
        const char *v = std::getenv("ECX_SHAPE_KNOBS");
        return ECX_DIAG || (v && std::strcmp(v, "1") == 0);
    }();
    return on;
}

// One ecx_tune key, under the tuning lock.
int set_tune(Tuning &t, const std::string &k, int value) {
    if (!ECX_DIAG && lab_key(k)) return ECX_E_ILLEGAL_ARGUMENT;
    if (!deployment_key(k) && !shape_knobs_enabled()) return ECX_E_ILLEGAL_ARGUMENT;
    if (k == "depth") {
        if (value != 0 && value != 2 && value != 4 && value != 8 && value != 10 && value != 12 && value != 16 &&
            value != 20 && value != 24)
            return ECX_E_ILLEGAL_ARGUMENT;
        t.depth = value;
    }
    else if (k == "nontemporal") {
        if (value < 0 || value > 2) return ECX_E_ILLEGAL_ARGUMENT;
        t.nontemporal = value;
    }
    else if (k == "xcd_group") {
        if (value < 0 || value > 3) return ECX_E_ILLEGAL_ARGUMENT;
        t.xcd_group = value;
    }
    else if (k == "xcd_misaligned") {
        if (value < 0 || value > 1) return ECX_E_ILLEGAL_ARGUMENT;
        t.xcd_misaligned = value;
    }
    else if (k == "xcd_run") {
        if (value < 1 || value > 4096) return ECX_E_ILLEGAL_ARGUMENT;
        t.xcd_run = value;
    }
    else if (k == "wave_groups") {
        if (value < 0 || value > 2) return ECX_E_ILLEGAL_ARGUMENT;
        t.wave_groups = value;
    }
    else if (k == "store_scope") t.store_scope = value != 0;
    else if (k == "occ_lds") {
        if (value < -1 || value > 65536) return ECX_E_ILLEGAL_ARGUMENT;
        t.occ_lds = value;
    }
    else if (k == "chunk_major") t.chunk_major = value != 0;
    else if (k == "stagger") {
        if (value < 0 || value > 64) return ECX_E_ILLEGAL_ARGUMENT;
        t.stagger = value;
    }
    else if (k == "small_tiles") {
        if (value < 0 || value > 2) return ECX_E_ILLEGAL_ARGUMENT;
        t.small_tiles = value;
    }
    else if (k == "host_zero_copy") t.host_zero_copy = value != 0;
    else if (k == "plan_cache") {
        if (value < 0 || value > 4096) return ECX_E_ILLEGAL_ARGUMENT;
        t.plan_cache = value;
    }
    else if (k == "skew_chunks") {
        if (value < 0 || value > 4 || value == 3) return ECX_E_ILLEGAL_ARGUMENT;
        t.skew_chunks = value;
    }
    else if (k == "layout_select") {
        if (value < 0 || value > 1) return ECX_E_ILLEGAL_ARGUMENT;
        t.layout_select = value;
    }
    else if (k == "wide_tiles") {
        if (value < 0 || value > 2) return ECX_E_ILLEGAL_ARGUMENT;
        t.wide_tiles = value;
    }
    else if (k == "block_threads") {
        if (value != 0 && value != 64 && value != 256) return ECX_E_ILLEGAL_ARGUMENT;
        t.block_threads = value;
    }
    else if (k == "lds_tables") {
        if (value < 0 || value > 2) return ECX_E_ILLEGAL_ARGUMENT;
        t.lds_tables = value;
    }
    else if (k == "host_chunk_kib") {
        if (value < 1) return ECX_E_ILLEGAL_ARGUMENT;
        t.host_chunk = (int64_t)value << 10;
    }
    else if (k == "host_gather_kib") {
        if (value < 0) return ECX_E_ILLEGAL_ARGUMENT;
        t.host_gather_max = (int64_t)value << 10;
    }
    else if (k == "clay_rtc") {
        if (value < 0 || value > 2) return ECX_E_ILLEGAL_ARGUMENT;
        t.clay_rtc = value;
    }
    else if (k == "rtc_lookahead") {
        if (value < 0 || value > 31) return ECX_E_ILLEGAL_ARGUMENT;
        // bit 4 is the DIAGNOSTIC movement-only build, whose outputs are not the repair:
        // refused unless this is the diagnostic library and the process opted in with ECX_DIAGNOSTIC=1
        if ((value & 16) && !(ECX_DIAG && diagnostic_builds_allowed())) return ECX_E_ILLEGAL_ARGUMENT;
        t.rtc_lookahead = value;
    }
    else if (k == "rtc_xcd") {
        if (value < 0 || value > 4) return ECX_E_ILLEGAL_ARGUMENT;
        t.rtc_xcd = value;
    }
    else if (k == "rtc_group") t.rtc_group = value != 0;
    else if (k == "rtc_diag") {
        if (value < 0 || value > 31) return ECX_E_ILLEGAL_ARGUMENT;
        if (value && !diagnostic_builds_allowed()) return ECX_E_ILLEGAL_ARGUMENT;  // outputs not the repair
        t.rtc_diag = value;
    }
    else if (k == "rtc_sched") {
        if (value < 0 || value > 2) return ECX_E_ILLEGAL_ARGUMENT;
        t.rtc_sched = value;
    }
    else if (k == "rtc_wide") {
        if (value < 0 || value > 1) return ECX_E_ILLEGAL_ARGUMENT;
        t.rtc_wide = value;
    }
    else if (k == "rtc_nt") {
        if (value < 0 || value > 15) return ECX_E_ILLEGAL_ARGUMENT;
        t.rtc_nt = value;
    }
    else if (k == "rtc_units") {
        if (value < 1 || value > 2) return ECX_E_ILLEGAL_ARGUMENT;
        t.rtc_units = value;
    }
    else if (k == "rtc_persist") {
        if (value < 0 || value > 8) return ECX_E_ILLEGAL_ARGUMENT;
        t.rtc_persist = value;
    }
    else if (k == "rtc_waves") {
        if (value < 2 || value > 4) return ECX_E_ILLEGAL_ARGUMENT;
        t.rtc_waves = value;
    }
    else if (k == "map_planes") {
        if (value < 0 || value > 2) return ECX_E_ILLEGAL_ARGUMENT;
        t.map_planes = value;
    }
    else if (k == "planes_lookahead") {
        if (value < 0 || value > 15) return ECX_E_ILLEGAL_ARGUMENT;
        t.planes_lookahead = value;
    }
    else if (k == "planes_waves") {
        if (value < 1 || value > 4) return ECX_E_ILLEGAL_ARGUMENT;
        t.planes_waves = value;
    }
    else if (k == "bitslice") {
        if (value < 0 || value > 2) return ECX_E_ILLEGAL_ARGUMENT;
        t.bitslice = value;
    }
    else if (k == "host_contexts") {
        if (value < 0 || value > 1) return ECX_E_ILLEGAL_ARGUMENT;
        t.host_contexts = value;
    }
    else if (k == "roctx") {
        if (value < 0 || value > 1) return ECX_E_ILLEGAL_ARGUMENT;
        g_roctx.store(value);
    }
    else if (k == "lds_lut") {
        if (value < 0 || value > 2) return ECX_E_ILLEGAL_ARGUMENT;
        t.lds_lut = value;
    }
    else if (k == "units") {
        if (value != 1 && value != 2 && value != 4) return ECX_E_ILLEGAL_ARGUMENT;
        t.units = value;
    }
    else if (k == "host_exec_kib") {
        if (value < 0 || value > (1 << 20)) return ECX_E_ILLEGAL_ARGUMENT;
        t.host_exec_max = (int64_t)value << 10;
    }
    else if (k == "host_buffers") {
        if (value < 1 || value > 8) return ECX_E_ILLEGAL_ARGUMENT;
        t.host_buffers = value;
    }
    else return ECX_E_ILLEGAL_ARGUMENT;
    return ECX_OK;
}
}  // namespace

int ecx_tune(const char *key, int value) {
    const std::string k = key ? key : "";
    int rc = ECX_OK;
    update_tuning([&](Tuning &t) { rc = set_tune(t, k, value); });
    return rc;
}

int ecx_tune_value(const char *key, int *value) {
    const std::string k = key ? key : "";
    if (!value || !deployment_key(k)) return ECX_E_ILLEGAL_ARGUMENT;
    const Tuning t = tuning();
    if (k == "host_chunk_kib") *value = (int)(t.host_chunk >> 10);
    else if (k == "host_buffers") *value = t.host_buffers;
    else if (k == "host_gather_kib") *value = (int)(t.host_gather_max >> 10);
    else if (k == "host_zero_copy") *value = t.host_zero_copy;
    else if (k == "host_contexts") *value = t.host_contexts;
    else if (k == "host_exec_kib") *value = (int)(t.host_exec_max >> 10);
    else if (k == "roctx") *value = g_roctx.load();
    else if (k == "plan_cache") *value = t.plan_cache;
    else *value = t.layout_select;  // deployment_key: the only one left
    return ECX_OK;
}

int ecx_probe_bandwidth(int kind, const uint8_t *src, uint8_t *dst, int64_t nbytes, int nontemporal, void *stream) {
    return guarded(__func__, [&]() -> int {
        launch_probe(kind, src, dst, nbytes, nontemporal != 0, (hipStream_t)stream);
        return ECX_OK;
    });
}

int ecx_map_plan_stats(const ecx_map *map, int *n_tiles, int *n_entries, int *n_groups, int *union_total) {
    return guarded(__func__, [&]() -> int {
        const CompiledMap &cm = map->cm;
        if (n_tiles) *n_tiles = cm.n_tiles();
        if (n_entries) *n_entries = cm.n_tiles() ? cm.n_entries() : 0;
        if (n_groups) *n_groups = cm.n_groups();
        if (union_total) *union_total = cm.union_total();
        return ECX_OK;
    });
}

int ecx_build_diag(void) { return ECX_DIAG ? 1 : 0; }

int ecx_host_exec_isa(void) { return host_exec_isa(); }

int ecx_stripe_range(int64_t nstripes, int parts, int j, int64_t *begin, int64_t *end) {
    if (nstripes < 0 || parts <= 0 || j < 0 || j >= parts || !begin || !end) return ECX_E_ILLEGAL_ARGUMENT;
    stripe_range(nstripes, parts, j, begin, end);
    return ECX_OK;
}

int ecx_map_layout_choice(const ecx_map *map, int64_t slot_pitch, float *median_ms, int n) {
    return guarded(__func__, [&]() -> int {
        if (!map) throw Error(ECX_E_NULL, "null map");
        if (slot_pitch <= 0 || n < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "slot pitch or count");
        std::vector<float> ms;
        const int c = const_cast<ecx_map *>(map)->cm.layout_choice(slot_pitch, median_ms ? &ms : nullptr);
        if (median_ms)
            for (int i = 0; i < n; ++i) median_ms[i] = i < (int)ms.size() ? ms[i] : -1.f;
        if (c < 0) return 0x200;  // none chosen yet (or the layout is not selected per launch)
        const int code = layout_candidate_code(c);
        return code == -1 ? 0x100 : code;  // 0x100 = the static rules' shape
    });
}

int ecx_map_layout_state(const ecx_map *map, int64_t slot_pitch, int *state, int *dropped) {
    return guarded(__func__, [&]() -> int {
        if (!map) throw Error(ECX_E_NULL, "null map");
        if (slot_pitch <= 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "slot pitch");
        int st = -1, dr = 0;
        const int c = const_cast<ecx_map *>(map)->cm.layout_choice(slot_pitch, nullptr, &st, &dr);
        if (state) *state = c < 0 ? -1 : st;
        if (dropped) *dropped = c < 0 ? 0 : dr;
        return ECX_OK;
    });
}

int ecx_map_host_plan(const ecx_map *map, int64_t in_stripe_stride, int64_t in_slot_stride, int64_t out_stripe_stride,
                      int64_t out_slot_stride, int64_t nstripes, int64_t byte_count, int64_t *plan) {
    return guarded(__func__, [&]() -> int {
        if (!map || !plan) throw Error(ECX_E_NULL, "null map or plan");
        if (nstripes < 0 || byte_count < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "negative count");
        const HostBatchPlan hp = plan_host_batch(const_cast<ecx_map *>(map)->cm, in_stripe_stride, in_slot_stride,
                                                 out_stripe_stride, out_slot_stride, nstripes, byte_count);
        const int64_t v[10] = {hp.chunk, hp.nchunks, hp.buffers, hp.h2d_copies, hp.h2d_rows, hp.d2h_copies,
                               hp.d2h_rows, hp.h2d_3d, hp.d2h_3d, hp.slices};
        std::memcpy(plan, v, sizeof(v));
        return ECX_OK;
    });
}

int ecx_last_launch_shape(char *buf, int len) {
    const std::string k = last_launch_shape();
    if (!buf || len < (int)k.size() + 1) return ECX_E_ILLEGAL_ARGUMENT;
    std::memcpy(buf, k.c_str(), k.size() + 1);
    return (int)k.size();
}

int ecx_last_kernel(char *buf, int len) {
    const std::string &k = last_kernel();
    if (!buf || len < (int)k.size() + 1) return ECX_E_ILLEGAL_ARGUMENT;
    std::memcpy(buf, k.c_str(), k.size() + 1);
    return (int)k.size();
}

int ecx_map_selftest(const ecx_map *map, uint64_t seed) {
    return guarded(__func__, [&]() -> int {
        const CompiledMap &cm = map->cm;
        const LinearMap &m = cm.map();
        const int64_t len = 97;  // ragged on purpose
        const int nin = cm.max_in_slot() + 1, nout = cm.max_out_slot() + 1;
        std::vector<uint8_t> in((size_t)std::max(1, nin) * len), ref((size_t)std::max(1, nout) * len, 0);
        uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
        for (uint8_t &b : in) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            b = (uint8_t)x;
        }
        const Field &f = Field::get();
        for (int o = 0; o < m.n_out; ++o)
            for (int j = 0; j < m.n_in; ++j) {
                const uint8_t c = m.at(o, j);
                if (!c) continue;
                for (int64_t i = 0; i < len; ++i)
                    ref[(size_t)m.out_slot[o] * len + i] ^= f.mul(c, in[(size_t)m.in_slot[j] * len + i]);
            }
        auto check = [&](const std::vector<uint8_t> &got, const char *what) {
            for (int o = 0; o < m.n_out; ++o)
                if (!std::equal(got.begin() + (size_t)m.out_slot[o] * len, got.begin() + (size_t)(m.out_slot[o] + 1) * len,
                                ref.begin() + (size_t)m.out_slot[o] * len))
                    throw Error(ECX_E_ILLEGAL_ARGUMENT, what);
        };
        for (bool via_unions : {false, true}) {
            std::vector<uint8_t> got(ref.size(), 0);
            cm.emulate(in.data(), got.data(), len, via_unions);
            check(got, via_unions ? "plan (union view) differs from the map" : "plan (slot view) differs from the map");
        }
        // The padded arrays the device receives, at both ring depths, with the split
        // tables read as k_gf_apply reads them (SGPRs only, or low dwords from LDS).
        for (int depth : {4, 8, 10, 12, 20}) {
            const HostPlan hp = cm.padded_plan(depth);
            if (cm.n_wide_tiles() > 0 && depth <= 8) {  // wide tiles run at depth 4 / 8
                std::vector<uint8_t> got(ref.size(), 0);
                cm.emulate_wide(hp, in.data(), got.data(), len);
                check(got, "padded plan (wide tiles) differs from the map");
            }
            for (bool tlds : {false, true}) {
                std::vector<uint8_t> got(ref.size(), 0);
                cm.emulate_padded(hp, in.data(), got.data(), len, tlds, depth);
                check(got, tlds ? "padded plan (LDS tables) differs from the map" : "padded plan differs from the map");
            }
        }
        // The bit-sliced kernel's arithmetic (bits.hpp, shared with apply_bits.hip) over
        // its padded entries at both of its ring depths, on one whole 4 KiB chunk.
        const int64_t blen = kChunkBytes;
        std::vector<uint8_t> bin((size_t)std::max(1, nin) * blen), bref((size_t)std::max(1, nout) * blen, 0);
        for (uint8_t &b : bin) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            b = (uint8_t)x;
        }
        for (int o = 0; o < m.n_out; ++o)
            for (int j = 0; j < m.n_in; ++j) {
                const uint8_t c = m.at(o, j);
                if (!c) continue;
                for (int64_t i = 0; i < blen; ++i)
                    bref[(size_t)m.out_slot[o] * blen + i] ^= f.mul(c, bin[(size_t)m.in_slot[j] * blen + i]);
            }
        for (int depth : {2, 4}) {
            if (!ECX_DIAG) break;  // bit-sliced entries exist in the diagnostic build only
            std::vector<uint8_t> got(bref.size(), 0);
            cm.emulate_bits(cm.padded_plan(depth), bin.data(), got.data(), blen);
            for (int o = 0; o < m.n_out; ++o)
                if (!std::equal(got.begin() + (size_t)m.out_slot[o] * blen, got.begin() + (size_t)(m.out_slot[o] + 1) * blen,
                                bref.begin() + (size_t)m.out_slot[o] * blen))
                    throw Error(ECX_E_ILLEGAL_ARGUMENT, "bit-sliced plan differs from the map");
        }
        return ECX_OK;
    });
}

// ---------------------------------------------------------------- synthetic data / verification
int ecx_fill_random(uint8_t *dst, int64_t nbytes, uint64_t seed, void *stream) {
    return guarded(__func__, [&]() -> int {
        launch_fill_random(dst, nbytes, seed, (hipStream_t)stream);
        return ECX_OK;
    });
}

int ecx_count_mismatch(const uint8_t *a, int64_t a_stride, const uint8_t *b, int64_t b_stride, int64_t nrows,
                       int64_t row_bytes, uint64_t *d_count, void *stream) {
    return guarded(__func__, [&]() -> int {
        launch_count_mismatch(a, a_stride, b, b_stride, nrows, row_bytes, d_count, (hipStream_t)stream);
        return ECX_OK;
    });
}

}  // extern "C"
