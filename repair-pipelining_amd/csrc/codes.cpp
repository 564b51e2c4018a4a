// codes.cpp -- see codes.hpp.
#include "codes.hpp"

#include <algorithm>
#include <cmath>

namespace ecx {

namespace {

SymBuf zeros(int w) { return std::make_shared<std::vector<uint8_t>>((size_t)w, 0); }

SymBuf unit(int w, int j) {
    SymBuf b = zeros(w);
    (*b)[(size_t)j] = 1;
    return b;
}

SymBuf clone(const SymBuf &b) { return std::make_shared<std::vector<uint8_t>>(*b); }

// y ^= c * x  (one GF(256) multiply-accumulate per coefficient)
void axpy(std::vector<uint8_t> &y, uint8_t c, const std::vector<uint8_t> &x) {
    if (!c) return;
    const uint8_t *t = Field::get().row(c);
    for (size_t i = 0; i < y.size(); ++i) y[i] ^= t[x[i]];
}

}  // namespace

int LinearMap::nnz() const {
    int s = 0;
    for (uint8_t v : a) s += v != 0;
    return s;
}

LinearMap LinearMap::pruned() const {
    std::vector<int> keep;
    for (int j = 0; j < n_in; ++j)
        for (int o = 0; o < n_out; ++o)
            if (at(o, j)) {
                keep.push_back(j);
                break;
            }
    LinearMap r;
    r.n_out = n_out;
    r.n_in = (int)keep.size();
    r.out_slot = out_slot;
    r.a.assign((size_t)r.n_out * r.n_in, 0);
    for (int jj = 0; jj < r.n_in; ++jj) {
        r.in_slot.push_back(in_slot[keep[jj]]);
        for (int o = 0; o < n_out; ++o) r.a[(size_t)o * r.n_in + jj] = at(o, keep[jj]);
    }
    return r;
}

// ---------------------------------------------------------------- RsCode
RsCode::RsCode(int data_shards, int parity_shards) : k_(data_shards), m_(parity_shards) {
    if (256 < data_shards + parity_shards) throw Error(ECX_E_TOO_MANY_SHARDS, "too many shards - max is 256");
    if (data_shards <= 0 || parity_shards < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "invalid shard counts");
    const Field &f = Field::get();
    const int n = k_ + m_;
    Matrix v(n, k_);  // Vandermonde V[r][c] = r^c (0^0 = 1)
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k_; ++c) v.at(r, c) = f.pow((uint8_t)r, c);
    Matrix top(k_, k_);
    for (int r = 0; r < k_; ++r)
        for (int c = 0; c < k_; ++c) top.at(r, c) = v.at(r, c);
    gen_ = v * top.inverse();
}

Matrix RsCode::data_decoder(const std::vector<bool> &present, std::vector<int> *rows_used) const {
    Matrix sub(k_, k_);
    int r = 0;
    for (int i = 0; i < n() && r < k_; ++i)
        if (present[i]) {
            std::copy(gen_.row(i), gen_.row(i) + k_, sub.row(r));
            if (rows_used) rows_used->push_back(i);
            ++r;
        }
    if (r < k_) throw Error(ECX_E_NOT_ENOUGH_SHARDS, "Not enough shards present");
    return sub.inverse();
}

void RsCode::decode_missing(std::vector<SymBuf> &shards, const std::vector<bool> &present) const {
    int np = 0;
    for (int i = 0; i < n(); ++i) np += present[i] ? 1 : 0;
    if (np == n()) return;
    if (np < k_) throw Error(ECX_E_NOT_ENOUGH_SHARDS, "Not enough shards present");
    std::vector<int> used;
    const Matrix dec = data_decoder(present, &used);
    // Missing data shards from the k "sub shards" (the first k present).
    for (int i = 0; i < k_; ++i) {
        if (present[i]) continue;
        std::vector<uint8_t> acc(shards[i]->size(), 0);
        for (int r = 0; r < k_; ++r) axpy(acc, dec.at(i, r), *shards[used[r]]);
        *shards[i] = std::move(acc);
    }
    // Missing parity shards from all data shards (now complete).
    for (int p = 0; p < m_; ++p) {
        if (present[k_ + p]) continue;
        std::vector<uint8_t> acc(shards[k_ + p]->size(), 0);
        for (int i = 0; i < k_; ++i) axpy(acc, parity_row(p)[i], *shards[i]);
        *shards[k_ + p] = std::move(acc);
    }
}

LinearMap RsCode::encode_map() const {
    LinearMap mp;
    mp.n_out = m_;
    mp.n_in = k_;
    mp.a.assign((size_t)m_ * k_, 0);
    for (int p = 0; p < m_; ++p) std::copy(parity_row(p), parity_row(p) + k_, mp.a.begin() + (size_t)p * k_);
    for (int i = 0; i < k_; ++i) mp.in_slot.push_back(i);
    for (int p = 0; p < m_; ++p) mp.out_slot.push_back(k_ + p);
    return mp;
}

LinearMap RsCode::decode_map(const std::vector<bool> &present) const {
    const int w = n();
    std::vector<SymBuf> sh(w);
    for (int i = 0; i < w; ++i) sh[i] = present[i] ? unit(w, i) : zeros(w);
    decode_missing(sh, present);
    LinearMap mp;
    mp.n_in = w;
    for (int i = 0; i < w; ++i) mp.in_slot.push_back(i);
    for (int i = 0; i < w; ++i) {
        if (present[i]) continue;
        mp.out_slot.push_back(i);
        mp.a.insert(mp.a.end(), sh[i]->begin(), sh[i]->end());
    }
    mp.n_out = (int)mp.out_slot.size();
    return mp.pruned();
}

// ---------------------------------------------------------------- LrcCode
namespace {
// Stack per-group maps (over group-local slots 0..R) into one map over the N blocks.
LinearMap stack_groups(const std::vector<std::pair<int, LinearMap>> &parts) {
    LinearMap mp;
    mp.n_in = LrcCode::kN;
    for (int i = 0; i < LrcCode::kN; ++i) mp.in_slot.push_back(i);
    for (const auto &gp : parts) {
        const int base = gp.first * (LrcCode::kR + 1);
        const LinearMap &g = gp.second;
        for (int o = 0; o < g.n_out; ++o) {
            std::vector<uint8_t> row(LrcCode::kN, 0);
            for (int j = 0; j < g.n_in; ++j) row[base + g.in_slot[j]] = g.at(o, j);
            mp.a.insert(mp.a.end(), row.begin(), row.end());
            mp.out_slot.push_back(base + g.out_slot[o]);
        }
    }
    mp.n_out = (int)mp.out_slot.size();
    return mp.pruned();
}
}  // namespace

LinearMap LrcCode::encode_map() const {
    std::vector<std::pair<int, LinearMap>> parts;
    for (int g = 0; g < kGroups; ++g) parts.push_back({g, group_.encode_map()});
    return stack_groups(parts);
}

LinearMap LrcCode::decode_map(const std::vector<bool> &present) const {
    if ((int)present.size() != kN) throw Error(ECX_E_ILLEGAL_ARGUMENT, "wrong number of blocks");
    std::vector<std::pair<int, LinearMap>> parts;
    for (int g = 0; g < kGroups; ++g) {
        std::vector<bool> p(present.begin() + g * (kR + 1), present.begin() + (g + 1) * (kR + 1));
        bool all = true;
        for (bool b : p) all &= b;
        if (!all) parts.push_back({g, group_.decode_map(p)});  // throws "Not enough shards present"
    }
    return stack_groups(parts);
}

// ---------------------------------------------------------------- ClayPlanner
namespace {
int ipow(int b, int e) {
    int r = 1;
    while (e-- > 0) r *= b;
    return r;
}
}  // namespace

ClayPlanner::ClayPlanner(int data_units, int parity_units, std::vector<int> erased, int virtual_units,
                         bool is_test)
    : k_(data_units + virtual_units), m_(parity_units), v_(virtual_units), is_test_(is_test),
      erased_real_(std::move(erased)), pair_(2, 2), rs_(data_units + virtual_units, parity_units) {
    if (parity_units <= 0 || virtual_units < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "invalid unit counts");
    for (int e : erased_real_) {
        if (v_ > 0 && (e < 0 || e >= n_real())) throw Error(ECX_E_INDEX, "erased index out of range");
        erased_.push_back(under(e));
    }
    q_ = parity_units;
    t_ = (parity_units + k_) / parity_units;  // integer division, ClayCodeUtil :692
    if (t_ > 16) throw Error(ECX_E_ILLEGAL_ARGUMENT, "sub-packetization too large");
    alpha_ = ipow(q_, t_);
    if ((long long)n() * alpha_ > 16384)
        throw Error(ECX_E_ILLEGAL_ARGUMENT, "n*alpha > 16384 sub-chunks per stripe is beyond the planner");
}

std::vector<int> ClayPlanner::zvec(int z) const {
    std::vector<int> v(t_);
    for (int i = t_ - 1; i >= 0; --i) {
        v[i] = z % q_;
        z /= q_;
    }
    return v;
}

int ClayPlanner::zindex(const std::vector<int> &v) const {
    int z = 0;
    for (int i = 0; i < t_; ++i) z = z * q_ + v[i];
    return z;
}

int ClayPlanner::couple_plane(int x, int y, int z) const {
    std::vector<int> v = zvec(z);
    if (y >= t_) throw Error(ECX_E_INDEX, "node outside the q x t grid");
    v[y] = x;
    return zindex(v);
}

bool ClayPlanner::is_erased(int idx) const { return std::find(erased_.begin(), erased_.end(), idx) != erased_.end(); }

int ClayPlanner::erasure_type(int idx, int z) const {
    const std::vector<int> v = zvec(z);
    const int x = nx(idx), y = ny(idx);
    if (y >= t_) throw Error(ECX_E_INDEX, "node outside the q x t grid");
    if (v[y] == x) return 0;
    return is_erased(node(v[y], y)) ? 2 : 1;
}

int ClayPlanner::intersection_score(int z) const {
    const std::vector<int> v = zvec(z);
    int s = 0;
    for (int e : erased_) {
        if (ny(e) >= t_) throw Error(ECX_E_INDEX, "node outside the q x t grid");
        s += v[ny(e)] == nx(e);
    }
    return s;
}

std::vector<int> ClayPlanner::helper_planes(int e_real) const {
    const int e = v_ > 0 ? under(e_real) : e_real;
    const int x = nx(e), y = ny(e);
    if (e < 0 || y >= t_) throw Error(ECX_E_INDEX, "erased node outside the q x t grid");
    std::vector<int> out;
    for (int z = 0; z < alpha_; ++z)
        if (zvec(z)[y] == x) out.push_back(z);
    return out;
}

// The Clay pair transform as RS(2,2) over (A, A', B, B') = (C(z,i), C(z',i'), U(z,i), U(z',i'))
// with exactly two unknown (null) entries; returns the array at the first null
// position (getPairWiseCouple, :630-666; callers use outputs[0] only).
SymBuf ClayPlanner::pair_couple(SymBuf a, SymBuf a2, SymBuf b, SymBuf b2, int width) const {
    std::vector<SymBuf> arr = {a, a2, b, b2};
    int lost[2] = {0, 0}, nl = 0;
    for (int i = 0; i < 4; ++i)
        if (!arr[i]) {
            if (nl == 2) throw Error(ECX_E_INDEX, "more than two unknowns in a coupled pair");
            lost[nl++] = i;
        }
    for (auto &p : arr)
        if (!p) p = zeros(width);
    std::vector<bool> present(4, true);
    present[lost[0]] = present[lost[1]] = false;
    pair_.decode_missing(arr, present);
    return arr[lost[0]];
}

// decodeDecoupledPlane (:542-597): the default branch (decodeMissing), or for a single repair of
// an is_test planner the -DisTest=true branch (:571-581).
void ClayPlanner::decode_plane(std::vector<SymBuf> &plane, const std::vector<int> &erased, int width,
                               bool single) const {
    if (single && is_test_) {
        decode_plane_is_test(plane, erased, width);
        return;
    }
    int nulls = 0;
    for (auto &p : plane) nulls += !p;
    if (nulls > (int)erased.size()) throw Error(ECX_E_INDEX, "more absent shards than erasures in a plane");
    std::vector<SymBuf> arr(plane.size());
    for (size_t i = 0; i < plane.size(); ++i) arr[i] = plane[i] ? plane[i] : zeros(width);
    std::vector<bool> present(plane.size(), true);
    for (int e : erased)
        if (e < (int)plane.size()) present[e] = false;
    rs_.decode_missing(arr, present);
    for (int e : erased) plane[e] = arr[e];
    for (auto &p : plane)
        if (!p) throw Error(ECX_E_NULL, "absent shard in a decoupled plane");
}

// decodeDecoupledPlane's isTest branch (:571-581): for i in 0 .. n-|E|-1,
// decodeMissingSingle(plane[i + |E|], shardIndex i + |E|, index i, ..., isFirst = i == 0)
// (ReedSolomon.java:288-333) -- i.e. shard i + |E| is taken as the i-th of the first k
// present shards, which holds only when the erased indices are 0..|E|-1 (bug B2: otherwise
// the map differs, reading the zero arrays getByteArray made for the erased rows).  Each call
// inverts the first-k-present submatrix; when isFirst and shardIndex < k it replaces the
// output of every missing DATA shard with a fresh array; it then writes outputs[j] (=, or ^=)
// rows[j][index] * shard for every j < |E|, and a missing PARITY shard has no row: the
// reference's NullPointerException (bug B3), here ECX_E_NULL.  The outputs replace the erased
// entries of the plane.
void ClayPlanner::decode_plane_is_test(std::vector<SymBuf> &plane, const std::vector<int> &erased, int width) const {
    const int nn = (int)plane.size(), ne = (int)erased.size();
    std::vector<SymBuf> arr(plane.size());  // getByteArray: a null entry becomes a fresh zero array
    for (int i = 0; i < nn; ++i) arr[(size_t)i] = plane[(size_t)i] ? plane[(size_t)i] : zeros(width);
    std::vector<bool> present((size_t)nn, true);
    for (int e : erased)
        if (e < nn) present[(size_t)e] = false;
    int np = 0;
    for (bool p : present) np += p ? 1 : 0;
    if (np < k_) throw Error(ECX_E_NOT_ENOUGH_SHARDS, "Not enough shards present");  // the inversion's submatrix
    std::vector<SymBuf> outputs((size_t)ne);  // new byte[|E|][bufSize]
    for (auto &o : outputs) o = zeros(width);
    std::vector<int> used;
    const Matrix dec = rs_.data_decoder(present, &used);
    std::vector<int> missing_data;  // matrixRows: D^-1 rows of the missing data shards, ascending
    for (int i = 0; i < k_; ++i)
        if (!present[(size_t)i]) missing_data.push_back(i);
    for (int i = 0; i < nn - ne; ++i) {
        const SymBuf shard = arr[(size_t)(i + ne)];
        const int shard_index = i + ne;
        const bool first = i == 0;
        if (shard_index < k_ && first)
            for (size_t j = 0; j < missing_data.size(); ++j) outputs[j] = zeros(width);
        for (int j = 0; j < ne; ++j) {
            if (j >= (int)missing_data.size())
                throw Error(ECX_E_NULL, "decodeMissingSingle: no matrix row for a missing parity shard (isTest branch)");
            if (i >= k_) throw Error(ECX_E_INDEX, "decodeMissingSingle: index beyond the data shards (isTest branch)");
            const uint8_t c = dec.at(missing_data[(size_t)j], i);
            std::vector<uint8_t> acc = first ? std::vector<uint8_t>((size_t)width, 0) : *outputs[(size_t)j];
            axpy(acc, c, *shard);
            *outputs[(size_t)j] = std::move(acc);
        }
    }
    for (int j = 0; j < ne; ++j) plane[(size_t)erased[(size_t)j]] = outputs[(size_t)j];
}

// Body of both doDecodeSingle overloads for helper plane i (:171-203, :255-281).
void ClayPlanner::single_plane(const std::vector<SymBuf> &helper, const std::vector<int> &hidx, int i, int e,
                               std::vector<SymBuf> &outputs, int width) const {
    const int nn = n(), z = hidx[i], ey = ny(e);
    const std::vector<int> v = zvec(z);
    std::vector<SymBuf> plane(nn);
    for (int j = 0; j < q_ * t_; ++j) {  // getDecoupledHelperPlane :435-492
        const int x = nx(j), y = ny(j);
        if (y == ey) continue;
        if (v[y] == x) {
            plane[j] = helper[(size_t)i * nn + j];
        } else {
            const int cz = couple_plane(x, y, z);
            int chp = 0;
            for (size_t h = 0; h < hidx.size(); ++h)
                if (hidx[h] == cz) {
                    chp = (int)h;
                    break;
                }
            const int cc = node(v[y], y);
            plane[j] = clone(pair_couple(helper[(size_t)i * nn + j], helper[(size_t)chp * nn + cc], nullptr, nullptr,
                                         width));
        }
    }
    std::vector<int> column;
    for (int x = 0; x < q_; ++x) column.push_back(node(x, ey));
    decode_plane(plane, column, width, true);
    for (int x = 0; x < q_; ++x) {
        const int nd = node(x, ey);
        if (nd == e) {
            outputs[z] = clone(plane[nd]);
        } else {
            const int cz = couple_plane(x, ey, z);
            outputs[cz] = clone(pair_couple(nullptr, helper[(size_t)i * nn + nd], nullptr, plane[nd], width));
        }
    }
}

// doDecodeMulti (:311-421); `in` is the method's private newIn[][] copy.
void ClayPlanner::decode_multi(std::vector<SymBuf> in, std::vector<SymBuf> &outputs, int width) const {
    const int nn = n(), ne = (int)erased_.size();
    int max_is = 0;
    for (int z = 0; z < alpha_; ++z) max_is = std::max(max_is, intersection_score(z));
    for (int is = 0; is <= max_is; ++is) {
        std::vector<int> zs;
        for (int z = 0; z < alpha_; ++z)
            if (intersection_score(z) == is) zs.push_back(z);
        if (zs.empty()) continue;
        std::vector<std::vector<SymBuf>> temp(zs.size(), std::vector<SymBuf>(nn));
        for (size_t j = 0; j < zs.size(); ++j) {
            const int z = zs[j];
            const std::vector<int> v = zvec(z);
            for (int i = 0; i < q_ * t_; ++i) {  // getDecoupledPlane :500-534
                const int x = nx(i), y = ny(i);
                if (!in[(size_t)z * nn + i]) continue;
                if (v[y] == x) {
                    temp[j][i] = in[(size_t)z * nn + i];
                } else {
                    const int cz = couple_plane(x, y, z), cc = node(v[y], y);
                    temp[j][i] = clone(pair_couple(in[(size_t)z * nn + i], in[(size_t)cz * nn + cc], nullptr, nullptr,
                                                   width));
                }
            }
            decode_plane(temp[j], erased_, width);
        }
        for (size_t j = 0; j < zs.size(); ++j) {
            const int z = zs[j];
            for (int kk = 0; kk < ne; ++kk) {
                const int e = erased_[kk];
                const int type = erasure_type(e, z);
                if (type == 0) {
                    in[(size_t)z * nn + e] = temp[j][e];
                    outputs[(size_t)z * ne + kk] = clone(temp[j][e]);
                    continue;
                }
                const std::vector<int> v = zvec(z);
                const int cz = couple_plane(nx(e), ny(e), z);
                const int cidx = node(v[ny(e)], ny(e));
                SymBuf o;
                if (type == 1) {
                    o = pair_couple(nullptr, in[(size_t)cz * nn + cidx], temp[j][e], nullptr, width);
                } else {
                    auto it = std::find(zs.begin(), zs.end(), cz);
                    if (it == zs.end()) throw Error(ECX_E_INDEX, "couple plane not in the current IS batch");
                    o = pair_couple(nullptr, nullptr, temp[j][e], temp[it - zs.begin()][cidx], width);
                }
                in[(size_t)z * nn + e] = clone(o);
                outputs[(size_t)z * ne + kk] = clone(o);
            }
        }
    }
}

LinearMap ClayRepairProgram::compose(int n_in_slots, int n_out_slots) const {
    const Field &f = Field::get();
    LinearMap mp;
    mp.n_in = n_in_slots;
    mp.n_out = n_out_slots;
    for (int j = 0; j < n_in_slots; ++j) mp.in_slot.push_back(j);
    for (int o = 0; o < n_out_slots; ++o) mp.out_slot.push_back(o);
    mp.a.assign((size_t)n_in_slots * n_out_slots, 0);
    auto axpy = [&](std::vector<uint8_t> &y, uint8_t c, const std::vector<uint8_t> &x) {
        for (size_t i = 0; i < y.size(); ++i) y[i] ^= f.mul(c, x[i]);
    };
    auto unit = [&](int slot) {
        std::vector<uint8_t> v(n_in_slots, 0);
        if (slot >= 0) v[slot] = 1;
        return v;
    };
    for (int p = 0; p < n_planes; ++p) {
        const int32_t *t = table.data() + (size_t)p * stride;
        std::vector<std::vector<uint8_t>> ucol(q, std::vector<uint8_t>(n_in_slots, 0));
        for (int j = 0; j < n_noncol; ++j) {
            std::vector<uint8_t> u(n_in_slots, 0);
            axpy(u, pair_a, unit(t[j]));
            axpy(u, pair_b, unit(t[n_noncol + j]));
            for (int r = 0; r < q; ++r) axpy(ucol[r], dmat[(size_t)r * n_noncol + j], u);
        }
        const int32_t *mates = t + 2 * n_noncol, *outs = mates + (q - 1);
        auto put = [&](int slot, const std::vector<uint8_t> &row) {
            if (slot < 0 || slot >= n_out_slots) throw Error(ECX_E_ILLEGAL_ARGUMENT, "program output slot out of range");
            std::copy(row.begin(), row.end(), mp.a.begin() + (size_t)slot * n_in_slots);
        };
        put(outs[0], ucol[e_row]);
        for (int i = 0; i < q - 1; ++i) {
            std::vector<uint8_t> row(n_in_slots, 0);
            axpy(row, rc_c, unit(mates[i]));
            axpy(row, rc_u, ucol[mate_row[i]]);
            put(outs[1 + i], row);
        }
    }
    return mp;
}

ClayRepairProgram ClayPlanner::repair_program(int erased_index) const {
    const int nr = n_real(), nn = n();
    if (erased_real_.size() != 1 || erased_real_[0] != erased_index)
        throw Error(ECX_E_ILLEGAL_ARGUMENT, "repair program: the planner's erasure set must be {erased_index}");
    const int e = erased_[0], ey = ny(e);
    if (e < 0 || e >= nn || ey >= t_) throw Error(ECX_E_INDEX, "erased node outside the q x t grid");
    ClayRepairProgram pg;
    pg.q = q_;
    // the pair transform's two directions (getPairWiseCouple :630-666 as the two callers use it)
    {
        const LinearMap dec = pair_.decode_map({true, true, false, false});  // U from (C, C')
        const LinearMap rec = pair_.decode_map({false, true, false, true});  // C(z',e) from (C(z,x), U(z,x))
        auto coef = [](const LinearMap &m, int out_slot, int in_slot) -> uint8_t {
            for (int o = 0; o < m.n_out; ++o)
                if (m.out_slot[o] == out_slot)
                    for (int j = 0; j < m.n_in; ++j)
                        if (m.in_slot[j] == in_slot) return m.at(o, j);
            return 0;
        };
        pg.pair_a = coef(dec, 2, 0);
        pg.pair_b = coef(dec, 2, 1);
        pg.rc_c = coef(rec, 0, 1);
        pg.rc_u = coef(rec, 0, 3);
    }
    if ((pg.pair_a ^ pg.pair_b) != 1) throw Error(ECX_E_ILLEGAL_ARGUMENT, "pair transform without the dot identity");
    std::vector<int> noncol, column;
    for (int j = 0; j < q_ * t_; ++j) (ny(j) == ey ? column : noncol).push_back(j);
    pg.n_noncol = (int)noncol.size();
    // the plane decode: column rows from the non-column nodes (decodeMissing's map)
    std::vector<bool> present(nn, true);
    for (int j : column) present[j] = false;
    const LinearMap dm = rs_.decode_map(present);
    pg.dmat.assign((size_t)q_ * pg.n_noncol, 0);
    for (int r = 0; r < q_; ++r)
        for (int o = 0; o < dm.n_out; ++o)
            if (dm.out_slot[o] == column[r])
                for (int jj = 0; jj < dm.n_in; ++jj) {
                    const auto it = std::find(noncol.begin(), noncol.end(), dm.in_slot[jj]);
                    if (it == noncol.end()) throw Error(ECX_E_ILLEGAL_ARGUMENT, "plane decode reads a column node");
                    pg.dmat[(size_t)r * pg.n_noncol + (it - noncol.begin())] = dm.at(o, jj);
                }
    for (int r = 0; r < q_; ++r) {
        if (column[r] == e) pg.e_row = r;
        else pg.mate_row.push_back(r);
    }
    pg.t = t_;
    pg.ex = nx(e);
    pg.ey = ey;
    pg.n_real = nr;
    pg.noncol = noncol;
    pg.column = column;
    for (int u = 0; u < q_ * t_; ++u) pg.real_of.push_back(is_virtual(u) ? -1 : (u < k_ - v_ ? u : u - v_));
    // real slot of (plane z, underlying node u), -1 for a virtual node
    auto slot = [&](int z, int u) -> int {
        if (is_virtual(u)) return -1;
        const int real = u < k_ - v_ ? u : u - v_;
        return z * nr + real;
    };
    const std::vector<int> hidx = helper_planes(erased_real_[0]);
    pg.n_planes = (int)hidx.size();
    pg.stride = 2 * pg.n_noncol + 2 * q_ - 1;
    for (int z : hidx) {
        const std::vector<int> v = zvec(z);
        std::vector<int32_t> rec(pg.stride, -1);
        for (int jj = 0; jj < pg.n_noncol; ++jj) {
            const int j = noncol[jj], x = nx(j), y = ny(j);
            rec[jj] = slot(z, j);
            // a dot pairs with itself: pair_a C + pair_b C = C
            rec[pg.n_noncol + jj] = v[y] == x ? slot(z, j) : slot(couple_plane(x, y, z), node(v[y], y));
        }
        int mi = 0;
        for (int r = 0; r < q_; ++r) {
            const int nd = column[r];
            if (nd == e) {
                rec[2 * pg.n_noncol + (q_ - 1)] = z;  // output slot z * |E| + 0 (single erasure)
            } else {
                rec[2 * pg.n_noncol + mi] = slot(z, nd);
                rec[2 * pg.n_noncol + (q_ - 1) + 1 + mi] = couple_plane(nx(nd), ey, z);
                ++mi;
            }
        }
        pg.table.insert(pg.table.end(), rec.begin(), rec.end());
    }
    for (int p = 0; p < pg.n_planes; ++p) {
        const int32_t *t = pg.table.data() + (size_t)p * pg.stride;
        for (int i = 0; i < 2 * pg.n_noncol + q_ - 1; ++i) pg.max_in_slot = std::max(pg.max_in_slot, (int)t[i]);
        for (int i = 0; i < q_; ++i) pg.max_out_slot = std::max(pg.max_out_slot, (int)t[2 * pg.n_noncol + q_ - 1 + i]);
    }
    // The program must be the reference's map exactly (standard null pattern: the
    // erased node absent, every other sub-chunk present).
    std::vector<bool> pres((size_t)nr * alpha_, true);
    for (int z = 0; z < alpha_; ++z) pres[(size_t)z * nr + erased_index] = false;
    const LinearMap ref = perform_coding_map(pres);
    const LinearMap got = pg.compose(nr * alpha_, alpha_);
    if (ref.n_out != alpha_ || got.nnz() != ref.nnz())
        throw Error(ECX_E_ILLEGAL_ARGUMENT, "repair program differs from the reference map");
    for (int o = 0; o < ref.n_out; ++o) {
        if (ref.out_slot[o] != o) throw Error(ECX_E_ILLEGAL_ARGUMENT, "unexpected output order");
        for (int j = 0; j < ref.n_in; ++j)
            if (ref.at(o, j) != got.at(o, ref.in_slot[j]))
                throw Error(ECX_E_ILLEGAL_ARGUMENT, "repair program differs from the reference map");
    }
    return pg;
}

LinearMap ClayPlanner::perform_coding_map(const std::vector<bool> &input_present) const {
    const int nn = n(), nr = n_real(), ne = (int)erased_.size();
    const int width = nr * alpha_;  // symbolic inputs = the real slots
    if ((int)input_present.size() != width) throw Error(ECX_E_ILLEGAL_ARGUMENT, "Invalid inputs length");
    LinearMap mp;
    mp.n_in = width;
    for (int j = 0; j < width; ++j) mp.in_slot.push_back(j);
    if (ne == 0) return mp;
    if (std::none_of(input_present.begin(), input_present.end(), [](bool b) { return b; }))
        throw Error(ECX_E_ILLEGAL_ARGUMENT, "Invalid inputs are found, all being null");
    for (int e : erased_)
        if (e < 0 || e >= nn) throw Error(ECX_E_INDEX, "erased index out of range");
    // underlying n*alpha inputs; virtual nodes are present, all-zero buffers
    std::vector<SymBuf> in((size_t)nn * alpha_);
    for (int z = 0; z < alpha_; ++z) {
        for (int r = 0; r < nr; ++r)
            if (input_present[(size_t)z * nr + r]) in[(size_t)z * nn + under(r)] = unit(width, z * nr + r);
        for (int u = 0; u < nn; ++u)
            if (is_virtual(u)) in[(size_t)z * nn + u] = zeros(width);
    }
    std::vector<SymBuf> outputs((size_t)ne * alpha_);
    if (ne == 1) {
        const int e = erased_[0];
        const std::vector<int> hidx = helper_planes(erased_real_[0]);
        std::vector<SymBuf> helper(hidx.size() * nn);
        for (size_t h = 0; h < hidx.size(); ++h)  // getHelperPlanes :291-300
            for (int j = 0; j < nn; ++j) helper[h * nn + j] = in[(size_t)hidx[h] * nn + j];
        for (size_t i = 0; i < hidx.size(); ++i) single_plane(helper, hidx, (int)i, e, outputs, width);
    } else {
        decode_multi(in, outputs, width);
    }
    mp.n_out = ne * alpha_;
    for (int o = 0; o < mp.n_out; ++o) {
        if (!outputs[o]) throw Error(ECX_E_INDEX, "output sub-chunk never written");
        mp.out_slot.push_back(o);
        mp.a.insert(mp.a.end(), outputs[o]->begin(), outputs[o]->end());
    }
    return mp.pruned();
}

LinearMap ClayPlanner::decode_single_helper_map(const std::vector<bool> &helper_present, int helper_i,
                                                int erased_index, std::vector<bool> *written) const {
    const int nn = n(), nr = n_real();
    const std::vector<int> hidx = helper_planes(erased_index);
    const int width = (int)hidx.size() * nr;
    if ((int)helper_present.size() != width) throw Error(ECX_E_ILLEGAL_ARGUMENT, "helper plane array size");
    if (helper_i < 0 || helper_i >= (int)hidx.size()) throw Error(ECX_E_INDEX, "helper plane index");
    std::vector<SymBuf> helper(hidx.size() * nn);
    for (size_t h = 0; h < hidx.size(); ++h) {
        for (int r = 0; r < nr; ++r)
            if (helper_present[h * nr + r]) helper[h * nn + under(r)] = unit(width, (int)h * nr + r);
        for (int u = 0; u < nn; ++u)
            if (is_virtual(u)) helper[h * nn + u] = zeros(width);
    }
    std::vector<SymBuf> outputs(alpha_);
    single_plane(helper, hidx, helper_i, v_ > 0 ? under(erased_index) : erased_index, outputs, width);
    LinearMap mp;
    mp.n_in = width;
    for (int j = 0; j < width; ++j) mp.in_slot.push_back(j);
    if (written) written->assign(alpha_, false);
    for (int z = 0; z < alpha_; ++z) {
        if (!outputs[z]) continue;
        if (written) (*written)[z] = true;
        mp.out_slot.push_back(z);
        mp.a.insert(mp.a.end(), outputs[z]->begin(), outputs[z]->end());
    }
    mp.n_out = (int)mp.out_slot.size();
    return mp.pruned();
}

}  // namespace ecx
