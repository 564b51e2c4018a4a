// engine.cpp -- plan compilation, device contexts, host-pointer execution.
#include "engine.hpp"
#include "bits.hpp"
#include "map_rtc.hpp"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <exception>
#include <functional>
#include <mutex>

namespace ecx {

namespace {
Tuning g_tuning;
std::mutex g_tuning_mu;
}  // namespace

Tuning tuning() {
    std::lock_guard<std::mutex> g(g_tuning_mu);
    return g_tuning;
}

namespace {
std::atomic<int64_t> g_host_exec_max{Tuning{}.host_exec_max};  // Tuning::host_exec_max, read per call
}

void update_tuning(const std::function<void(Tuning &)> &f) {
    std::lock_guard<std::mutex> g(g_tuning_mu);
    f(g_tuning);
    g_host_exec_max.store(g_tuning.host_exec_max, std::memory_order_relaxed);
}

static thread_local std::string g_last_kernel;
namespace {
thread_local std::string g_last_shape_order;  // the unit order of the last noted launch
thread_local uint64_t g_kernel_notes = 0;
}  // namespace
void set_last_kernel(std::string name) {
    g_last_kernel = std::move(name);
    g_last_shape_order.clear();
    ++g_kernel_notes;
}
const std::string &last_kernel() { return g_last_kernel; }
uint64_t kernel_notes() { return g_kernel_notes; }
void set_last_shape_order(std::string order) { g_last_shape_order = std::move(order); }
std::string last_launch_shape() {
    return g_last_shape_order.empty() ? g_last_kernel : g_last_kernel + " " + g_last_shape_order;
}

void check_hip(hipError_t e, const char *what) {
    if (e != hipSuccess) throw Error(ECX_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

namespace {

uint32_t pack4(const uint8_t *t) {
    return (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
}

// The five split-table dwords of coefficient c (engine.hpp).
void split_tables(uint8_t c, uint32_t *out) {
    const Field &f = Field::get();
    uint8_t lo[8], mid[8], hi[4];
    for (int v = 0; v < 8; ++v) {
        lo[v] = f.mul(c, (uint8_t)v);
        mid[v] = f.mul(c, (uint8_t)(v << 3));
    }
    for (int v = 0; v < 4; ++v) hi[v] = f.mul(c, (uint8_t)(v << 6));
    out[0] = pack4(lo);
    out[1] = pack4(lo + 4);
    out[2] = pack4(mid);
    out[3] = pack4(mid + 4);
    out[4] = pack4(hi);
}

// Group output rows into tiles of kTileRows so that rows sharing inputs land in
// the same tile: every tile reads each of its inputs once, so the total tile
// entry count is the input re-read factor.  Greedy: seed each tile with the
// lowest unassigned row, then add the row with the most shared inputs (ties:
// fewest new inputs, then lowest index).  Clay(10,4) repair: 3776 -> 1280
// entries for 832 distinct inputs; single-tile maps are unchanged.
std::vector<int> group_rows(const LinearMap &m) {
    std::vector<int> order;
    if (m.n_out <= kTileRows) {
        for (int r = 0; r < m.n_out; ++r) order.push_back(r);
        return order;
    }
    std::vector<std::vector<int>> sup(m.n_out);
    for (int r = 0; r < m.n_out; ++r)
        for (int j = 0; j < m.n_in; ++j)
            if (m.at(r, j)) sup[r].push_back(j);
    std::vector<char> used(m.n_out, 0), in_tile(m.n_in, 0);
    for (int seed = 0; seed < m.n_out; ++seed) {
        if (used[seed]) continue;
        std::vector<int> tile = {seed};
        used[seed] = 1;
        std::fill(in_tile.begin(), in_tile.end(), 0);
        for (int j : sup[seed]) in_tile[j] = 1;
        while ((int)tile.size() < kTileRows) {
            int best = -1, best_shared = -1, best_new = 0;
            for (int r = 0; r < m.n_out; ++r) {
                if (used[r]) continue;
                int shared = 0;
                for (int j : sup[r]) shared += in_tile[j];
                const int fresh = (int)sup[r].size() - shared;
                if (shared - fresh > best_shared - best_new || best < 0) {
                    best = r;
                    best_shared = shared;
                    best_new = fresh;
                }
            }
            if (best < 0) break;
            used[best] = 1;
            tile.push_back(best);
            for (int j : sup[best]) in_tile[j] = 1;
        }
        order.insert(order.end(), tile.begin(), tile.end());
    }
    return order;
}

// Group tiles that share inputs into workgroups of up to kWaveGroup tiles (one
// wave each, k_gf_apply_lds): seed with the lowest unassigned tile, then add
// the unassigned tile sharing the most inputs with the group (ties: lowest index).
// Clay(10,4) repair: the 32 tiles form 4 groups of 8 in which every pair shares
// 4 inputs -- each group reads its 208 distinct inputs, 832 in all.
std::vector<std::vector<int>> group_tiles(const std::vector<std::vector<int>> &cols, int n_in) {
    const int n = (int)cols.size();
    std::vector<std::vector<int>> groups;
    std::vector<char> used(n, 0), in_group(n_in, 0);
    for (int seed = 0; seed < n; ++seed) {
        if (used[seed]) continue;
        std::vector<int> g = {seed};
        used[seed] = 1;
        std::fill(in_group.begin(), in_group.end(), 0);
        for (int j : cols[seed]) in_group[j] = 1;
        while ((int)g.size() < kWaveGroup) {
            int best = -1, best_shared = -1;
            for (int t = 0; t < n; ++t) {
                if (used[t]) continue;
                int shared = 0;
                for (int j : cols[t]) shared += in_group[j];
                if (shared > best_shared) {
                    best = t;
                    best_shared = shared;
                }
            }
            if (best < 0 || best_shared == 0) break;
            used[best] = 1;
            g.push_back(best);
            for (int j : cols[best]) in_group[j] = 1;
        }
        groups.push_back(g);
    }
    return groups;
}

// Schedule a group's inputs so that every stage of k_gf_apply_lds (one input per
// wave, staged through LDS) gives each tile about the same amount of work: greedy
// list scheduling, shared inputs first (most sharers first), each into the
// earliest slot free in every tile that uses it; private inputs fill the holes.
// Returns the group's union of inputs in schedule order (slot, then column): the
// order in which k_gf_apply_lds stages them through LDS.  Every tile's list is
// increasing in that order.
std::vector<int> align_group(const std::vector<int> &group, std::vector<std::vector<int>> &cols) {
    std::map<int, std::vector<int>> users;  // input column -> tiles of the group using it
    for (int t : group)
        for (int j : cols[t]) users[j].push_back(t);
    std::vector<std::pair<int, int>> order;  // (-#users, column)
    for (auto &kv : users) order.push_back({-(int)kv.second.size(), kv.first});
    std::sort(order.begin(), order.end());
    std::map<int, std::vector<char>> busy;  // tile -> slot occupancy
    std::map<int, std::vector<std::pair<int, int>>> placed;  // tile -> (slot, column)
    for (auto &oc : order) {
        const int j = oc.second;
        const std::vector<int> &ts = users[j];
        for (int slot = 0;; ++slot) {
            bool free = true;
            for (int t : ts) {
                std::vector<char> &b = busy[t];
                if ((int)b.size() > slot && b[slot]) {
                    free = false;
                    break;
                }
            }
            if (!free) continue;
            for (int t : ts) {
                std::vector<char> &b = busy[t];
                if ((int)b.size() <= slot) b.resize(slot + 1, 0);
                b[slot] = 1;
                placed[t].push_back({slot, j});
            }
            break;
        }
    }
    std::map<int, int> slot_of;
    for (int t : group) {
        std::vector<std::pair<int, int>> &p = placed[t];
        std::sort(p.begin(), p.end());
        cols[t].clear();
        for (auto &sj : p) {
            cols[t].push_back(sj.second);
            slot_of[sj.second] = sj.first;
        }
    }
    std::vector<std::pair<int, int>> u;
    for (auto &kv : slot_of) u.push_back({kv.second, kv.first});
    std::sort(u.begin(), u.end());
    std::vector<int> uni;
    for (auto &sj : u) uni.push_back(sj.second);
    return uni;
}

}  // namespace

CompiledMap::CompiledMap(LinearMap m) : map_(std::move(m)) {
    for (int s : map_.in_slot) max_in_slot_ = std::max(max_in_slot_, s);
    for (int s : map_.out_slot) max_out_slot_ = std::max(max_out_slot_, s);
    const std::vector<int> order = group_rows(map_);
    // Tiles of kTileRows output rows and the input columns each one reads.
    std::vector<std::vector<int>> cols;
    for (int r0 = 0; r0 < map_.n_out; r0 += kTileRows) {
        const int rows = std::min(kTileRows, map_.n_out - r0);
        std::vector<int> c;
        for (int j = 0; j < map_.n_in; ++j) {
            bool any = false;
            for (int r = 0; r < rows; ++r) any |= map_.at(order[r0 + r], j) != 0;
            if (any) c.push_back(j);
        }
        cols.push_back(c);
    }
    n_tiles_ = (int)cols.size();
    // (tile, column) -> position in the tile's group union; a column read by
    // several groups has a different position in each.
    std::vector<std::map<int, int>> upos(n_tiles_);
    if (n_tiles_ > 1) {
        for (const std::vector<int> &g : group_tiles(cols, map_.n_in)) {
            const std::vector<int> uni = align_group(g, cols);
            std::map<int, int> pos;
            for (size_t u = 0; u < uni.size(); ++u) pos[uni[u]] = (int)u;
            for (int t : g) upos[t] = pos;
            uint32_t rec[kGroupDwords];
            std::fill(rec, rec + kGroupDwords, 0u);
            for (int w = 0; w < kWaveGroup; ++w) rec[w] = w < (int)g.size() ? (uint32_t)g[w] : kNoTile;
            rec[8] = (uint32_t)unions_.size();
            rec[9] = (uint32_t)uni.size();
            for (size_t u = 0; u < uni.size(); ++u) unions_.push_back((uint32_t)map_.in_slot[uni[u]]);
            groups_.insert(groups_.end(), rec, rec + kGroupDwords);
            group_size_ = std::max(group_size_, (int)g.size());
            ++n_groups_;
        }
    }
    for (int t = 0; t < n_tiles_; ++t) {
        const int r0 = t * kTileRows;
        const int rows = std::min(kTileRows, map_.n_out - r0);
        const uint32_t begin = (uint32_t)(entries_.size() / kEntryDwords);
        for (int j : cols[t]) {
            uint32_t mmul = 0, mone = 0;
            for (int r = 0; r < rows; ++r) {
                const uint8_t c = map_.at(order[r0 + r], j);
                if (c == 1) mone |= 1u << r;
                else if (c) mmul |= 1u << r;
            }
            uint32_t rec[kEntryDwords] = {0};
            rec[0] = (uint32_t)map_.in_slot[j];
            rec[1] = mmul;
            rec[2] = mone;
            rec[3] = n_tiles_ > 1 ? (uint32_t)upos[t].at(j) : 0u;
            for (int r = 0; r < rows; ++r)
                if (mmul & (1u << r)) split_tables(map_.at(order[r0 + r], j), rec + 4 + 5 * r);
            entries_.insert(entries_.end(), rec, rec + kEntryDwords);
        }
        uint32_t tile[kTileDwords] = {0};
        tile[0] = begin;
        tile[1] = (uint32_t)cols[t].size();
        tile[2] = (uint32_t)rows;
        tile[3] = (uint32_t)cols[t].size();  // unpadded count (k_gf_apply_lds)
        max_tile_rows_ = std::max(max_tile_rows_, rows);
        for (int r = 0; r < rows; ++r) tile[4 + r] = (uint32_t)map_.out_slot[order[r0 + r]];
        tiles_.insert(tiles_.end(), tile, tile + kTileDwords);
    }
    // Wide tiles: pair the 8-row tiles greedily by shared inputs (ties: lowest index);
    // each pair's entries run over the sorted union of the two tiles' input columns.
    if (n_tiles_ > 1) {
        std::vector<std::map<int, uint32_t>> entry_of(n_tiles_);  // column -> entry index
        for (int t = 0; t < n_tiles_; ++t) {
            const uint32_t b = tiles_[(size_t)t * kTileDwords], n = tiles_[(size_t)t * kTileDwords + 1];
            for (uint32_t e = 0; e < n; ++e) entry_of[t][cols[t][e]] = b + e;
        }
        std::vector<char> paired(n_tiles_, 0);
        int min_count = 1 << 30;
        for (int a = 0; a < n_tiles_; ++a) {
            if (paired[a]) continue;
            paired[a] = 1;
            int b = -1, best = -1;
            for (int t = 0; t < n_tiles_; ++t) {
                if (paired[t]) continue;
                int shared = 0;
                for (auto &kv : entry_of[t]) shared += entry_of[a].count(kv.first) ? 1 : 0;
                if (shared > best) {
                    best = shared;
                    b = t;
                }
            }
            if (b >= 0) paired[b] = 1;
            std::vector<int> uni;
            for (auto &kv : entry_of[a]) uni.push_back(kv.first);
            if (b >= 0)
                for (auto &kv : entry_of[b]) uni.push_back(kv.first);
            std::sort(uni.begin(), uni.end());
            uni.erase(std::unique(uni.begin(), uni.end()), uni.end());
            uint32_t rec[kWideTileDwords] = {0};
            rec[0] = (uint32_t)(wentries_.size() / kWideEntryDwords);
            rec[1] = (uint32_t)uni.size();
            rec[2] = tiles_[(size_t)a * kTileDwords + 2];
            rec[3] = b >= 0 ? tiles_[(size_t)b * kTileDwords + 2] : 0u;
            for (int r = 0; r < kTileRows; ++r) {
                rec[4 + r] = tiles_[(size_t)a * kTileDwords + 4 + r];
                rec[12 + r] = b >= 0 ? tiles_[(size_t)b * kTileDwords + 4 + r] : 0u;
            }
            for (int j : uni) {
                for (int half = 0; half < 2; ++half) {
                    const int t = half == 0 ? a : b;
                    uint32_t e[kEntryDwords] = {0};
                    e[0] = (uint32_t)map_.in_slot[j];
                    if (t >= 0) {
                        auto it = entry_of[t].find(j);
                        if (it != entry_of[t].end()) {
                            std::copy(entries_.begin() + (size_t)it->second * kEntryDwords,
                                      entries_.begin() + (size_t)(it->second + 1) * kEntryDwords, e);
                            e[3] = 0;
                        }
                    }
                    wentries_.insert(wentries_.end(), e, e + kEntryDwords);
                }
            }
            wtiles_.insert(wtiles_.end(), rec, rec + kWideTileDwords);
            wide_reads_ += (int64_t)entry_of[a].size() + (b >= 0 ? (int64_t)entry_of[b].size() : 0);
            wide_union_ += (int64_t)uni.size();
            min_count = std::min(min_count, (int)uni.size());
            ++n_wide_;
        }
        wide_depth_ = min_count >= 12 ? 8 : 4;
    }
    if (tiles_.empty()) tiles_.assign(kTileDwords, 0);
    if (entries_.empty()) entries_.assign(kEntryDwords, 0);
    if (groups_.empty()) {
        groups_.assign(kGroupDwords, 0u);
        std::fill(groups_.begin(), groups_.begin() + kWaveGroup, kNoTile);
    }
    int min_count = 1 << 30;
    for (int t = 0; t < n_tiles_; ++t) {
        const int c = (int)tiles_[(size_t)t * kTileDwords + 1];
        if (c > 0) min_count = std::min(min_count, c);
    }
    preferred_depth_ = (min_count != (1 << 30) && min_count >= 12) ? 8 : 4;
    // A single full (8-row) tile of 17-20 entries -- every Clay(4,2) single repair
    // (20 helper sub-chunks) -- runs best with all of its loads in flight at once:
    // a 20-deep ring, no refill, 3 waves/SIMD (+2.3-2.9 % over depth 8 in interleaved
    // runs, scripts/depth_bench.py, profiles/r01_depth.jsonl).  Shorter or narrower
    // tiles (RS decode, LRC) measured flat or slower with deep rings.
    if (n_tiles_ == 1 && max_tile_rows_ == kTileRows && min_count > 16 && min_count <= 20) preferred_depth_ = 20;
}

void CompiledMap::emulate(const uint8_t *in, uint8_t *out, int64_t len, bool via_unions) const {
    auto table_byte = [](const uint32_t *t, int idx) { return (uint8_t)(t[idx >> 2] >> (8 * (idx & 3))); };
    std::vector<int> group_of(n_tiles_, -1);
    for (int g = 0; g < n_groups_; ++g)
        for (int w = 0; w < kWaveGroup; ++w)
            if (groups_[(size_t)g * kGroupDwords + w] != kNoTile) group_of[groups_[(size_t)g * kGroupDwords + w]] = g;
    std::vector<uint8_t> acc((size_t)kTileRows * len);
    for (int t = 0; t < n_tiles_; ++t) {
        const uint32_t *tile = tiles_.data() + (size_t)t * kTileDwords;
        std::fill(acc.begin(), acc.end(), 0);
        uint32_t prev = 0;
        for (uint32_t e = 0; e < tile[1]; ++e) {
            const uint32_t *rec = entries_.data() + (size_t)(tile[0] + e) * kEntryDwords;
            uint32_t slot = rec[0];
            if (via_unions && n_tiles_ > 1) {
                const int g = group_of[t];
                if (g < 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "tile without a group");
                const uint32_t *grp = groups_.data() + (size_t)g * kGroupDwords;
                if (rec[3] >= grp[9] || (e > 0 && rec[3] <= prev))
                    throw Error(ECX_E_ILLEGAL_ARGUMENT, "union positions not increasing within a tile");
                prev = rec[3];
                slot = unions_[grp[8] + rec[3]];
                if (slot != rec[0]) throw Error(ECX_E_ILLEGAL_ARGUMENT, "union position names another input");
            }
            const uint8_t *x = in + (int64_t)slot * len;
            for (int r = 0; r < (int)tile[2]; ++r) {
                uint8_t *a = acc.data() + (size_t)r * len;
                if (rec[2] & (1u << r))
                    for (int64_t i = 0; i < len; ++i) a[i] ^= x[i];
                if (rec[1] & (1u << r)) {
                    const uint32_t *tb = rec + 4 + 5 * r;
                    for (int64_t i = 0; i < len; ++i)
                        a[i] ^= table_byte(tb, x[i] & 7) ^ table_byte(tb + 2, (x[i] >> 3) & 7) ^ table_byte(tb + 4, x[i] >> 6);
                }
            }
        }
        for (int r = 0; r < (int)tile[2]; ++r)
            std::copy(acc.begin() + (size_t)r * len, acc.begin() + (size_t)(r + 1) * len, out + (int64_t)tile[4 + r] * len);
    }
}

const uint8_t *zero_page_for_current_device() {
    static std::mutex mu;
    static std::map<int, uint8_t *> pages;
    int dev = 0;
    check_hip(hipGetDevice(&dev), "hipGetDevice");
    std::lock_guard<std::mutex> lk(mu);
    uint8_t *&p = pages[dev];
    if (!p) {
        check_hip(hipMalloc(&p, 4096), "hipMalloc(zero page)");
        check_hip(hipMemset(p, 0, 4096), "hipMemset(zero page)");
    }
    return p;
}

CompiledMap::~CompiledMap() {
    for (auto &kv : layout_sel_) {
        for (auto &p : kv.second.pending) {
            if (p.e1) close_probe(p.dev, p.e1);
            if (p.e0) (void)hipEventDestroy(p.e0);
            if (p.e1) (void)hipEventDestroy(p.e1);
        }
    }
    for (auto &kv : dev_) {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) continue;
        (void)hipSetDevice(kv.first.first);
        (void)hipFree(kv.second.entries);
        (void)hipFree(kv.second.tiles);
        (void)hipFree(kv.second.groups);
        (void)hipFree(kv.second.unions);
        (void)hipFree(kv.second.atab);
        (void)hipFree(kv.second.wentries);
        (void)hipFree(kv.second.wtiles);
        (void)hipFree(kv.second.bentries);
        (void)hipSetDevice(cur);
    }
}

HostPlan CompiledMap::padded_plan(int depth) const {
    HostPlan p;
    // Pad each tile to a multiple of `depth` entries so the kernel's load ring
    // runs branch-free (engine.hpp); padding entries load the zero page.
    p.tiles = tiles_;
    for (int t = 0; t < n_tiles_; ++t) {
        uint32_t *tile = p.tiles.data() + (size_t)t * kTileDwords;
        const uint32_t begin = tile[0], count = tile[1];
        tile[0] = (uint32_t)(p.entries.size() / kEntryDwords);
        p.entries.insert(p.entries.end(), entries_.begin() + (size_t)begin * kEntryDwords,
                         entries_.begin() + (size_t)(begin + count) * kEntryDwords);
        const uint32_t padded = count == 0 ? 0 : (count + depth - 1) / depth * depth;
        for (uint32_t d = count; d < padded; ++d) {
            uint32_t rec[kEntryDwords] = {0};
            rec[0] = kDummySlot;
            p.entries.insert(p.entries.end(), rec, rec + kEntryDwords);
        }
        tile[1] = padded;
        p.max_tile_entries = std::max(p.max_tile_entries, (int)padded);
    }
    if (p.entries.empty()) p.entries.assign(kEntryDwords, 0);
    for (size_t e = 0; e < p.entries.size() / kEntryDwords; ++e)
        for (int r = 0; r < kTileRows; ++r) {
            p.atab.push_back(p.entries[e * kEntryDwords + 4 + 5 * r]);      // T0a
            p.atab.push_back(p.entries[e * kEntryDwords + 4 + 5 * r + 2]);  // T1a
        }
    // Bit-sliced entries (k_gf_bits, diagnostic build only): the coefficient of each row,
    // recovered from its table (T0a byte 1 = c * 1), or 1 for a plain-XOR row.
    for (size_t e = 0; ECX_DIAG && e < p.entries.size() / kEntryDwords; ++e) {
        const uint32_t *rec = p.entries.data() + e * kEntryDwords;
        uint32_t coef[2] = {0u, 0u};
        for (int r = 0; r < kTileRows; ++r) {
            const uint32_t c = (rec[2] >> r) & 1u ? 1u : ((rec[1] >> r) & 1u ? (rec[4 + 5 * r] >> 8) & 0xFFu : 0u);
            coef[r >> 2] |= c << (8 * (r & 3));
        }
        p.bentries.push_back(rec[0]);
        p.bentries.push_back(rec[1] | rec[2]);
        p.bentries.push_back(coef[0]);
        p.bentries.push_back(coef[1]);
    }
    // Unions: each group's list padded with zero-page entries to a multiple of
    // group_size * depth, i.e. whole stages of the LDS kernel's load ring.
    p.groups = groups_;
    const int gsz = std::max(1, group_size_);
    for (int g = 0; g < n_groups_; ++g) {
        uint32_t *rec = p.groups.data() + (size_t)g * kGroupDwords;
        const uint32_t begin = rec[8], count = rec[9];
        rec[8] = (uint32_t)p.unions.size();
        p.unions.insert(p.unions.end(), unions_.begin() + begin, unions_.begin() + begin + count);
        const uint32_t quantum = (uint32_t)(gsz * depth);
        const uint32_t padded = (count + quantum - 1) / quantum * quantum;
        p.unions.resize(p.unions.size() + (padded - count), kDummySlot);
        rec[9] = padded;
    }
    if (p.unions.empty()) p.unions.assign(1, kDummySlot);
    // Wide tiles: entry lists padded to a multiple of `depth` with zero-page pairs.
    p.wtiles = wtiles_;
    for (int w = 0; w < n_wide_; ++w) {
        uint32_t *rec = p.wtiles.data() + (size_t)w * kWideTileDwords;
        const uint32_t begin = rec[0], count = rec[1];
        rec[0] = (uint32_t)(p.wentries.size() / kWideEntryDwords);
        p.wentries.insert(p.wentries.end(), wentries_.begin() + (size_t)begin * kWideEntryDwords,
                          wentries_.begin() + (size_t)(begin + count) * kWideEntryDwords);
        const uint32_t padded = count == 0 ? 0 : (count + depth - 1) / depth * depth;
        for (uint32_t d = count; d < padded; ++d) {
            uint32_t e[kWideEntryDwords] = {0};
            e[0] = e[kEntryDwords] = kDummySlot;
            p.wentries.insert(p.wentries.end(), e, e + kWideEntryDwords);
        }
        rec[1] = padded;
    }
    if (p.wentries.empty()) p.wentries.assign(kWideEntryDwords, 0);
    if (p.wtiles.empty()) p.wtiles.assign(kWideTileDwords, 0);
    return p;
}

void CompiledMap::emulate_wide(const HostPlan &p, const uint8_t *in, uint8_t *out, int64_t len) const {
    auto table_byte = [](uint32_t lo, uint32_t hi, int idx) {
        return (uint8_t)((idx < 4 ? lo : hi) >> (8 * (idx & 3)));
    };
    std::vector<uint8_t> acc((size_t)2 * kTileRows * len);
    for (int w = 0; w < n_wide_; ++w) {
        const uint32_t *rec = p.wtiles.data() + (size_t)w * kWideTileDwords;
        std::fill(acc.begin(), acc.end(), 0);
        if (rec[1] % 4) throw Error(ECX_E_ILLEGAL_ARGUMENT, "wide tile not padded to the ring depth");
        for (uint32_t e = 0; e < rec[1]; ++e) {
            const uint32_t *we = p.wentries.data() + ((size_t)rec[0] + e) * kWideEntryDwords;
            if (we[0] != we[kEntryDwords]) throw Error(ECX_E_ILLEGAL_ARGUMENT, "wide entry halves name different inputs");
            if (we[0] == kDummySlot) {
                if (we[1] | we[2] | we[kEntryDwords + 1] | we[kEntryDwords + 2])
                    throw Error(ECX_E_ILLEGAL_ARGUMENT, "padding entry with coefficients");
                continue;
            }
            const uint8_t *x = in + (int64_t)we[0] * len;
            for (int half = 0; half < 2; ++half) {
                const uint32_t *r = we + half * kEntryDwords;
                for (int o = 0; o < kTileRows; ++o) {
                    uint8_t *a = acc.data() + (size_t)(half * kTileRows + o) * len;
                    if (r[2] & (1u << o))
                        for (int64_t i = 0; i < len; ++i) a[i] ^= x[i];
                    if (r[1] & (1u << o)) {
                        const uint32_t *tb = r + 4 + 5 * o;
                        for (int64_t i = 0; i < len; ++i)
                            a[i] ^= table_byte(tb[0], tb[1], x[i] & 7) ^ table_byte(tb[2], tb[3], (x[i] >> 3) & 7) ^
                                    table_byte(tb[4], tb[4], x[i] >> 6);
                    }
                }
            }
        }
        for (int half = 0; half < 2; ++half)
            for (uint32_t o = 0; o < rec[2 + half]; ++o)
                std::copy(acc.begin() + (size_t)(half * kTileRows + o) * len,
                          acc.begin() + (size_t)(half * kTileRows + o + 1) * len,
                          out + (int64_t)rec[4 + 8 * half + o] * len);
    }
}

void CompiledMap::emulate_padded(const HostPlan &p, const uint8_t *in, uint8_t *out, int64_t len, bool tlds,
                                 int depth) const {
    auto table_byte = [](uint32_t lo, uint32_t hi, int idx) {
        return (uint8_t)((idx < 4 ? lo : hi) >> (8 * (idx & 3)));
    };
    std::vector<uint8_t> acc((size_t)kTileRows * len);
    for (int t = 0; t < n_tiles_; ++t) {
        const uint32_t *tile = p.tiles.data() + (size_t)t * kTileDwords;
        std::fill(acc.begin(), acc.end(), 0);
        if (tile[1] % depth) throw Error(ECX_E_ILLEGAL_ARGUMENT, "tile entry count not padded to the ring depth");
        for (uint32_t e = 0; e < tile[1]; ++e) {
            const size_t ei = (size_t)tile[0] + e;
            const uint32_t *rec = p.entries.data() + ei * kEntryDwords;
            if (rec[0] == kDummySlot) {
                if (rec[1] | rec[2]) throw Error(ECX_E_ILLEGAL_ARGUMENT, "padding entry with coefficients");
                continue;  // reads the zero page: contributes nothing
            }
            const uint8_t *x = in + (int64_t)rec[0] * len;
            for (int r = 0; r < (int)tile[2]; ++r) {
                uint8_t *a = acc.data() + (size_t)r * len;
                if (rec[2] & (1u << r))
                    for (int64_t i = 0; i < len; ++i) a[i] ^= x[i];
                if (rec[1] & (1u << r)) {
                    const uint32_t *tb = rec + 4 + 5 * r;
                    const uint32_t t0a = tlds ? p.atab[ei * kAtabDwords + 2 * r] : tb[0];
                    const uint32_t t1a = tlds ? p.atab[ei * kAtabDwords + 2 * r + 1] : tb[2];
                    for (int64_t i = 0; i < len; ++i)
                        a[i] ^= table_byte(t0a, tb[1], x[i] & 7) ^ table_byte(t1a, tb[3], (x[i] >> 3) & 7) ^
                                table_byte(tb[4], tb[4], x[i] >> 6);
                }
            }
        }
        for (int r = 0; r < (int)tile[2]; ++r)
            std::copy(acc.begin() + (size_t)r * len, acc.begin() + (size_t)(r + 1) * len, out + (int64_t)tile[4 + r] * len);
    }
}

void CompiledMap::emulate_bits(const HostPlan &p, const uint8_t *in, uint8_t *out, int64_t len) const {
    if (len % kChunkBytes) throw Error(ECX_E_ILLEGAL_ARGUMENT, "bit-sliced emulation needs whole 4 KiB chunks");
    const bits::Masks mk{0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
    auto get = [](const uint8_t *b) { return (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24; };
    for (int t = 0; t < n_tiles_; ++t) {
        const uint32_t *tile = p.tiles.data() + (size_t)t * kTileDwords;
        for (int64_t c = 0; c < len; c += kChunkBytes)
            for (int lane = 0; lane < kBitsThreads; ++lane) {
                // the lane's 32 bytes: [16 l, 16 l + 16) and [2048 + 16 l, ...) of the chunk
                const int64_t off[2] = {c + 16 * lane, c + kChunkBytes / 2 + 16 * lane};
                uint32_t acc[8][8] = {};
                for (uint32_t e = 0; e < tile[1]; ++e) {
                    const uint32_t *r = p.bentries.data() + ((size_t)tile[0] + e) * kBitsEntryDwords;
                    if (!r[1]) continue;
                    if (r[0] == kDummySlot) throw Error(ECX_E_ILLEGAL_ARGUMENT, "padding entry with coefficients");
                    uint32_t x[8];
                    for (int h = 0; h < 2; ++h)
                        for (int d = 0; d < 4; ++d) x[4 * h + d] = get(in + (int64_t)r[0] * len + off[h] + 4 * d);
                    bits::transpose8(x, mk);
                    bits::apply_entry_bits(acc, x, r[1], r[2], r[3]);
                }
                for (int o = 0; o < (int)tile[2]; ++o) {
                    bits::untranspose8(acc[o], mk);
                    for (int h = 0; h < 2; ++h)
                        for (int d = 0; d < 4; ++d)
                            for (int b = 0; b < 4; ++b)
                                out[(int64_t)tile[4 + o] * len + off[h] + 4 * d + b] = (uint8_t)(acc[o][4 * h + d] >> (8 * b));
                }
            }
    }
}

const DevicePlan &CompiledMap::plan_for_current_device(int depth) {
    int dev = 0;
    check_hip(hipGetDevice(&dev), "hipGetDevice");
    std::lock_guard<std::mutex> lk(mu_);
    auto it = dev_.find({dev, depth});
    if (it != dev_.end()) return it->second;
    const HostPlan h = padded_plan(depth);
    DevicePlan p;
    p.max_tile_entries = h.max_tile_entries;
    auto upload = [](uint32_t **dst, const std::vector<uint32_t> &src, const char *what) {
        check_hip(hipMalloc(dst, src.size() * 4), what);
        check_hip(hipMemcpy(*dst, src.data(), src.size() * 4, hipMemcpyHostToDevice), "plan upload");
    };
    upload(&p.entries, h.entries, "hipMalloc(plan entries)");
    upload(&p.tiles, h.tiles, "hipMalloc(plan tiles)");
    upload(&p.groups, h.groups, "hipMalloc(plan groups)");
    upload(&p.unions, h.unions, "hipMalloc(plan unions)");
    upload(&p.atab, h.atab, "hipMalloc(plan atab)");
    upload(&p.wentries, h.wentries, "hipMalloc(plan wide entries)");
    upload(&p.wtiles, h.wtiles, "hipMalloc(plan wide tiles)");
    if (!h.bentries.empty()) upload(&p.bentries, h.bentries, "hipMalloc(plan bit-sliced entries)");
    return dev_.emplace(std::make_pair(dev, depth), p).first->second;
}

namespace {
std::vector<int> sorted_unique(std::vector<int> v) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    return v;
}
int rank_of(const std::vector<int> &sorted, int slot) {
    return (int)(std::lower_bound(sorted.begin(), sorted.end(), slot) - sorted.begin());
}
}  // namespace

CompiledMap &CompiledMap::compact() {
    std::lock_guard<std::mutex> lk(mu_);
    if (!compact_) {
        used_in_ = sorted_unique(map_.in_slot);
        used_out_ = sorted_unique(map_.out_slot);
        LinearMap c = map_;
        for (int &s : c.in_slot) s = rank_of(used_in_, s);
        for (int &s : c.out_slot) s = rank_of(used_out_, s);
        compact_ = std::make_unique<CompiledMap>(std::move(c));
    }
    return *compact_;
}

MapPlanes *CompiledMap::planes() {
    std::lock_guard<std::mutex> lk(mu_);
    if (!planes_checked_) {
        planes_checked_ = true;
        if (map_planes_supported(map_)) planes_ = std::make_unique<MapPlanes>(map_);
    }
    return planes_.get();
}

namespace {
constexpr float kLayoutMargin = 0.98f;   // another shape replaces the static rules' only if 2 % faster
constexpr size_t kMaxLayouts = 64;       // layouts selected per map; past that, new ones use the static rules
constexpr int kLayoutMaxDropped = 64;    // contaminated probes before a layout is declared contended
constexpr int64_t kLayoutRevalidate = 512;  // launches after a choice before its one re-validation

float median_of(std::vector<float> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? -1.f : v[v.size() / 2];
}

// A filled layout probe still open to contamination: until a launch on another stream of its
// device finds its end event done, such a launch may share the GPU with it (`dirty`).
struct OpenProbe {
    hipStream_t stream;
    hipEvent_t e1;
    std::shared_ptr<std::atomic<bool>> dirty;
};
// A stream's launches: the latest one's serial, and an event recorded behind its latest LARGE
// launch (>= kMarkBytes of input), so a probe can tell whether one may still run.  A smaller
// launch runs for microseconds, negligible against a multi-millisecond probe, and is not marked.
struct StreamMark {
    uint64_t serial = 0;
    hipEvent_t done = nullptr;
    bool marked = false;  // `done` was recorded behind a large launch of this stream
};
constexpr int64_t kMarkBytes = 64 << 20;
constexpr uint64_t kUnmarkedLarge = 1ull << 63;  // serial flag: a large launch whose event failed
struct DevLaunches {
    uint64_t serial = 0;
    std::map<hipStream_t, StreamMark> last;  // aged out, below
    std::vector<OpenProbe> open;
};
constexpr uint64_t kStreamAge = 4096;  // a stream silent for this many launches leaves `last`
std::mutex g_launch_mu;
std::map<int, DevLaunches> g_launches;
}  // namespace

uint64_t note_device_launch(int dev, hipStream_t s, int64_t bytes) {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    DevLaunches &d = g_launches[dev];
    StreamMark &mk = d.last[s];
    mk.serial = ++d.serial;
    if (bytes >= kMarkBytes) {
        if (!mk.done && hipEventCreateWithFlags(&mk.done, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            mk.done = nullptr;
        }
        // unmarked when the record fails: this large launch then counts as possibly running
        mk.marked = mk.done && hipEventRecord(mk.done, s) == hipSuccess;
        if (!mk.marked) {
            (void)hipGetLastError();
            mk.serial |= kUnmarkedLarge;
        }
    }
    // An open probe on another stream, at a large launch: still running -> this launch may
    // overlap it (dirty); finished -> no later launch can, so its window closes here.  Either way
    // it leaves the list.
    for (auto it = d.open.begin(); bytes >= kMarkBytes && it != d.open.end();) {
        if (it->stream == s) {  // same stream: queued behind the probe
            ++it;
            continue;
        }
        const hipError_t q = hipEventQuery(it->e1);
        if (q == hipErrorNotReady) it->dirty->store(true);
        else if (q != hipSuccess) (void)hipGetLastError();
        it = d.open.erase(it);
    }
    if (d.serial % 256 == 0)  // bounded: streams not seen for kStreamAge launches are forgotten
        for (auto it = d.last.begin(); it != d.last.end();) {
            if ((it->second.serial & ~kUnmarkedLarge) + kStreamAge >= d.serial) {
                ++it;
                continue;
            }
            if (it->second.done) (void)hipEventDestroy(it->second.done);
            it = d.last.erase(it);
        }
    return d.serial;
}

uint64_t stream_last_launch(int dev, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    auto it = g_launches.find(dev);
    if (it == g_launches.end()) return 0;
    auto jt = it->second.last.find(s);
    return jt == it->second.last.end() ? 0 : jt->second.serial & ~kUnmarkedLarge;
}

bool other_stream_may_run(int dev, hipStream_t s, uint64_t since) {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    auto it = g_launches.find(dev);
    if (it == g_launches.end()) return false;
    for (const auto &kv : it->second.last) {
        if (kv.first == s) continue;
        const StreamMark &mk = kv.second;
        if (mk.serial & kUnmarkedLarge) {  // a large launch without an event: assume it may run
            if ((mk.serial & ~kUnmarkedLarge) > since) return true;
        } else if (mk.marked) {  // its latest large launch: running iff the event is not done
            const hipError_t q = hipEventQuery(mk.done);
            if (q == hipErrorNotReady) return true;
            if (q != hipSuccess) (void)hipGetLastError();
        }
    }
    return false;
}

std::shared_ptr<std::atomic<bool>> open_probe(int dev, hipStream_t s, hipEvent_t e1, bool dirty) {
    auto flag = std::make_shared<std::atomic<bool>>(dirty);
    std::lock_guard<std::mutex> lk(g_launch_mu);
    if (!dirty) g_launches[dev].open.push_back({s, e1, flag});
    return flag;
}

void close_probe(int dev, hipEvent_t e1) {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    auto it = g_launches.find(dev);
    if (it == g_launches.end()) return;
    auto &v = it->second.open;
    for (auto jt = v.begin(); jt != v.end(); ++jt)
        if (jt->e1 == e1) {
            v.erase(jt);
            return;
        }
}

// Reads the finished probes of `s` (non-blocking): clean timings go to the exploration's
// per-candidate lists, or to the re-validation's pair; contaminated ones are counted and dropped.
void CompiledMap::harvest(LayoutSel &s, int n_cand) {
    for (auto it = s.pending.begin(); it != s.pending.end();) {
        if (!it->e1) {  // reserved, not yet launched
            ++it;
            continue;
        }
        const hipError_t q = hipEventQuery(it->e1);
        if (q == hipErrorNotReady) {
            ++it;
            continue;
        }
        float ms = 0.f;
        const bool timed = q == hipSuccess && hipEventElapsedTime(&ms, it->e0, it->e1) == hipSuccess && ms > 0.f;
        close_probe(it->dev, it->e1);  // before its events go
        if (!timed) (void)hipGetLastError();  // a failed probe is dropped; its candidate is timed again
        else if (it->dirty && it->dirty->load()) ++s.dropped;
        else if (s.state == kLayoutRevalidating) {
            if (it->cand == s.reval_alt) s.reval_ms[0].push_back(ms);
            else if (it->cand == s.chosen) s.reval_ms[1].push_back(ms);
        } else if (s.state == kLayoutExploring && it->cand < n_cand) {
            s.ms[it->cand].push_back(ms);
        }
        (void)hipEventDestroy(it->e0);
        (void)hipEventDestroy(it->e1);
        it = s.pending.erase(it);
    }
}

int CompiledMap::next_layout_pick(const std::array<int64_t, 8> &key, int n_cand, int samples, int dev,
                                  hipStream_t stream, uint64_t *ticket) {
    std::lock_guard<std::mutex> lk(mu_);
    *ticket = 0;
    const bool fresh = !layout_sel_.count(key);
    if (fresh && layout_sel_.size() >= kMaxLayouts) return 0;  // bounded: the static rules
    LayoutSel &s = layout_sel_[key];
    if ((int)s.ms.size() != n_cand) s.ms.assign(n_cand, {});
    harvest(s, n_cand);  // also after the choice, so late probes free their events
    auto reserve = [&](int cand) {
        *ticket = ++ticket_serial_;
        s.pending.push_back({cand, nullptr, nullptr, *ticket, dev, stream, stream_last_launch(dev, stream), nullptr});
        return cand;
    };
    auto in_flight = [&](int cand) {
        int n = 0;
        for (const auto &p : s.pending) n += p.cand == cand;
        return n;
    };
    if (s.state == kLayoutContended || s.state == kLayoutRevalidated) return s.chosen;
    if (s.state == kLayoutChosen) {
        if (s.chosen == s.reval_alt || ++s.steady < kLayoutRevalidate) return s.chosen;
        s.state = kLayoutRevalidating;  // once: the kept shape against its alternative, clean timings
    }
    if (s.dropped >= kLayoutMaxDropped) {
        // another stream keeps the device busy while probes run: no timing here is trustworthy
        s.chosen = 0;
        s.state = kLayoutContended;
        s.serial = ++layout_serial_;
        return 0;
    }
    if (s.state == kLayoutRevalidating) {
        const int have[2] = {(int)s.reval_ms[0].size() + in_flight(s.reval_alt),
                             (int)s.reval_ms[1].size() + in_flight(s.chosen)};
        if ((int)s.reval_ms[0].size() >= samples && (int)s.reval_ms[1].size() >= samples) {
            const float alt = median_of(s.reval_ms[0]), kept = median_of(s.reval_ms[1]);
            // a shape other than the static rules (candidate 0) must keep beating them by the margin;
            // a kept static choice is replaced only by a runner-up that beats it by the margin
            const bool keep = s.reval_alt == 0 ? kept < kLayoutMargin * alt : !(alt < kLayoutMargin * kept);
            if (!keep) s.chosen = s.reval_alt;
            s.state = kLayoutRevalidated;
            s.serial = ++layout_serial_;
                return s.chosen;
        }
        if (have[0] >= samples && have[1] >= samples) return s.chosen;  // all in flight: untimed
        return reserve(have[0] <= have[1] ? s.reval_alt : s.chosen);
    }
    // exploring
    std::vector<int> queued(n_cand, 0);
    bool done = true;
    for (int c = 0; c < n_cand; ++c) {
        queued[c] = (int)s.ms[c].size();
        done = done && queued[c] >= samples;
    }
    if (done) {
        const float base = median_of(s.ms[0]);
        int best = 0, second = -1;
        float best_ms = base;
        for (int c = 1; c < n_cand; ++c) {
            const float m = median_of(s.ms[c]);
            if (m < best_ms && m < kLayoutMargin * base) {
                best = c;
                best_ms = m;
            }
        }
        for (int c = 0; c < n_cand; ++c)  // the runner-up: what a kept static choice is re-checked against
            if (c != best && (second < 0 || median_of(s.ms[c]) < median_of(s.ms[second]))) second = c;
        s.chosen = best;
        s.reval_alt = best != 0 ? 0 : (second >= 0 ? second : 0);
        s.state = kLayoutChosen;
        s.steady = 0;
        s.serial = ++layout_serial_;
        return best;
    }
    for (const auto &p : s.pending) ++queued[p.cand];
    int c = 0;
    for (int k = 1; k < n_cand; ++k)
        if (queued[k] < queued[c]) c = k;
    if (queued[c] >= samples) return 0;  // every probe is in flight: the static rules, untimed
    return reserve(c);
}

void CompiledMap::fill_layout_probe(const std::array<int64_t, 8> &key, uint64_t ticket, hipEvent_t e0,
                                    hipEvent_t e1) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto &p : layout_sel_[key].pending)
        if (p.ticket == ticket) {
            p.e0 = e0;
            p.e1 = e1;
            // contaminated already if another stream's latest launch may still run as the probe
            // is enqueued; later launches are judged by note_device_launch while it is open
            p.dirty = open_probe(p.dev, p.stream, e1, other_stream_may_run(p.dev, p.stream, p.since));
            return;
        }
    (void)hipEventDestroy(e0);  // not reserved (cannot happen): drop the events
    (void)hipEventDestroy(e1);
}

void CompiledMap::cancel_layout_probe(const std::array<int64_t, 8> &key, uint64_t ticket) {
    std::lock_guard<std::mutex> lk(mu_);
    auto &v = layout_sel_[key].pending;
    for (auto it = v.begin(); it != v.end(); ++it)
        if (it->ticket == ticket) {
            v.erase(it);
            return;
        }
}

int CompiledMap::layout_choice(int64_t pitch, std::vector<float> *ms, int *state, int *dropped) {
    std::lock_guard<std::mutex> lk(mu_);
    const LayoutSel *latest = nullptr;
    for (const auto &kv : layout_sel_)
        if (kv.first[0] == pitch && kv.second.chosen >= 0 && (!latest || kv.second.serial > latest->serial))
            latest = &kv.second;
    if (!latest) return -1;
    if (ms) {
        ms->clear();
        for (const auto &v : latest->ms) ms->push_back(median_of(v));
    }
    if (state) *state = latest->state;
    if (dropped) *dropped = latest->dropped;
    return latest->chosen;
}

const std::vector<int> &CompiledMap::used_in_slots() {
    compact();
    return used_in_;
}

const std::vector<int> &CompiledMap::used_out_slots() {
    compact();
    return used_out_;
}

// ---------------------------------------------------------------- contexts
DeviceContext::Lease DeviceContext::acquire() {
    static std::mutex reg_mu;
    static std::map<int, std::vector<std::unique_ptr<DeviceContext>>> reg;  // never shrinks: reused
    thread_local DeviceContext *last = nullptr;  // this thread's previous lease: usually still free
    int dev = 0;
    check_hip(hipGetDevice(&dev), "hipGetDevice");
    const bool pool = tuning().host_contexts != 0;
    if (pool && last && last->device == dev) {
        std::unique_lock<std::mutex> l(last->mu, std::try_to_lock);
        if (l.owns_lock()) return Lease{last, std::move(l)};
    }
    DeviceContext *shared = nullptr;
    {
        std::lock_guard<std::mutex> lk(reg_mu);
        auto &v = reg[dev];
        if (pool) {
            for (auto &c : v) {  // a free context of this device (try_lock never blocks under reg_mu)
                std::unique_lock<std::mutex> l(c->mu, std::try_to_lock);
                if (l.owns_lock()) {
                    last = c.get();
                    return Lease{c.get(), std::move(l)};
                }
            }
        } else if (!v.empty()) {
            shared = v.front().get();
        }
        if (!shared) {  // every context busy (or none yet): a new one, leased before it is published
            auto ctx = std::make_unique<DeviceContext>();
            ctx->device = dev;
            check_hip(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking), "hipStreamCreate");
            DeviceContext *c = ctx.get();
            std::unique_lock<std::mutex> l(c->mu);
            v.push_back(std::move(ctx));
            last = c;
            return Lease{c, std::move(l)};
        }
    }
    return Lease{shared, std::unique_lock<std::mutex>(shared->mu)};  // one shared context: wait for it
}

uint8_t *DeviceContext::ensure(size_t bytes) {
    if (bytes <= staging_size_) return staging_;
    if (staging_) check_hip(hipFree(staging_), "hipFree(staging)");
    staging_ = nullptr;
    staging_size_ = 0;
    size_t sz = std::max<size_t>(bytes, 1 << 20);
    check_hip(hipMalloc(&staging_, sz), "hipMalloc(staging)");
    staging_size_ = sz;
    return staging_;
}

uint8_t *DeviceContext::ensure_pinned(size_t bytes) {
    if (bytes <= pinned_size_) return pinned_;
    if (pinned_) check_hip(hipHostFree(pinned_), "hipHostFree(staging)");
    pinned_ = nullptr;
    pinned_size_ = 0;
    size_t sz = std::max<size_t>(bytes, 1 << 20);
    check_hip(hipHostMalloc(reinterpret_cast<void **>(&pinned_), sz, hipHostMallocDefault), "hipHostMalloc(staging)");
    pinned_size_ = sz;
    return pinned_;
}

uint64_t *DeviceContext::counter() {
    if (!counter_) check_hip(hipMalloc(&counter_, sizeof(uint64_t)), "hipMalloc(counter)");
    return counter_;
}

// ---------------------------------------------------------------- host execution
namespace {

struct Staged {
    uint8_t *in;
    uint8_t *out;
    int64_t pitch;
};

Staged stage_inputs(DeviceContext &ctx, CompiledMap &cm, const uint8_t *const *inputs, int64_t offset,
                    int64_t byte_count) {
    const LinearMap &m = cm.map();
    const int64_t pitch = (byte_count + 255) / 256 * 256;
    const int64_t in_slots = cm.max_in_slot() + 1, out_slots = cm.max_out_slot() + 1;
    uint8_t *base = ctx.ensure((size_t)(pitch * (in_slots + out_slots)));
    Staged st{base, base + pitch * in_slots, pitch};
    for (int j = 0; j < m.n_in; ++j) {
        const int slot = m.in_slot[j];
        if (!inputs[slot]) throw Error(ECX_E_NULL, "input buffer is null");
        check_hip(hipMemcpyAsync(st.in + pitch * slot, inputs[slot] + offset, (size_t)byte_count,
                                 hipMemcpyHostToDevice, ctx.stream),
                  "hipMemcpyAsync H2D");
    }
    return st;
}

}  // namespace

namespace {
// Gather path: used input slots -> pinned [U][pitch] -> HBM; compact map; rows -> pinned [V][pitch].
// Returns the pinned output rows (valid after the stream synchronises).
const uint8_t *run_gathered(DeviceContext &ctx, CompiledMap &cm, const uint8_t *const *inputs, int64_t offset,
                            int64_t byte_count, uint8_t **dev_out, int64_t *pitch_out) {
    CompiledMap &cc = cm.compact();
    const std::vector<int> &ins = cm.used_in_slots(), &outs = cm.used_out_slots();
    const int64_t pitch = (byte_count + 255) / 256 * 256;
    const int64_t nin = (int64_t)ins.size(), nout = (int64_t)outs.size();
    uint8_t *host = ctx.ensure_pinned((size_t)(pitch * (nin + nout)));
    uint8_t *dev = ctx.ensure((size_t)(pitch * (nin + nout)));
    for (int64_t u = 0; u < nin; ++u) {
        const uint8_t *src = inputs[ins[u]];
        if (!src) throw Error(ECX_E_NULL, "input buffer is null");
        std::memcpy(host + u * pitch, src + offset, (size_t)byte_count);
    }
    check_hip(hipMemcpyAsync(dev, host, (size_t)(pitch * nin), hipMemcpyHostToDevice, ctx.stream), "hipMemcpyAsync H2D");
    launch_apply(cc, dev, 0, pitch, dev + pitch * nin, 0, pitch, 1, byte_count, ctx.stream);
    *dev_out = dev + pitch * nin;
    *pitch_out = pitch;
    return host + pitch * nin;
}
}  // namespace

namespace {
// Every buffer the map reads or writes must exist before anything is enqueued: a null
// found halfway would leave copies to or from the caller's (e.g. JNI-pinned) arrays in flight.
void check_host_buffers(const LinearMap &m, const uint8_t *const *inputs, uint8_t *const *outputs) {
    for (int j = 0; j < m.n_in; ++j)
        if (!inputs[m.in_slot[j]]) throw Error(ECX_E_NULL, "input buffer is null");
    if (outputs)
        for (int o = 0; o < m.n_out; ++o)
            if (!outputs[m.out_slot[o]]) throw Error(ECX_E_NULL, "output buffer is null");
}

// Drains the leased stream when an error unwinds a host call, before the lease (and the
// caller's buffers) are released: no DMA to or from caller memory outlives the call.
struct DrainOnUnwind {
    hipStream_t stream;
    int depth = std::uncaught_exceptions();
    ~DrainOnUnwind() {
        if (std::uncaught_exceptions() > depth) (void)hipStreamSynchronize(stream);
    }
};
}  // namespace

bool host_exec_wanted(int64_t byte_count) {
    const int64_t max = g_host_exec_max.load(std::memory_order_relaxed);
    if (max <= 0 || byte_count <= 0 || byte_count > max) return false;
    static const int count = [] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) {
            (void)hipGetLastError();
            n = 0;
        }
        return n;
    }();
    if (count <= 0) throw Error(ECX_E_DEVICE, "hipGetDeviceCount: no HIP device");
    return true;
}

void run_host(CompiledMap &cm, const uint8_t *const *inputs, uint8_t *const *outputs, int64_t offset,
              int64_t byte_count) {
    if (byte_count <= 0 || cm.map().n_out == 0) return;
    check_host_buffers(cm.map(), inputs, outputs);
    if (host_exec_wanted(byte_count)) {  // below the per-call crossover (host_exec.cpp)
        host_exec_apply(cm.map(), inputs, outputs, offset, byte_count);
        return;
    }
    DeviceContext::Lease lease = DeviceContext::acquire();
    DeviceContext &ctx = *lease.ctx;
    DrainOnUnwind drain{ctx.stream};
    const int64_t zc_pitch = (byte_count + 255) / 256 * 256;
    void *zc_dev = nullptr;
    const Tuning tu = tuning();  // one snapshot for the whole call
    bool zero_copy = byte_count <= tu.host_gather_max && tu.host_zero_copy;
    if (zero_copy) {
        const size_t bytes = (size_t)(zc_pitch * (int64_t)(cm.used_in_slots().size() + cm.used_out_slots().size()));
        if (hipHostGetDevicePointer(&zc_dev, ctx.ensure_pinned(bytes), 0) != hipSuccess) {
            (void)hipGetLastError();  // clear the sticky error; use the copy path
            zero_copy = false;
        }
    }
    if (zero_copy) {
        // Zero-copy variant: the kernel reads the gathered inputs from, and writes the
        // output rows to, the pinned staging area itself over PCIe (no DMA copies).  If
        // the staging area is not mapped into the device's address space, the copy path
        // below runs instead.
        CompiledMap &cc = cm.compact();
        const std::vector<int> &ins = cm.used_in_slots(), &outs = cm.used_out_slots();
        for (int slot : outs)
            if (!outputs[slot]) throw Error(ECX_E_NULL, "output buffer is null");
        const int64_t pitch = zc_pitch;
        const int64_t nin = (int64_t)ins.size(), nout = (int64_t)outs.size();
        uint8_t *host = ctx.ensure_pinned((size_t)(pitch * (nin + nout)));  // the same area (already large enough)
        for (int64_t u = 0; u < nin; ++u) {
            const uint8_t *src = inputs[ins[u]];
            if (!src) throw Error(ECX_E_NULL, "input buffer is null");
            std::memcpy(host + u * pitch, src + offset, (size_t)byte_count);
        }
        uint8_t *dev = static_cast<uint8_t *>(zc_dev);
        launch_apply(cc, dev, 0, pitch, dev + pitch * nin, 0, pitch, 1, byte_count, ctx.stream);
        check_hip(hipStreamSynchronize(ctx.stream), "hipStreamSynchronize");
        for (int64_t v = 0; v < nout; ++v)
            std::memcpy(outputs[outs[v]] + offset, host + (nin + v) * pitch, (size_t)byte_count);
        return;
    }
    if (byte_count <= tu.host_gather_max) {
        const std::vector<int> &outs = cm.used_out_slots();
        for (int slot : outs)
            if (!outputs[slot]) throw Error(ECX_E_NULL, "output buffer is null");
        uint8_t *dev_rows = nullptr;
        int64_t pitch = 0;
        const uint8_t *host_rows = run_gathered(ctx, cm, inputs, offset, byte_count, &dev_rows, &pitch);
        check_hip(hipMemcpyAsync(const_cast<uint8_t *>(host_rows), dev_rows, (size_t)(pitch * (int64_t)outs.size()),
                                 hipMemcpyDeviceToHost, ctx.stream),
                  "hipMemcpyAsync D2H");
        check_hip(hipStreamSynchronize(ctx.stream), "hipStreamSynchronize");
        for (size_t v = 0; v < outs.size(); ++v)
            std::memcpy(outputs[outs[v]] + offset, host_rows + (int64_t)v * pitch, (size_t)byte_count);
        return;
    }
    Staged st = stage_inputs(ctx, cm, inputs, offset, byte_count);
    launch_apply(cm, st.in, 0, st.pitch, st.out, 0, st.pitch, 1, byte_count, ctx.stream);
    const LinearMap &m = cm.map();
    for (int o = 0; o < m.n_out; ++o) {
        const int slot = m.out_slot[o];
        if (!outputs[slot]) throw Error(ECX_E_NULL, "output buffer is null");
        check_hip(hipMemcpyAsync(outputs[slot] + offset, st.out + st.pitch * slot, (size_t)byte_count,
                                 hipMemcpyDeviceToHost, ctx.stream),
                  "hipMemcpyAsync D2H");
    }
    check_hip(hipStreamSynchronize(ctx.stream), "hipStreamSynchronize");
}

bool run_host_all_zero(CompiledMap &cm, const uint8_t *const *inputs, int64_t offset, int64_t byte_count) {
    if (byte_count <= 0 || cm.map().n_out == 0) return true;
    check_host_buffers(cm.map(), inputs, nullptr);
    if (host_exec_wanted(byte_count)) return host_exec_all_zero(cm.map(), inputs, offset, byte_count);
    DeviceContext::Lease lease = DeviceContext::acquire();
    DeviceContext &ctx = *lease.ctx;
    DrainOnUnwind drain{ctx.stream};
    uint64_t *cnt = ctx.counter();
    check_hip(hipMemsetAsync(cnt, 0, sizeof(uint64_t), ctx.stream), "hipMemsetAsync");
    if (byte_count <= tuning().host_gather_max) {
        uint8_t *dev_rows = nullptr;
        int64_t pitch = 0;
        (void)run_gathered(ctx, cm, inputs, offset, byte_count, &dev_rows, &pitch);
        launch_count_mismatch(dev_rows, pitch, nullptr, 0, (int64_t)cm.used_out_slots().size(), byte_count, cnt,
                              ctx.stream);
    } else {
        Staged st = stage_inputs(ctx, cm, inputs, offset, byte_count);
        launch_apply(cm, st.in, 0, st.pitch, st.out, 0, st.pitch, 1, byte_count, ctx.stream);
        const LinearMap &m = cm.map();
        for (int o = 0; o < m.n_out; ++o)
            launch_count_mismatch(st.out + st.pitch * m.out_slot[o], 0, nullptr, 0, 1, byte_count, cnt, ctx.stream);
    }
    uint64_t host = 0;
    check_hip(hipMemcpyAsync(&host, cnt, sizeof(uint64_t), hipMemcpyDeviceToHost, ctx.stream), "hipMemcpyAsync D2H");
    check_hip(hipStreamSynchronize(ctx.stream), "hipStreamSynchronize");
    return host == 0;
}

}  // namespace ecx
