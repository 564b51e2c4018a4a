// engine.hpp -- compiled GF(256) maps, device contexts and kernel launches.
//
// Kernel plan format (one "entry" per (output tile, input slot) pair with a
// non-zero coefficient; tiles of up to kTileRows output rows):
//
//   entry (kEntryDwords u32):
//     [0] input slot   [1] rows with a general coefficient (bitmask)
//     [2] rows whose coefficient is 1 (bitmask: plain XOR)   [3] 0
//     [4+5r .. 8+5r]  split multiply tables for tile row r:
//        T0a,T0b = c*v for v in 0..7        (low 3 bits of the byte)
//        T1a,T1b = c*(v<<3) for v in 0..7   (middle 3 bits)
//        T2      = c*(v<<6) for v in 0..3   (top 2 bits)
//     so that c*b = T0[b&7] ^ T1[(b>>3)&7] ^ T2[b>>6]; each lookup is one
//     v_perm_b32 over four bytes at once (GF(2)-linearity of c*b).
//   tile (kTileDwords u32): [0] first entry [1] entry count [2] rows
//     [4..4+kTileRows) output slot of each row.
#pragma once

#include <hip/hip_runtime.h>

#ifndef ECX_DIAG
#define ECX_DIAG 0  // 1: the diagnostic build (Makefile DIAG=1) with the measured-and-rejected kernels
#endif

#include <array>
#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "codes.hpp"
#include "host_exec.hpp"

namespace ecx {

constexpr int kTileRows = 8;
constexpr int kEntryDwords = 48;
constexpr int kTileDwords = 16;
constexpr int kChunkBytes = 4096;  // one 256-thread workgroup x 16 bytes per lane
constexpr int kBlockThreads = 256;
constexpr size_t kLdsPerCu = 160 * 1024;  // MI355X (gfx950) LDS per CU
constexpr int kSimdsPerCu = 4;
constexpr int kOccWavesPerSimd = 4;       // the residency cap of the many-stream single-tile maps
constexpr int kWaveGroup = 8;       // k_gf_apply_lds: up to 8 tiles (one wave each) per workgroup
constexpr int kGroupDwords = 16;    // group: [0..7] tiles (kNoTile = none), [8] union begin, [9] union count
constexpr int kWaveChunkBytes = 1024;  // k_gf_apply_lds: 64 lanes x 16 bytes per wave
constexpr uint32_t kNoTile = 0xFFFFFFFFu;

void check_hip(hipError_t e, const char *what);

class MapPlanes;  // map_rtc.hpp

constexpr uint32_t kDummySlot = 0xFFFFFFFFu;  // entry padding: loads the device's zero page

struct DevicePlan {
    uint32_t *entries = nullptr;
    uint32_t *tiles = nullptr;
    uint32_t *groups = nullptr;  // n_groups x kGroupDwords
    uint32_t *unions = nullptr;  // per group: input slots in staging order, padded (kDummySlot)
    // Per padded entry, kTileRows x {T0a, T1a}: the low table dwords of every row,
    // staged per workgroup into LDS by k_gf_apply<..., TLDS=true> (kernels.hip).
    uint32_t *atab = nullptr;
    uint32_t *wentries = nullptr;  // wide tiles (k_gf_apply_wide)
    uint32_t *wtiles = nullptr;
    uint32_t *bentries = nullptr;  // bit-sliced kernel (k_gf_bits): kBitsEntryDwords per padded entry
    int max_tile_entries = 0;  // padded
};
constexpr int kAtabDwords = 2 * kTileRows;
// Wide tiles (k_gf_apply_wide): two 8-row tiles A, B applied by one workgroup over the
// union of their inputs.  A wide entry is A's entry for the input followed by B's
// (kEntryDwords each; zero masks where a half does not read the input).  A wide tile
// record: [0] first wide entry [1] entry count [2] rows of A [3] rows of B
// [4..12) output slots of A's rows [12..20) output slots of B's rows.
constexpr int kWideEntryDwords = 2 * kEntryDwords;
constexpr int kWideTileDwords = 32;
constexpr int kMaxLdsTileEntries = 512;  // 32 KiB of LDS per workgroup at most
// Bit-sliced kernel (k_gf_bits, apply_bits.hip): per padded entry [0] input slot
// [1] rows with a non-zero coefficient (bitmask) [2] coefficients of rows 0-3 (one
// byte each) [3] coefficients of rows 4-7.  Parallel to the padded `entries` array,
// so the padded `tiles` index both.
constexpr int kBitsEntryDwords = 4;
constexpr int kBitsThreads = 128;  // 128 lanes x 32 bytes = one 4 KiB chunk (kChunkBytes)

// The padded plan exactly as uploaded to a device for one load-ring depth
// (CompiledMap::padded_plan): entries/tiles padded to multiples of `depth`,
// group unions padded to whole LDS stages, and the TLDS low-table array.
struct HostPlan {
    std::vector<uint32_t> entries, tiles, groups, unions, atab, wentries, wtiles, bentries;
    int max_tile_entries = 0;
};

// 4 KiB of zeros per device, never written: the load target of padding entries
// (always L2-resident, so padding costs no HBM traffic).
const uint8_t *zero_page_for_current_device();

// A LinearMap compiled to the kernel's table format, uploaded lazily per device.
class CompiledMap {
public:
    explicit CompiledMap(LinearMap m);
    ~CompiledMap();
    const LinearMap &map() const { return map_; }
    int n_tiles() const { return n_tiles_; }
    // Multi-tile maps: tiles grouped by shared inputs, one workgroup per group
    // (engine.cpp group_tiles / align_group).
    int n_groups() const { return n_groups_; }
    int group_size() const { return group_size_; }
    int n_entries() const { return (int)(entries_.size() / kEntryDwords); }  // unpadded (1 if empty)
    // Wide tiles: the 8-row tiles paired by shared inputs (multi-tile maps only).
    int n_wide_tiles() const { return n_wide_; }
    int wide_entries() const { return (int)(wentries_.size() / kWideEntryDwords); }  // unpadded
    int wide_depth() const { return wide_depth_; }
    // Input reads saved by pairing: (sum of the paired tiles' input counts) / (sum of
    // the pairs' union sizes); 1.0 = the pairs share nothing.
    double wide_sharing() const { return wide_union_ ? (double)wide_reads_ / (double)wide_union_ : 1.0; }
    int union_total() const { return (int)unions_.size(); }                   // unpadded
    int max_in_slot() const { return max_in_slot_; }
    int max_out_slot() const { return max_out_slot_; }
    // Load-ring depth for this map: 8 when every non-empty tile has >= 12 entries
    // (padding to a multiple of 8 then costs little), else 4 (profiles/r01_configs_depth.jsonl, r01_configs_sweep2.jsonl).
    int preferred_depth() const { return preferred_depth_; }
    int max_tile_rows() const { return max_tile_rows_; }
    // The plan uploaded for the current device, each tile's entry list padded to a
    // multiple of `depth` with zero-coefficient kDummySlot entries.
    const DevicePlan &plan_for_current_device(int depth);
    // The same map over densely renumbered slots: input column j reads compact slot
    // rank(in_slot[j]) among used_in_slots() (sorted), likewise for outputs.  This is
    // the device-side layout of the host-batch pipeline (host_pipe.cpp).
    // Host interpretation of the compiled plan (diagnostics, ecx_map_selftest):
    // applies the entry tables exactly as the kernels read them -- by input slot
    // (k_gf_apply) or through the group unions (k_gf_apply_lds) -- to `in`
    // ([max_in_slot+1][len]) and writes `out` ([max_out_slot+1][len]).  Throws
    // if the union bookkeeping is inconsistent.
    void emulate(const uint8_t *in, uint8_t *out, int64_t len, bool via_unions) const;
    // The host arrays plan_for_current_device(depth) uploads.
    HostPlan padded_plan(int depth) const;
    // Host interpretation of a padded plan as k_gf_apply reads it: padding entries
    // read zeros, and with `tlds` the low dword of each 8-entry table comes from
    // HostPlan::atab (the LDS copy) instead of the entry.
    void emulate_padded(const HostPlan &p, const uint8_t *in, uint8_t *out, int64_t len, bool tlds, int depth) const;
    // The same for the padded wide-tile arrays (k_gf_apply_wide).
    void emulate_wide(const HostPlan &p, const uint8_t *in, uint8_t *out, int64_t len) const;
    // k_gf_bits on the host: the bit-sliced arithmetic of apply_bits.hip (the same
    // __host__ __device__ transpose / xtime / nibble code) over the padded
    // `bentries`, for `len` a multiple of kChunkBytes (the kernel's chunk).
    void emulate_bits(const HostPlan &p, const uint8_t *in, uint8_t *out, int64_t len) const;
    CompiledMap &compact();
    // The generated bit-plane kernel for this map (map_rtc.hpp), created on first use;
    // nullptr when the map does not fit it (more than 16 rows, too many coefficients).
    MapPlanes *planes();
    const std::vector<int> &used_in_slots();
    const std::vector<int> &used_out_slots();
    // Per-layout launch-shape selection (kernels.hip launch_apply, ecx_tune "layout_select"):
    // the candidate to run for this call of the batch layout `key` on `stream` of device `dev`.
    // Finished timing probes are harvested first (non-blocking).  A probe is DROPPED, not
    // counted, when another stream of the same device had a large libecx launch that may still
    // run when the probe was enqueued, or enqueued one while the probe was still running (the
    // first such launch that finds the probe's end event done closes its window;
    // note_device_launch): that kernel may have shared the GPU with the probe.  Once every
    // one of the n_cand candidates has `samples` clean
    // timings the fastest median is kept (candidate 0 -- the static rules -- unless another is
    // faster by kLayoutMargin); after kLayoutMaxDropped dropped probes the layout is CONTENDED
    // and keeps candidate 0 untimed.  Any kept shape is re-validated once, after
    // kLayoutRevalidate further launches, against its alternative -- the static rules for a
    // non-static choice, the runner-up for a static one: `samples` clean timings of each, and
    // the alternative takes over if it wins by the margin (a non-static choice must keep
    // beating the static rules by it).  At most kMaxLayouts layouts are selected per map (later ones get candidate 0,
    // untimed).  When the call is to be timed, *ticket is set to a non-zero probe slot
    // reserved in the layout's pending list (so concurrent callers are never handed the same
    // probe twice): the caller brackets its launch with two events on `stream` and hands them
    // to fill_layout_probe, or gives the slot back with cancel_layout_probe.
    int next_layout_pick(const std::array<int64_t, 8> &key, int n_cand, int samples, int dev, hipStream_t stream,
                         uint64_t *ticket);
    void fill_layout_probe(const std::array<int64_t, 8> &key, uint64_t ticket, hipEvent_t e0, hipEvent_t e1);
    void cancel_layout_probe(const std::array<int64_t, 8> &key, uint64_t ticket);
    // The candidate kept for the most recently selected layout with input slot pitch
    // `pitch`, -1 if none yet; with `ms`, the per-candidate median launch times (ms, -1 =
    // unsampled) of that layout; with `state` its state (LayoutState) and with `dropped` the
    // probes it dropped as contaminated.
    int layout_choice(int64_t pitch, std::vector<float> *ms = nullptr, int *state = nullptr, int *dropped = nullptr);
    enum LayoutState { kLayoutExploring = 0, kLayoutChosen = 1, kLayoutRevalidating = 2, kLayoutRevalidated = 3,
                       kLayoutContended = 4 };

private:
    struct LayoutSel {
        struct Probe {
            int cand;
            hipEvent_t e0, e1;   // null until fill_layout_probe
            uint64_t ticket;
            int dev;
            hipStream_t stream;
            uint64_t since;      // the stream's last launch serial before this probe (note_device_launch)
            std::shared_ptr<std::atomic<bool>> dirty;  // set when another stream's launch may overlap it
        };
        std::vector<std::vector<float>> ms;  // per candidate: clean launch times of its probes
        std::vector<Probe> pending;          // reserved or unfinished probes
        int chosen = -1;
        int state = kLayoutExploring;
        int dropped = 0;                     // probes discarded as contaminated
        int64_t steady = 0;                  // launches since the choice (re-validation trigger)
        int reval_alt = 0;                   // the shape the kept one is re-validated against
        std::vector<float> reval_ms[2];      // re-validation timings: [0] the alternative, [1] the kept shape
        uint64_t serial = 0;                 // order of the choices (layout_choice reports the latest)
    };
    void harvest(LayoutSel &s, int n_cand);
    std::map<std::array<int64_t, 8>, LayoutSel> layout_sel_;
    uint64_t layout_serial_ = 0;
    uint64_t ticket_serial_ = 0;
    LinearMap map_;
    std::unique_ptr<CompiledMap> compact_;
    std::unique_ptr<MapPlanes> planes_;
    bool planes_checked_ = false;
    std::vector<int> used_in_, used_out_;
    std::vector<uint32_t> entries_, tiles_;  // unpadded
    std::vector<uint32_t> groups_, unions_;  // unpadded unions
    std::vector<uint32_t> wentries_, wtiles_;  // unpadded wide tiles
    int n_groups_ = 0, group_size_ = 0, n_wide_ = 0, wide_depth_ = 4;
    int64_t wide_reads_ = 0, wide_union_ = 0;
    int n_tiles_ = 0, max_in_slot_ = -1, max_out_slot_ = -1, preferred_depth_ = 4, max_tile_rows_ = 0;
    std::mutex mu_;
    std::map<std::pair<int, int>, DevicePlan> dev_;  // (device, depth)
};

struct ApplyArgs {
    const uint8_t *in;
    uint8_t *out;
    const uint32_t *entries;
    const uint32_t *tiles;
    const uint32_t *groups;
    const uint32_t *unions;
    const uint32_t *atab;
    const uint32_t *wentries;
    const uint32_t *wtiles;
    const uint32_t *bentries;
    const uint8_t *zero_page;
    int64_t in_stripe_stride, in_slot_stride, out_stripe_stride, out_slot_stride;
    int64_t nbytes, chunk_begin, n_chunks, stripe_begin;
    int n_tiles;
    int n_wide;           // k_gf_apply_wide: wide tiles (workgroups per chunk)
    int n_groups;         // k_gf_apply_lds: tile groups (workgroups per chunk)
    int xcd_group;        // k_gf_apply: keep the tiles of one chunk on one XCD
    int xcd_run;          // k_gf_apply, xcd_group 3: units (stripe, chunk) per XCD run
    int accumulate;       // 1: out ^= M * in (partial sums along a repair chain), 0: out = M * in
    int lane_zero;        // always 0 (keeps k_gf_apply's LDS table base in a VGPR)
    int chunk_major;      // k_gf_apply block order: 0 = stripe by stripe, 1 = chunk c of every stripe, then c + 1
    int stagger;          // k_gf_apply / _skew unit order: > 1 = groups of that many stripes interleaved (unit_of)
    // k_gf_apply (not byte-safe): the chunk index holding a shard's partial last chunk when it
    // runs in the same launch as the full chunks (-1: none), and its byte count (a multiple of 16)
    int64_t tail_chunk;
    int tail_bytes;
    int64_t multi_total;  // k_gf_apply_multi: (stripe, chunk) units in the launch
};

// Launch-shape knobs (diagnostics / tuning, include/ecx_tune.h).
struct Tuning {
    // Defaults are the fastest shape measured on MI355X (profiles/r01_kbench.txt).
    int depth = 0;            // k_gf_apply load ring depth: 0 = per map (preferred_depth), or forced
    int nontemporal = 1;      // 0 never, 1 auto (NT stores; NT loads for single-tile maps), 2 always
    int xcd_group = 0;        // multi-tile maps: tiles of a chunk on one XCD (measured slower: off)
    int xcd_run = 8;          // xcd_group 3 (any map): runs of this many consecutive units per XCD
    int xcd_misaligned = 1;   // xcd_group 0: single-tile maps with inputs not 128-B aligned use the runs of 3
    // Multi-tile maps: 1 = k_gf_apply_lds (tile groups share inputs via LDS), 2 =
    // k_gf_apply_grp (tile groups in one workgroup, direct loads).  Off by
    // default: Clay(10,4)'s 64-row groups still need 1.23x the unique inputs and the
    // per-stage barriers cost more than the saved traffic (profiles/r01_multitile.jsonl).
    int wave_groups = 0;
    // k_gf_apply: 0 = every table dword from the plan in SGPRs (a v_mov per 8-entry table
    // and row); 1 = the low table dwords staged once per workgroup in LDS and read as
    // VGPRs, for multi-tile maps; 2 = for every map.
    int lds_tables = 1;
    // Non-temporal output stores: 0 = `nt`; 1 = `nt sc0 sc1` (written through, dropped
    // from L2; scripts/copy_probe.hip).
    int store_scope = 0;
    // k_gf_apply: extra dynamic LDS bytes per workgroup, which caps the workgroups resident
    // per CU (160 KiB of LDS each) without touching the kernel.  0 = no cap (default); -1 =
    // single-tile maps over >= 8 inputs on rings of <= 8 loads held to 4 waves per SIMD; > 0 =
    // that many bytes.  Measured mixed on the RS maps (+2 % in fresh-process A/B runs, -2 to
    // -5 % in one-process interleaved sweeps; profiles/r03_occupancy.jsonl, r03_occ_bench.jsonl).
    int occ_lds = 0;
    // k_gf_apply block order: 0 = stripe-major (a stripe's chunks back to back), 1 = chunk-major.
    int chunk_major = 0;
    // k_gf_apply / k_gf_apply_skew unit order: 0 / 1 = none; G >= 2 = G stripes interleaved,
    // each starting at a different chunk offset (apply.hpp unit_of).
    int stagger = 0;
    // k_gf_apply workgroup: 256 threads over 4 KiB chunks (default) or 64 threads (one
    // wave) over 1 KiB chunks.
    int block_threads = 0;  // 0 = auto (launch_apply), 256 or 64 forced
    // Single-tile maps of at most 2 / 4 rows: 1 = k_gf_apply variants with that many
    // accumulator rows (fewer VGPRs, depth-12 rings possible); 0 = the 8-row kernel.
    int small_tiles = 2;  // 2 = auto (launch_apply), 1 = forced, 0 = the 8-row kernel
    // Per-call host APIs on the gather path: 1 = the kernel reads / writes the pinned
    // staging area directly over PCIe instead of one H2D and one D2H copy (20-40 % lower
    // latency per call, profiles/r01_percall_native.jsonl).
    int host_zero_copy = 1;
    // Multi-tile maps: 1 = wide tiles (pairs of 8-row tiles sharing inputs, one
    // workgroup each: 16 accumulator rows, each shared input loaded once per pair).
    int wide_tiles = 1;
    // Single-tile maps: 2 / 4 = k_gf_apply_skew with that many 4 KiB chunks per
    // workgroup, each entry's chunk rotated; 1 = 4 when the input slot pitch is a
    // multiple of 4 MiB; 0 = off.
    int skew_chunks = 1;
    // Many-stream single-tile maps (>= 8 inputs, <= 4 rows) with the shape knobs on auto: 1 =
    // the launch shape chosen per batch layout by timing the caller's own first launches
    // (kernels.hip launch_apply; default), 0 = the static rules only.
    int layout_select = 1;
    // Per-call CodingLoop entry points: compiled plans kept, by map content (0 = none).
    int plan_cache = 256;
    // Bit-sliced kernel (k_gf_bits): 2 = for every map it can run (aligned layout, 32-bit
    // slot offsets, 4 KiB chunks), 1 = for multi-tile maps that do not pair into wide
    // tiles, 0 = never (default: it measured 4-10 % slower on every BASELINE map, bound
    // by its scalar branches -- profiles/r02_bits_ab.jsonl, r02_bits_sq_ab.json).
    int bitslice = 0;
    // LDS lookup-table kernel (k_gf_lut, apply_lut.hip) for the full 4 KiB chunks of
    // aligned layouts, forced-only: 1 = log/antilog tables, 2 = one 256-B product row per
    // coefficient (single-tile maps of <= kLutMaxPairs general coefficients); 0 = never
    // (default: measured against the split tables in DESIGN.md 4.4).
    int lds_lut = 0;
    // Clay single-node repair batches: the per-helper-plane kernel generated for the
    // repair and compiled with hiprtc (clay_rtc.hpp) for whole 4 KiB chunks -- 1 = when
    // the composed map spans several tiles (auto), 2 = always, 0 = never.
    int clay_rtc = 1;
    int rtc_lookahead = 1;  // the generated kernel's load lookahead (items), 0..3
    int rtc_waves = 3;      // its __launch_bounds__ minimum waves per SIMD, 2..4
    int rtc_group = 1;      // 1: the plane-group kernel (k_clay_repair_grp) where the program allows it
                            // (+4-8 % over one plane per workgroup on Clay(10,4), profiles/r02_grp_sweep.jsonl)
    int rtc_persist = 0;    // its persistent grid: workgroups per CU (0 = one workgroup per unit)
    int rtc_diag = 0;       // its DIAGNOSTIC builds (clay_rtc.hpp RtcShape::diag; ECX_DIAGNOSTIC=1 only)
    int rtc_units = 1;      // plane-group kernel: 512-B slices per workgroup, 1 or 2 (software-pipelined)
    int rtc_sched = 2;      // plane-group kernel load schedule: 0 = rtc_lookahead's, 1 = lean, 2 = all loads
                            // up front with pinned accumulators (+0.8-2.4 % over 0 on two boxes,
                            // profiles/r03_clay104_final.jsonl, r03_clay104_lean_run2.jsonl)
    int rtc_wide = 0;       // plane-group kernel: 1 = 64-bit load addresses on every layout (auto, 0: only
                            // where slot offsets exceed 31 bits, RtcShape::wide)
    int rtc_nt = 5;         // non-temporal loads in the generated Clay kernels (RtcShape::nt bits):
                            // 5 = the plane-group kernel's read-once rows and row-yc partner loads,
                            // +3-6 % on Clay(10,4) over cached loads (profiles/r03_clay104_nt.jsonl)
    int rtc_xcd = 2;        // its block order: 1 = the helper planes of a (stripe, chunk) on one XCD;
                            // 2 (plane-group kernel): whole (stripe, chunk) units per XCD, +4.5 %
                            // (+1.1 % on Clay(10,4), profiles/r02_rtc_sweep.jsonl)
    // Generated bit-plane kernel for one composed map (k_map_planes, map_rtc.hpp): 1 = auto
    // for multi-tile maps of <= 16 rows whose coefficients outnumber their inputs by 4x or
    // more (vector-bound under the split tables: the Clay(4,2) two-node repairs), on
    // batches of >= 64 MiB of input; 2 = wherever it fits; 0 = never.
    int map_planes = 1;
    int planes_lookahead = 12;  // its load lookahead (inputs in flight), 0..15 (profiles/r02_planes_ab.jsonl)
    int planes_waves = 2;      // its __launch_bounds__ minimum waves per SIMD, 1..4
    int64_t host_chunk = 64 << 20;  // host-batch pipeline: input bytes per H2D chunk
    int host_buffers = 3;           // host-batch pipeline: device buffer sets in flight
    // per-call host APIs: byte counts up to this gather the used slots into pinned staging (one
    // H2D / one D2H); above it the runtime copies each slot (512 KiB: the crossover of the two,
    // profiles/r02_percall_sizes.jsonl)
    int64_t host_gather_max = 512 << 10;
    int host_contexts = 1;  // per-call host APIs: 1 = a pool of contexts (streams) leased per call, 0 = one per device
    // per-call host APIs: byte counts up to this run on the calling thread (host_exec.cpp) instead of
    // the device -- the measured per-call crossover (profiles/r06_percall_threshold.jsonl): with one
    // caller thread the device first wins at 2 MiB (Clay(4,2) performCoding; the RS(2,2) pair never,
    // to 4 MiB), with 16 at no size to 4 MiB; 0 = never
    int64_t host_exec_max = 1 << 20;
    // single-tile maps: (stripe, chunk) units per workgroup with one load ring across them
    // (k_gf_apply_multi, apply_multi.hip): 1 = one unit per workgroup (k_gf_apply), 2 or 4
    int units = 1;
};
void launch_probe(int kind, const uint8_t *src, uint8_t *dst, int64_t nbytes, bool nt, hipStream_t stream);
// The process-wide tuning (include/ecx_tune.h).  tuning() returns a snapshot taken under
// the lock update_tuning() holds while ecx_tune changes a field, so a launch reads one
// consistent set of knobs even while another thread tunes.
Tuning tuning();
void update_tuning(const std::function<void(Tuning &)> &f);

// The kernel instance of the last full-chunk (non-byte-safe) launch enqueued on this
// thread, as rocprofv3 names it ("k_gf_apply<false, true, 1, 20, false, 256, 8>").
// Diagnostics: bench.py's roofline.kernel and its PMC-profile match (ecx_last_kernel).
void set_last_kernel(std::string name);
const std::string &last_kernel();
// The full launch shape of that launch: the kernel instance plus the unit order the kernel name
// does not encode ("stagger=G xcd_group=X xcd_run=R"), set by the launcher after the kernel is
// noted (ecx_last_launch_shape; bench.py's roofline.launch_shape and its PMC-profile key).
uint64_t kernel_notes();  // set_last_kernel calls on this thread so far
void set_last_shape_order(std::string order);
std::string last_launch_shape();
inline std::string kernel_param(bool v) { return v ? "true" : "false"; }
inline std::string kernel_param(int v) { return std::to_string(v); }
template <typename... P>
void note_kernel(const char *name, P... params) {
    std::string s = name;
    s += '<';
    const char *sep = "";
    ((s += sep, s += kernel_param(params), sep = ", "), ...);
    s += '>';
    set_last_kernel(std::move(s));
}

// Per-device launch registry (engine.cpp), read by the layout selection's contamination check:
// every batch launch of the library (launch_apply, launch_check, the generated Clay kernels)
// records its stream and input bytes here.  note_device_launch returns the launch's serial and,
// for a launch of >= 64 MiB, records an event behind it (smaller launches run for microseconds
// and never count as overlapping a probe); stream_last_launch is the serial of a stream's latest
// launch (0 = none); other_stream_may_run whether a stream other than `s` on device `dev` has a
// large launch that may still run (its event is not done; or no event could be recorded and it
// came after `since`).  Streams unseen for 4,096 launches age out of the registry.
uint64_t note_device_launch(int dev, hipStream_t s, int64_t bytes);
uint64_t stream_last_launch(int dev, hipStream_t s);
bool other_stream_may_run(int dev, hipStream_t s, uint64_t since);
// A layout probe whose end event `e1` is recorded on `s`: registered (unless already `dirty`)
// so that note_device_launch on another stream of `dev` flags it while it runs; close_probe
// unregisters it before its events are destroyed.
std::shared_ptr<std::atomic<bool>> open_probe(int dev, hipStream_t s, hipEvent_t e1, bool dirty);
void close_probe(int dev, hipEvent_t e1);

// Enqueue out = M * in over nstripes stripes (kernels.hip).
// The launch_apply_core pick of per-layout candidate `cand` (kernels.hip kLayoutCand):
// -1 = the static rules, else shape (0 = 256-thread / 4 KiB, 1 = skewed chunks, 2 = one-wave
// / 1 KiB) + 8 * stagger; -2 for an index out of range.
int layout_candidate_code(int cand);
void launch_apply(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride, uint8_t *out,
                  int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes, int64_t nbytes,
                  hipStream_t stream, bool accumulate = false);
// isParityCorrect over device-resident stripes (apply_check.hip k_gf_check): `cm` is a check
// map (one syndrome row per parity shard); verdict[s] = 1 when every syndrome byte of stripe s
// over [0, nbytes) is zero, else 0.  Read-only on the stripes.
void launch_check(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                  uint8_t *verdict, int64_t nstripes, int64_t nbytes, hipStream_t stream);
void launch_fill_random(uint8_t *dst, int64_t nbytes, uint64_t seed, hipStream_t stream);
void launch_count_mismatch(const uint8_t *a, int64_t a_stride, const uint8_t *b, int64_t b_stride, int64_t nrows,
                           int64_t row_bytes, uint64_t *d_count, hipStream_t stream);

// Per-device contexts for the host (byte[][]) entry points: a stream and growable
// device / pinned staging areas each.  A call leases a free context of the current
// device for its duration (acquire), so calls from different threads run on different
// streams and overlap; a new context is created only when every existing one is busy,
// so their number follows the peak concurrency, not the thread count (a JVM thread pool
// that replaces its threads creates none).  Tuning::host_contexts 0 = one shared,
// serialised context per device.
class DeviceContext {
public:
    struct Lease {
        DeviceContext *ctx;
        std::unique_lock<std::mutex> lk;
    };
    static Lease acquire();
    std::mutex mu;
    hipStream_t stream = nullptr;
    int device = 0;
    uint8_t *ensure(size_t bytes);
    uint8_t *ensure_pinned(size_t bytes);  // page-locked host staging
    uint64_t *counter();

private:
    uint8_t *staging_ = nullptr;
    size_t staging_size_ = 0;
    uint8_t *pinned_ = nullptr;
    size_t pinned_size_ = 0;
    uint64_t *counter_ = nullptr;
};

// Host-pointer execution of a compiled map: moves each used input slot
// (`inputs[slot] + offset`, byte_count bytes) into HBM, applies the map and
// copies each output row back to `outputs[slot] + offset`.  Synchronous.  Up to
// Tuning::host_gather_max bytes the used slots are gathered into pinned staging
// (one H2D, the compact map, one D2H, scatter): per-call latency is then a few
// copies, not one pageable transfer per slot.
void run_host(CompiledMap &cm, const uint8_t *const *inputs, uint8_t *const *outputs, int64_t offset,
              int64_t byte_count);
// As run_host, but instead of copying outputs back, returns whether every
// output byte is zero (used for checkSomeShards / isParityCorrect).
bool run_host_all_zero(CompiledMap &cm, const uint8_t *const *inputs, int64_t offset, int64_t byte_count);

// The per-call executor below the CPU/GPU crossover (host_exec.hpp): whether a per-call entry point
// of `byte_count` bytes runs on the calling thread (Tuning::host_exec_max); throws ECX_E_DEVICE
// when the process has no HIP device, as the device path would.
bool host_exec_wanted(int64_t byte_count);

// Host-memory batch over many stripes (host_pipe.cpp): the batch layout of
// launch_apply, but `in`/`out` are host pointers.  Chunks of stripes are
// pipelined H2D (copy stream) -> kernel (compute stream) -> D2H (copy stream)
// through `host_buffers` device buffer sets; only the map's used slots cross
// PCIe.  Synchronous.  Pinned host memory runs at the PCIe rate.
void run_host_batch(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                    uint8_t *out, int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes,
                    int64_t nbytes);

// Part j of `parts` contiguous stripe ranges of nstripes, the remainder on the first parts (the
// rule of shard_stripes, __init__.py; run_host_batch_devices' split).
void stripe_range(int64_t nstripes, int parts, int j, int64_t *begin, int64_t *end);
// run_host_batch over several devices (host_pipe.cpp): device j of `devices` takes the
// contiguous stripe range j of ndev (remainder on the first), on a worker thread of its own
// with that device's pipe.  Refuses bad device ids before any copy; joins every worker, then
// throws the first failing device's error.
void run_host_batch_devices(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                            uint8_t *out, int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes,
                            int64_t nbytes, const int *devices, int ndev);

}  // namespace ecx
