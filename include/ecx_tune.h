/*
 * ecx_tune.h -- launch-shape knobs of libecx.so for diagnostics and tuning.
 * Not part of the reference's coding interface (include/ecx.h is the boundary);
 * results are bit-identical for every setting, only speed changes.
 *
 * Two classes of keys.  DEPLOYMENT keys -- "layout_select", "plan_cache", "roctx" and the
 * host_* keys (host_exec_kib included) -- are always accepted.  Every other key below is a SHAPE key: the product
 * library accepts it only when the process set ECX_SHAPE_KNOBS=1 in its environment before
 * its first ecx_tune call (read once; tests, bench.py --tune and the scripts/ A/B harnesses
 * do), and otherwise refuses it with ECX_E_ILLEGAL_ARGUMENT -- so no caller sharing the
 * process (another library in the same JVM) can reshape every other caller's launches.  The
 * diagnostic library (make DIAG=1) accepts every key.
 *
 *   "depth"            16-B loads per lane in the kernel's load ring: 0 = per map (default:
 *                      20 for a single full tile of 17-20 entries, 8 when every tile has >= 12
 *                      entries, else 4), or force 2 / 4 / 8 / 10 / 12 / 16 / 20 / 24 (2: 8-row
 *                      tiles only; 10-24: single-tile maps with non-temporal loads; otherwise
 *                      clamped)
 *   "nontemporal"      0 = plain loads/stores; 1 = auto (default): non-temporal stores, and
 *                      non-temporal loads for single-tile maps (no input re-read); 2 = always
 *   "xcd_group"        multi-tile maps: 0 = identity block order; 1 = each XCD runs a contiguous
 *                      eighth of the grid; 2 = each XCD runs whole (stripe, chunk) units, all
 *                      tiles of a unit back to back (default: see engine.hpp Tuning); 3 = (any
 *                      map) each XCD runs runs of "xcd_run" consecutive units
 *   "xcd_run"          xcd_group 3: consecutive (stripe, chunk) units per XCD run, 1..4096 (default 8)
 *   "xcd_misaligned"   single-tile maps with "xcd_group" 0 whose input slots are not 128-B aligned
 *                      (their chunks share boundary cache lines): 1 = use the runs of "xcd_group" 3
 *                      (default), 0 = the identity block order
 *   "lds_tables"       0 = all split-table dwords read as scalars (one v_mov per 8-entry table
 *                      and row); 1 = the low dword of each 8-entry table staged per workgroup
 *                      in LDS, for multi-tile maps (default); 2 = for every map
 *   "store_scope"      0 = non-temporal output stores (`nt`, default); 1 = `nt sc0 sc1`
 *                      (system scope: written through, dropped from L2)
 *   "chunk_major"      block order of the one-workgroup-per-tile kernel: 0 = stripe-major
 *                      (default), 1 = chunk-major (chunk c of every stripe, then chunk c + 1)
 *   "stagger"          unit order of the single-tile kernels (k_gf_apply, k_gf_apply_skew): 0 = none
 *                      (default); G = 2..64: G stripes interleaved unit by unit, stripe j of a group
 *                      starting at chunk j*C/G of its C chunks, so the streams in flight sit at G
 *                      different shard offsets (scripts/addr_probe.hip)
 *   "block_threads"    one-workgroup-per-tile kernel: 256 threads over 4 KiB chunks or 64 threads
 *                      (one wave) over 1 KiB chunks; 0 = auto (default): one wave for single-tile
 *                      maps of <= 2 rows over >= 8 inputs on slot pitches that are not 4 MiB multiples
 *   "small_tiles"      single-tile maps of <= 2 or <= 4 rows: 1 = kernel variants with that many
 *                      accumulator rows (fewer VGPRs); 0 = the 8-row kernel; 2 = auto (default):
 *                      the small variant for maps of <= 2 rows over <= 4 inputs (LRC block repair)
 *   "plan_cache"       per-call entry points that receive or derive their coefficients per call
 *                      (ecx_code_some_shards, ecx_check_some_shards, ecx_code_single,
 *                      ecx_rs_encode_parity_single, ecx_rs_decode_missing_single): compiled plans
 *                      kept, by matrix content (default 256; 0 = compile every call)
 *   "skew_chunks"      single-tile maps: 2 / 4 = each workgroup takes that many 4 KiB chunks and
 *                      rotates the chunk each input is read at; 1 = auto (default): per layout by the
 *                      layout selection ("layout_select"), else 4 when the pitch is a multiple of 4 MiB
 *                      and one chunk per workgroup otherwise; 0 = never
 *   "layout_select"    single-tile maps over >= 8 inputs with <= 4 rows (the many-stream RS maps), with the
 *                      knobs "skew_chunks", "block_threads" and "stagger" on auto, on batches of >= 256 MiB of
 *                      input: 1 = the launch shape is chosen per batch layout (map, strides, size classes
 *                      (log2) of the shard and of the batch, device; up to 64 layouts per map) by timing the caller's own first launches -- the static
 *                      rules' shape, 4 KiB and one-wave workgroups, skewed chunks, staggered stripes,
 *                      5 timings each, events read without blocking on later calls -- and the fastest
 *                      median is kept (default; every candidate computes the same bytes, nothing extra
 *                      is launched).  Any kept shape is re-validated once, 512 launches later, against
 *                      its alternative: the static rules for a non-static choice, the runner-up for a
 *                      static one.  0 = the static rules only (skew on 4 MiB-multiple pitches, one
 *                      wave for <= 2-row maps over >= 8 inputs)
 *   "wide_tiles"       multi-tile maps: pairs of 8-row tiles that share inputs in one workgroup
 *                      (16 accumulator rows, each shared input loaded once).  1 = when pairing
 *                      saves >= 1/6 of the input reads (default), 2 = always, 0 = never
 *   "clay_rtc"         Clay single-node repair batches (ecx_clay_perform_coding_batch): the
 *                      per-helper-plane kernel generated for the repair and compiled with hiprtc, for
 *                      the whole 4 KiB chunks of 16-B-aligned layouts: 1 = when the composed map spans
 *                      several 8-row tiles (alpha > 8: Clay(10,4), Clay(12,4); default), 2 = always,
 *                      0 = never (the composed-map kernel only).  If the kernel cannot be compiled
 *                      or loaded (no libhiprtc, another GPU target), auto falls back to the composed
 *                      map (the failure is remembered, not retried); 2 returns ECX_E_DEVICE
 *   "rtc_lookahead"    that kernel's generated load schedule: items (non-column nodes, mates) whose
 *                      loads are issued ahead of the one being computed, 0..3 (bits 0-1; default 1);
 *                      for the plane-group kernel bit 0 = partner and mate loads after row ya, bit 1
 *                      = skip the dot's and virtual partners' transposes by uniform branches, bit 2
 *                      = a second body for plane groups whose memory-row partner is virtual, bit 3 =
 *                      every load issued at the start, bit 4 = DIAGNOSTIC data-movement-only build
 *                      (coefficients taken as 1, no transposes: the outputs are not the repair;
 *                      refused with ECX_E_ILLEGAL_ARGUMENT except in the diagnostic library with
 *                      ECX_DIAGNOSTIC=1 in the environment)
 *   "rtc_waves"        that kernel's __launch_bounds__ minimum waves per SIMD, 2..4 (default 3)
 *   "rtc_group"        Clay single-node repairs of q = 4 codes (Clay(12,4), shortened Clay(10,4)): 1 =
 *                      the plane-group kernel (k_clay_repair_grp: a q x q square of helper planes
 *                      per workgroup, partners exchanged in registers and LDS; default), 0 = one
 *                      helper plane per workgroup
 *   "rtc_sched"        the plane-group kernel's load schedule: 0 = rtc_lookahead's, 1 = lean: no
 *                      row-yc load in flight during the row-ya exchange, the row-yc (own, partner)
 *                      pairs loaded 1 + (rtc_lookahead & 3) pairs ahead of use, the accumulators pinned
 *                      after every node -- 119 VGPRs and 4 waves per SIMD instead of 154 and 3; 2 =
 *                      every load of a unit issued up front, the accumulators pinned (151 VGPRs;
 *                      default)
 *   "rtc_wide"         the plane-group kernel's load addresses: 0 = 32-bit buffer offsets, and 64-bit
 *                      flat addresses only where a stripe's slot offsets exceed 31 bits (1 MiB sub-chunks
 *                      of Clay(10,4), default); 1 = 64-bit on every layout (A/B, tests)
 *   "rtc_nt"           non-temporal loads in the generated Clay kernels, bits: plane-group kernel --
 *                      1 the sub-chunks read once (rows ya and yb, the column mates), 2 the row-yc
 *                      own sub-chunks (re-read as partners by the neighbouring plane groups), 4 the
 *                      row-yc partner loads; per-plane kernel -- 8 every load; 0..15, default 5
 *   "rtc_xcd"          that kernel's block order: 1 = the helper planes of one (stripe, chunk) on one
 *                      XCD (their shared partner loads meet in its L2), 0 = plane-fastest; 2 = the
 *                      same, and for the plane-group kernel all slices and plane groups of one
 *                      (stripe, chunk) on one XCD, plane-group-fastest (default); 3 = the same, slice-fastest; 4 = as 3
 *                      with a contiguous range of (stripe, chunk) units per XCD
 *   "map_planes"       the bit-plane kernel generated for one composed map and compiled with hiprtc
 *                      (k_map_planes: every row of a <= 16-row map in registers, coefficients as
 *                      fixed XOR networks over the 8 bit planes of each input), for the full 4 KiB
 *                      chunks of 16-B-aligned layouts whose slot offsets fit 31 bits: 1 = auto
 *                      (default) for multi-tile maps with >= 4 coefficients per used input on
 *                      batches of >= 64 MiB of input (the Clay(4,2) two-node repairs), 2 = wherever
 *                      it fits, 0 = never; the same compile/load fallback as "clay_rtc"
 *   "planes_lookahead" that kernel's load schedule: inputs in flight ahead of the one being
 *                      computed, 0..15 (default 12)
 *   "planes_waves"     that kernel's __launch_bounds__ minimum waves per SIMD, 1..4 (default 2)
 *   "host_contexts"    per-call host entry points: 1 = each call leases a free context (stream and
 *                      staging areas) of the device, so calls from several threads overlap (default);
 *                      0 = one context per device, calls serialised
 *   "roctx"            1 = a roctx range named after the entry point around every C-ABI call that
 *                      can fail (shown by `rocprofv3 --marker-trace`; also ECX_ROCTX=1 in the
 *                      environment at load), 0 = none (default)
 *   "host_chunk_kib"   host-memory batches: input KiB per pipelined H2D chunk (default 65536)
 *   "host_buffers"     host-memory batches: device buffer sets in flight, 1..8 (default 3)
 *   "host_gather_kib"  per-call host entry points: byte counts up to this many KiB are gathered
 *                      through pinned staging (one H2D / one D2H); 0 = always per-slot copies
 *                      (default 512)
 *   "host_exec_kib"    per-call host entry points (the CodingLoop / ReedSolomon / Clay byte[][] calls):
 *                      byte counts up to this many KiB run on the calling thread (host_exec.cpp:
 *                      AVX-512 GFNI affine multiplies, else AVX2 nibble tables) instead of a device
 *                      round trip (default 1024: the measured crossover -- one caller thread, the
 *                      device first beats the executor at 2 MiB on Clay(4,2) performCoding and at no
 *                      size up to 4 MiB on the RS(2,2) pair; 16 caller threads, at no size;
 *                      profiles/r06_percall_threshold.jsonl; 0 = every call on the device).  Never a
 *                      fallback: without a HIP device these calls fail with ECX_E_DEVICE like the
 *                      device path
 *   "host_zero_copy"   per-call host entry points on the gather path: 1 = the kernel reads and
 *                      writes the pinned staging area over PCIe (no DMA copies; default);
 *                      0 = one H2D and one D2H copy
 *
 * Diagnostic library only ("make DIAG=1" builds libecx_diag.so with the same ABI; load it with
 * ECX_LIB_PATH).  These are the measured-and-rejected kernels and builds DESIGN.md section 4
 * records; the product library libecx.so does not contain them and ecx_tune refuses their keys
 * with ECX_E_ILLEGAL_ARGUMENT (ecx_build_diag() tells the two apart):
 *   [DIAG] "wave_groups"      multi-tile maps: one workgroup per group of tiles sharing inputs, one
 *                      wave per tile, 1 KiB chunks: 1 = the group's input union staged once
 *                      through LDS; 2 = each wave loads its own entries (no LDS, no barriers);
 *                      0 = one workgroup per tile (default)
 *   [DIAG] "occ_lds"          extra dynamic LDS bytes per k_gf_apply workgroup, which caps the workgroups
 *                      resident per CU at floor(160 KiB / bytes): 0 = no cap (default), -1 = the
 *                      single-tile maps over >= 8 inputs on rings of <= 8 loads at 4 waves per
 *                      SIMD, 1..65536 = that many bytes
 *   [DIAG] "bitslice"         the bit-sliced kernel (k_gf_bits: 32 bytes per lane as 8 bit planes, GF
 *                      multiplies as XORs of the planes of 2^k x) for the full 4 KiB chunks of
 *                      aligned layouts whose slot offsets fit 31 bits: 1 = for multi-tile maps
 *                      that do not run as wide tiles, 2 = for every such map, 0 = never (default;
 *                      measured slower, bound by its scalar branches)
 *   [DIAG] "lds_lut"          per-byte lookup tables in LDS (k_gf_lut) for the full 4 KiB chunks of
 *                      aligned layouts: 1 = log/antilog tables (LOG u16, EXP 1 KiB), 2 = one 256-B
 *                      product row per coefficient (single-tile maps of <= 256 general
 *                      coefficients); 0 = never (default: measured slower)
 *   [DIAG] "rtc_diag"         the plane-group kernel's DIAGNOSTIC builds, 0 = none (default); bits remove one
 *                      part each to price it (1 row-yc partner loads, 2 LDS exchange + barrier, 4
 *                      lane-row exchange, 8 output stores but one, 16 bit-plane transposes): the
 *                      outputs are not the repair, so any non-zero value is refused with
 *                      ECX_E_ILLEGAL_ARGUMENT unless the environment has ECX_DIAGNOSTIC=1
 *   [DIAG] "rtc_units"        the plane-group kernel's 512-B slices per workgroup: 1 (default), or 2 with the
 *                      second slice's first two rows loaded while the first slice finishes (software
 *                      pipelining across the exchange barrier; no persistent grid)
 *   [DIAG] "units"            single-tile maps on the default non-temporal shape: (stripe, chunk) units per
 *                      workgroup with one load ring running across them, so a unit's stores leave
 *                      while the next unit's loads are in flight (k_gf_apply_multi): 1 = one unit per
 *                      workgroup (default), 2 or 4; measured 3-16 % slower on every single-tile map
 *                      (profiles/r05_units_ab.jsonl)
 *   [DIAG] "rtc_persist"      the plane-group kernel's grid: 0 = one workgroup per unit (default), 1..8 =
 *                      a persistent grid of that many workgroups per CU walking the units
 */
#ifndef ECX_TUNE_H
#define ECX_TUNE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
int ecx_tune(const char *key, int value); /* 0, or ECX_E_ILLEGAL_ARGUMENT for an unknown key */
/* The current value of a DEPLOYMENT key (in ecx_tune's units, e.g. "host_exec_kib" in KiB) into
 * *value: 0, or ECX_E_ILLEGAL_ARGUMENT for a shape key, an unknown key or a null pointer. */
int ecx_tune_value(const char *key, int *value);
/* 1 in the diagnostic library (make DIAG=1, libecx_diag.so), 0 in the product library. */
int ecx_build_diag(void);
/* The per-call host executor's instruction set ("host_exec_kib"): 2 AVX-512BW + GFNI, 1 AVX2,
 * 0 scalar. */
int ecx_host_exec_isa(void);
/* The stripe range [*begin, *end) that device entry j of `parts` takes in the multi-GPU host
 * batches (ecx_*_batch_host_devices): contiguous ranges, the remainder on the first entries.
 * Host-only; ECX_E_ILLEGAL_ARGUMENT for a bad request. */
int ecx_stripe_range(int64_t nstripes, int parts, int j, int64_t *begin, int64_t *end);
/* Pure-bandwidth probes over nbytes (multiple of 16 KiB) of device memory:
 * kind 0 = read-only stream, kind 1 = copy src -> dst.  Enqueued on `stream`. */
int ecx_probe_bandwidth(int kind, const uint8_t *src, uint8_t *dst, int64_t nbytes, int nontemporal, void *stream);
/* Host-only plan self-test: interprets the compiled plan of `map` (entry tables,
 * tiles, tile groups and their LDS unions) on pseudo-random bytes and compares
 * with the dense GF(256) map.  0 = consistent, else ECX_E_ILLEGAL_ARGUMENT. */
struct ecx_map;
int ecx_map_selftest(const struct ecx_map *map, uint64_t seed);
/* Plan shape: row tiles, tile entries (= input loads of the one-workgroup-per-tile
 * kernel), tile groups, and the summed group unions (= input loads of the LDS kernel). */
int ecx_map_plan_stats(const struct ecx_map *map, int *n_tiles, int *n_entries, int *n_groups, int *union_total);
/* The launch shape "layout_select" kept for the most recently selected batch layout of
 * `map` with input slot pitch `slot_pitch`: 0x200 = none chosen yet (still exploring, or not
 * eligible); the static rules' shape = 0x100; any other = shape + 8 * stagger, shape 0 =
 * 256-thread workgroups over 4 KiB chunks, 1 = skewed chunks, 2 = one-wave workgroups over
 * 1 KiB chunks.  With median_ms (n entries), the median launch time of each candidate in the
 * selector's order (-1 = unsampled).  Negative: a status (null map, pitch <= 0, n < 0). */
int ecx_map_layout_choice(const struct ecx_map *map, int64_t slot_pitch, float *median_ms, int n);
/* State of that layout's selection: -1 none yet, 0 exploring, 1 chosen, 2 re-validating, 3
 * re-validated (final), 4 contended (probes kept overlapping other streams' launches: the static
 * rules, untimed); `dropped` = timing probes discarded because another stream of the device
 * launched between the probing stream's previous launch and the probe's end (a launch that
 * finds the probe already finished does not count).  Either pointer may be NULL. */
int ecx_map_layout_state(const struct ecx_map *map, int64_t slot_pitch, int *state, int *dropped);
/* How ecx_map_apply_batch_host would move a batch of this layout (host_pipe.cpp; host-only, no
 * device touched): plan[10] = {stripes per pipelined chunk, chunks, device buffer sets in flight,
 * H2D copies per chunk, the most rows per stripe one H2D copy moves, D2H copies per chunk, the
 * same for D2H, H2D copies that are 3D, D2H copies that are 3D, column slices}.  Runs of used
 * slots that repeat with a fixed step across the stripe are folded into one 2D copy per period,
 * other progressions of equal runs at fixed steps are one 3D copy each (rows per stripe > 1).  A
 * batch that fits one chunk of stripes but holds at least 4 chunks of input is pipelined over
 * column slices of ~host_chunk_kib instead (slices > 1; the copies are then per slice: one per
 * progression of runs per stripe).  All zero when the batch moves nothing. */
int ecx_map_host_plan(const struct ecx_map *map, int64_t in_stripe_stride, int64_t in_slot_stride,
                      int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes, int64_t byte_count,
                      int64_t *plan);
/* The kernel instance of the last full-chunk launch this thread enqueued, named as
 * rocprofv3 names it (e.g. "k_gf_apply<false, true, 1, 20, false, 256, 8>"), copied
 * NUL-terminated into buf.  Returns its length (0 = no launch yet), or
 * ECX_E_ILLEGAL_ARGUMENT if buf is null or shorter than length + 1. */
int ecx_last_kernel(char *buf, int len);
/* The same launch's full shape: the kernel instance followed by the unit order its name does not
 * encode -- "k_gf_apply<...> stagger=G xcd_group=X xcd_run=R [skew=K]" for the composed-map
 * kernels, the bare name for the generated Clay kernels.  Same buffer contract. */
int ecx_last_launch_shape(char *buf, int len);
/* The per-helper-plane Clay repair kernel (ecx_tune "clay_rtc"): builds the clay
 * step's repair program (checked against the composed reference map), generates the
 * kernel source and compiles it with hiprtc for gfx950 -- no device needed.  Returns
 * the code-object size, ECX_E_ILLEGAL_ARGUMENT if the step has no such program (not a
 * single-node repair), ECX_E_DEVICE if hiprtc is missing or fails. */
struct ecx_clay;
int ecx_clay_rtc_compile_check(struct ecx_clay *clay);
/* The generated kernel source: copied NUL-terminated into buf when len exceeds its
 * length; returns the length. */
int ecx_clay_rtc_source(struct ecx_clay *clay, char *buf, int len);
/* The bit-plane kernel of a composed map (ecx_tune "map_planes"), overwriting or, with
 * accumulate != 0, XOR-accumulating its outputs: compile it with hiprtc for gfx950 (no
 * device needed) and return the code-object size, or copy its source NUL-terminated into
 * buf when len exceeds its length and return the length.  ECX_E_ILLEGAL_ARGUMENT if the
 * map does not fit the kernel (more than 16 rows), ECX_E_DEVICE if hiprtc fails. */
int ecx_map_planes_compile_check(const struct ecx_map *map, int accumulate);
int ecx_map_planes_source(const struct ecx_map *map, int accumulate, char *buf, int len);
/* The process-wide codec registry (ecx.h, ecx_rs_create): codecs with live references and
 * idle cached ones, for RS and Clay.  Any pointer may be NULL. */
int ecx_codec_stats(int *rs_live, int *rs_idle, int *clay_live, int *clay_idle);
#ifdef __cplusplus
}
#endif
#endif
