// clay_rtc.hpp -- the per-helper-plane Clay repair kernel, generated for one repair
// program (ClayRepairProgram, codes.hpp) and compiled at run time with hiprtc.
//
// The composed-map kernels (k_gf_apply) spend 3 half-rate v_perm_b32 + 2 v_bitop3 per
// dword and coefficient: Clay(10,4)'s 4,672 coefficients per byte position keep the
// vector pipe busy.  This kernel executes the repair in its stage
// structure instead, in bit planes (bits.hpp's transpose), with every coefficient a
// compile-time constant: a multiply is a fixed XOR network over the 8 planes, chosen
// by the generator, with no table operands and no scalar branches.  The plane-decode
// matrix is the same for every helper plane, so one loop body (one helper plane per
// workgroup) serves all of them and the code stays small.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "codes.hpp"

namespace ecx {

constexpr int kRtcThreads = 128;  // 128 lanes x 32 bytes = one 4 KiB chunk

// Code-generation shape (ecx_tune "rtc_lookahead" / "rtc_waves" / "rtc_xcd"): items whose
// loads are issued ahead of the one being computed, the minimum waves per SIMD the
// register budget is set for, and the block order.
struct RtcShape {
    int lookahead = 1;
    int waves = 3;
    int xcd_local = 0;  // 1: the helper planes of one (stripe, chunk) run on one XCD (shared L2)
    int group = 0;      // 1: the plane-group kernel (k_clay_repair_grp) where the program allows it
    int persist = 0;    // plane-group kernel: > 0 = a persistent grid of this many workgroups per CU
    // plane-group kernel, DIAGNOSTIC builds (ecx_tune "rtc_diag", needs ECX_DIAGNOSTIC=1; the
    // outputs are not the repair): each bit removes one part of the kernel, to price it --
    // 1 the row-yc partner loads (the partner is the node's own sub-chunk), 2 the LDS exchange
    // and its barrier (row yb partners = own values), 4 the lane-row exchange (row ya partners
    // = own values), 8 the output stores but one, 16 the bit-plane transposes
    int diag = 0;
    // plane-group kernel: 512-B slices per workgroup, 1 or 2 (software-pipelined: the second
    // slice's rows yb and ya are loaded while the first finishes; ecx_tune "rtc_units")
    int units = 1;
    // plane-group kernel load schedule: 0 = rtc_lookahead's, 1 = lean (row-yc pairs loaded just
    // ahead of use, none in flight during the row-ya exchange: 119 VGPRs, 4 waves/SIMD), 2 =
    // every load of a unit issued up front, the accumulators pinned after every node
    int sched = 2;
    // non-temporal loads (ecx_tune "rtc_nt", bits): plane-group kernel -- 1 the sub-chunks read
    // once (rows ya and yb, the column mates), 2 the row-yc own sub-chunks (re-read as partners
    // by the neighbouring plane groups), 4 the row-yc partner loads; per-plane kernel -- 8: every
    // load (its own sub-chunks are re-read as partners, from L2)
    int nt = 5;
    // plane-group kernel: 64-bit load addresses (flat global loads) instead of 32-bit buffer
    // offsets, for layouts whose input slot offsets exceed 31 bits (1 MiB sub-chunks: a 3.5 GiB
    // Clay(10,4) stripe).  Set by the launcher from the layout, not a tuning knob.
    int wide = 0;
};

// HIP source of the kernel `k_clay_repair` for this program (exposed for tests).
std::string clay_rtc_source(const ClayRepairProgram &pg, const RtcShape &shape = RtcShape());

// The plane-group kernel `k_clay_repair_grp` (clay_rtc.cpp): one 256-thread workgroup
// per (stripe, 512-B slice, q x q square of helper planes), partners exchanged on chip.
// Supported for q == 4 codes with at least two free plane digits (Clay(12,4), the
// shortened Clay(10,4), Clay(8,4), ...); `why` gets the reason otherwise.
bool clay_grp_supported(const ClayRepairProgram &pg, std::string *why = nullptr);
std::string clay_grp_source(const ClayRepairProgram &pg, const RtcShape &shape = RtcShape());
// The shape the current tuning (ecx_tune "rtc_lookahead", "rtc_group", ...) selects, read
// in one snapshot, and the source of the kernel it selects for `pg`.
RtcShape rtc_current_shape();
std::string clay_rtc_selected_source(const ClayRepairProgram &pg, const RtcShape &shape);

class ClayRtc {
public:
    explicit ClayRtc(ClayRepairProgram pg);
    ~ClayRtc();
    const ClayRepairProgram &program() const { return pg_; }
    // The kernel `shape` selects for this program: "k_clay_repair_grp" or "k_clay_repair".
    const char *kernel_name(const RtcShape &shape) const;
    // Compile (hiprtc, once per process and target) and load (once per device) the kernel
    // `shape` selects, uploading its program table on `stream`.  False (with the reason)
    // when hiprtc, the compile or the module load fails; a failure is remembered per
    // (source, device) and not retried, so an auto path falls back at no further cost.
    bool available(const RtcShape &shape, hipStream_t stream, std::string *why = nullptr);
    // Enqueue the repair of `nchunks` whole 4 KiB chunks (bytes [0, nchunks * 4 KiB) of
    // every sub-chunk) over nstripes stripes, in the performCoding batch layout, with the
    // kernel `shape` selects.  Throws ECX_E_DEVICE when that kernel is not available.
    void launch(const RtcShape &shape, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                uint8_t *out, int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes, int64_t nchunks,
                hipStream_t stream);

private:
    bool prepare(const RtcShape &shape, const std::string &src, hipStream_t stream, std::string *why);
    struct Impl;
    ClayRepairProgram pg_;
    std::unique_ptr<Impl> impl_;
};

// Compile `source` with hiprtc (diagnostics / tests: no device needed).
// Returns the code object size, throws ECX_E_DEVICE with the compiler log on failure.
size_t rtc_compile_check(const std::string &source);

// Shared by the generated kernels (clay_rtc.cpp, map_rtc.cpp): hiprtc compilation to a
// code object for `arch` (empty = the current device's target ID, or the library's build
// ARCH without a device; throws ECX_E_DEVICE with the log), the common device prelude
// (bit-plane transpose tr/untr, the 3-input XOR x3, uniform64), and the bit-plane
// multiply: plane i of c*x is the XOR of the planes j in plane_sets(c)[i].
std::string rtc_offload_arch();
std::vector<char> rtc_compile(const std::string &source, const std::string &arch = std::string());
const char *rtc_prelude();
std::vector<std::vector<int>> plane_sets(uint8_t c);

}  // namespace ecx
