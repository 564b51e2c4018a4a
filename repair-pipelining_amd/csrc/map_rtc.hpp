// map_rtc.hpp -- a composed GF(256) map executed in bit planes by a kernel generated for
// that map and compiled at run time with hiprtc (k_map_planes).
//
// The split-table kernels (k_gf_apply*, kernels.hip) spend 3 half-rate v_perm_b32 +
// 2 v_bitop3 per dword and coefficient; on maps with many coefficients per input (the
// Clay(4,2) two-node repair: 184 over 32 inputs) that vector work, not HBM, sets the
// pace.  Here every input sub-chunk is turned into 8 bit planes
// once, and each coefficient is a fixed XOR network over them, baked into the code: the
// planes of one input are split into a low and a high nibble, every subset of a nibble
// that some output plane needs is materialised once, and each output plane then takes
// one 3-input XOR per input.  All rows of the map (at most kPlanesMaxRows) stay in
// registers, so each input is read from HBM exactly once per chunk.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>

#include "codes.hpp"

namespace ecx {

constexpr int kPlanesThreads = 128;  // 128 lanes x 32 bytes = one 4 KiB chunk
constexpr int kPlanesMaxRows = 16;   // 16 rows x 8 planes = 128 accumulator VGPRs
constexpr int kPlanesMaxNnz = 1024;  // code size bound (~12 instructions per coefficient)

struct PlanesShape {
    int lookahead = 12;  // inputs whose loads are in flight ahead of the one being computed
    int waves = 2;      // __launch_bounds__ minimum waves per SIMD (VGPR budget)
    bool nt_loads = true;
};

// Whether `m` fits the generated kernel (rows, code size); `why` gets the reason if not.
bool map_planes_supported(const LinearMap &m, std::string *why = nullptr);
// HIP source of k_map_planes for `m` (exposed for tests).  With `accumulate` the kernel
// XORs into the existing outputs (out ^= M * in) instead of overwriting them.
std::string map_planes_source(const LinearMap &m, const PlanesShape &shape, bool accumulate);

class MapPlanes {
public:
    explicit MapPlanes(LinearMap m);
    ~MapPlanes();
    const LinearMap &map() const { return map_; }
    static const char *kernel_name() { return "k_map_planes"; }
    // Enqueue out (^)= M * in over bytes [0, nchunks * 4 KiB) of every slot of nstripes
    // stripes (the launch_apply batch layout).  Inputs are read through a buffer
    // descriptor with 32-bit slot offsets: the caller guarantees max_in_slot * slot
    // stride + 4 KiB < 2^31 and 16-byte alignment.  Compiles (once per process) and
    // loads (once per device) on first use; throws ECX_E_DEVICE if hiprtc or the load fails.
    void launch(const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride, uint8_t *out,
                int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes, int64_t nchunks, bool accumulate,
                hipStream_t stream);

    // Compiles and loads the kernel the current tuning selects; false (with the reason)
    // when hiprtc, the compile or the module load fails.  A failure is remembered per
    // (source, device), so the auto path falls back to the composed map at no further cost.
    bool available(bool accumulate, std::string *why = nullptr);

private:
    bool load(const PlanesShape &shape, bool accumulate, hipFunction_t *fn, std::string *why);
    struct Impl;
    LinearMap map_;
    std::unique_ptr<Impl> impl_;
};

}  // namespace ecx
