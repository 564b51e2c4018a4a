// host_exec.hpp -- the per-call executor below the CPU/GPU crossover (host_exec.cpp).  Plain C++:
// run_host / run_host_all_zero (engine.cpp) call it after checking Tuning::host_exec_max and that
// the process has a HIP device (the library never computes on the host without one).
#pragma once
#include <cstdint>

#include "codes.hpp"

namespace ecx {
// outputs[out_slot[o]][offset..+byte_count) = sum_j M[o][j] * inputs[in_slot[j]][...]; an output
// may be an input (each 4 KiB block of every row is computed before any is stored), and an
// input that overlaps an output at a shifted address is read from a copy taken first
void host_exec_apply(const LinearMap &m, const uint8_t *const *inputs, uint8_t *const *outputs, int64_t offset,
                     int64_t byte_count);
// whether every output row of the map over the range is zero (isParityCorrect / checkSomeShards)
bool host_exec_all_zero(const LinearMap &m, const uint8_t *const *inputs, int64_t offset, int64_t byte_count);
// the one-coefficient call of encodeParitySingle / code_single: out (=, or ^= with accumulate) c * in
// (in may be out, or overlap it anywhere)
void host_exec_scale(uint8_t c, const uint8_t *in, uint8_t *out, int64_t n, bool accumulate);
int host_exec_isa();  // 2 AVX-512BW + GFNI, 1 AVX2, 0 scalar
// Test hook (tests/native/host_exec_check.cpp): run the given level (-1 = detect) if this CPU has it;
// returns the level, or -1 when the CPU lacks it.  Not thread-safe; not exported by libecx.
int host_exec_force_isa(int level);
}  // namespace ecx
