// host_pipe.hpp -- the read-only host-memory batches of host_pipe.cpp (the check; the
// map batches are declared with the engine, engine.hpp).
#pragma once

#include <functional>

#include "engine.hpp"

namespace ecx {

// launch_check over host-memory stripes: the check map's used slots of each chunk of stripes
// go H2D, k_gf_check writes the chunk's verdict bytes on the device and only those come back
// into the host array `verdict` (one byte per stripe).  Synchronous, on the current device.
void run_host_check_batch(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                          int64_t nstripes, int64_t nbytes, uint8_t *verdict);
// run_host_check_batch split over a device list, as run_host_batch_devices (engine.hpp).
void run_host_check_batch_devices(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride,
                                  int64_t in_slot_stride, int64_t nstripes, int64_t nbytes, uint8_t *verdict,
                                  const int *devices, int ndev);

// How run_host_batch moves a batch (ecx_map_host_plan, include/ecx_tune.h): stripes per chunk, the
// chunk count, device buffer sets in flight, and per chunk the H2D / D2H copies, the most rows per
// stripe one copy moves (> 1 where runs are folded or copied in 3D) and how many copies are 3D.
struct HostBatchPlan {
    int64_t chunk = 0, nchunks = 0;
    int buffers = 0;
    int64_t h2d_copies = 0, h2d_rows = 0, d2h_copies = 0, d2h_rows = 0, h2d_3d = 0, d2h_3d = 0;
    int64_t slices = 0;  // column slices of a one-chunk batch (1: whole slots)
};
HostBatchPlan plan_host_batch(CompiledMap &cm, int64_t in_stripe_stride, int64_t in_slot_stride,
                              int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes, int64_t nbytes);

// range(lo, count) over contiguous stripe ranges of nstripes split over a device list, one worker
// thread per entry with that device current: the split, validation and error reporting of
// run_host_batch_devices, for host batches made of several passes (the blocked RS layout).
void for_device_ranges(const int *devices, int ndev, int64_t nstripes,
                       const std::function<void(int64_t, int64_t)> &range);

}  // namespace ecx
