// copy3d_probe.hip -- can one 3D copy replace a chunk's per-run strided copies on the host pipe?
// Shortened Clay(10,4), node 0 erased, 4 KiB sub-chunks: a stripe is 3,584 sub-chunks (256 planes x
// 14 nodes); the repair reads nodes 1-13 of planes 0-63: 64 runs of 13 sub-chunks, 14 apart, which
// do not span the stripe, so host_pipe.cpp's fold (2D, count x stripes rows) cannot take them.
// Timed H2D from pinned memory into a compact [stripe][832][4 KiB] buffer, 157 stripes a chunk:
//   runs2d: one hipMemcpy2DAsync per run (157 rows each) -- what the host pipe does now;
//   copy3d: one hipMemcpy3DAsync (13 x 4 KiB wide, 64 rows 57,344 B apart, 157 slices a stripe apart);
//   span:   one hipMemcpy2DAsync of the whole 896-sub-chunk span per stripe (7.7 % more bytes).
// Bytes compared between runs2d and copy3d; prints GB/s of the 832 used sub-chunks.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/copy3d_probe.hip -o scripts/copy3d_probe && ./scripts/copy3d_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 1;                                                           \
        }                                                                       \
    } while (0)

int main() {
    const int64_t B = 4096, slots = 3584, used = 832, run = 13, step = 14, nruns = 64, rows = 157;
    const int64_t stripe = slots * B, per = used * B, chunks = 2;
    uint8_t *host = nullptr, *dev = nullptr, *dev2 = nullptr;
    CK(hipHostMalloc(&host, (size_t)(stripe * rows * chunks), hipHostMallocDefault));
    for (int64_t i = 0; i < stripe * rows * chunks; i += 4096) host[i] = (uint8_t)(i >> 12), host[i + 1] = (uint8_t)(i >> 20);
    CK(hipMalloc(&dev, (size_t)(per * rows)));
    CK(hipMalloc(&dev2, (size_t)(896 * B * rows)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto runs2d = [&](int c) -> hipError_t {
        const uint8_t *src = host + c * rows * stripe + 1 * B;  // node 1 of plane 0
        for (int64_t r = 0; r < nruns; ++r) {
            hipError_t e = hipMemcpy2DAsync(dev + r * run * B, (size_t)per, src + r * step * B, (size_t)stripe,
                                            (size_t)(run * B), (size_t)rows, hipMemcpyHostToDevice, s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    };
    auto copy3d = [&](int c) -> hipError_t {
        hipMemcpy3DParms p;
        memset(&p, 0, sizeof(p));
        p.srcPtr = make_hipPitchedPtr((void *)(host + c * rows * stripe + 1 * B), (size_t)(step * B), (size_t)(run * B),
                                      (size_t)(stripe / (step * B)));
        p.dstPtr = make_hipPitchedPtr(dev, (size_t)(run * B), (size_t)(run * B), (size_t)(per / (run * B)));
        p.extent = make_hipExtent((size_t)(run * B), (size_t)nruns, (size_t)rows);
        p.kind = hipMemcpyHostToDevice;
        return hipMemcpy3DAsync(&p, s);
    };
    auto span = [&](int c) -> hipError_t {
        return hipMemcpy2DAsync(dev2, (size_t)(896 * B), host + c * rows * stripe, (size_t)stripe, (size_t)(896 * B),
                                (size_t)rows, hipMemcpyHostToDevice, s);
    };
    // bytes: runs2d and copy3d must fill dev identically
    std::vector<uint8_t> a((size_t)(per * rows)), b((size_t)(per * rows));
    CK(runs2d(1));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(a.data(), dev, a.size(), hipMemcpyDeviceToHost));
    CK(hipMemset(dev, 0, a.size()));
    CK(copy3d(1));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(b.data(), dev, b.size(), hipMemcpyDeviceToHost));
    const bool same = a == b;
    const char *names[3] = {"runs2d", "copy3d", "span"};
    std::vector<float> ms[3];
    for (int round = 0; round < 5; ++round)
        for (int k = 0; k < 3; ++k) {
            CK(hipEventRecord(e0, s));
            for (int c = 0; c < chunks; ++c) CK(k == 0 ? runs2d(c) : k == 1 ? copy3d(c) : span(c));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (round) ms[k].push_back(t);
        }
    for (int k = 0; k < 3; ++k) {
        std::sort(ms[k].begin(), ms[k].end());
        const float med = ms[k][ms[k].size() / 2];
        printf("{\"probe\": \"copy3d\", \"case\": \"%s\", \"copies_per_chunk\": %d, \"ms_2_chunks\": %.3f, "
               "\"used_GBps\": %.2f, \"same_bytes_as_runs2d\": %s}\n",
               names[k], k == 0 ? (int)nruns : 1, med, (double)per * rows * chunks / (med * 1e-3) / 1e9,
               k == 1 ? (same ? "true" : "false") : "null");
    }
    return same ? 0 : 4;
}
