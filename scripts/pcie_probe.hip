// pcie_probe.hip -- the link's own ceiling for the e2e leg: one large pinned H2D copy alone, one D2H
// alone, and the two at once on separate streams (the host pipe's h2d / d2h streams), GB/s each.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/pcie_probe.hip -o scripts/pcie_probe && ./scripts/pcie_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                           \
    do {                                                                \
        hipError_t e_ = (x);                                            \
        if (e_ != hipSuccess) {                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));   \
            return 1;                                                   \
        }                                                               \
    } while (0)

int main() {
    const size_t up = (size_t)1 << 31, down = (size_t)1 << 30;  // 2 GiB up, 1 GiB down
    uint8_t *hu = nullptr, *hd = nullptr, *du = nullptr, *dd = nullptr;
    CK(hipHostMalloc(&hu, up, hipHostMallocDefault));
    CK(hipHostMalloc(&hd, down, hipHostMallocDefault));
    CK(hipMalloc(&du, up));
    CK(hipMalloc(&dd, down));
    for (size_t i = 0; i < up; i += 4096) hu[i] = (uint8_t)i;
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t a0, a1, b0, b1;
    CK(hipEventCreate(&a0));
    CK(hipEventCreate(&a1));
    CK(hipEventCreate(&b0));
    CK(hipEventCreate(&b1));
    std::vector<float> h2d, d2h, both_up, both_down;
    for (int r = 0; r < 6; ++r) {
        float t = 0;
        CK(hipEventRecord(a0, s1));
        CK(hipMemcpyAsync(du, hu, up, hipMemcpyHostToDevice, s1));
        CK(hipEventRecord(a1, s1));
        CK(hipEventSynchronize(a1));
        CK(hipEventElapsedTime(&t, a0, a1));
        if (r) h2d.push_back(up / (t * 1e-3) / 1e9);
        CK(hipEventRecord(b0, s2));
        CK(hipMemcpyAsync(hd, dd, down, hipMemcpyDeviceToHost, s2));
        CK(hipEventRecord(b1, s2));
        CK(hipEventSynchronize(b1));
        CK(hipEventElapsedTime(&t, b0, b1));
        if (r) d2h.push_back(down / (t * 1e-3) / 1e9);
        CK(hipEventRecord(a0, s1));
        CK(hipEventRecord(b0, s2));
        CK(hipMemcpyAsync(du, hu, up, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(hd, dd, down, hipMemcpyDeviceToHost, s2));
        CK(hipEventRecord(a1, s1));
        CK(hipEventRecord(b1, s2));
        CK(hipEventSynchronize(a1));
        CK(hipEventSynchronize(b1));
        float tu = 0, td = 0;
        CK(hipEventElapsedTime(&tu, a0, a1));
        CK(hipEventElapsedTime(&td, b0, b1));
        if (r) both_up.push_back(up / (tu * 1e-3) / 1e9), both_down.push_back(down / (td * 1e-3) / 1e9);
    }
    auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    // D2H into host memory pinned other ways: hipHostMalloc non-coherent / coherent, and
    // hipHostRegister of ordinary pages (what ecx_host_register does for a caller's buffer)
    struct Kind {
        const char *name;
        unsigned flags;
        bool reg, touch;
    } kinds[] = {{"default", hipHostMallocDefault, false, false},
                 {"default_touched", hipHostMallocDefault, false, true},
                 {"noncoherent", hipHostMallocNonCoherent, false, false},
                 {"coherent", hipHostMallocCoherent, false, false},
                 {"registered", 0, true, true}};
    for (const Kind &k : kinds) {
        uint8_t *h = nullptr;
        if (k.reg) {
            h = (uint8_t *)aligned_alloc(4096, down);
        } else {
            CK(hipHostMalloc(&h, down, k.flags));
        }
        if (k.touch)
            for (size_t i = 0; i < down; i += 4096) h[i] = 0;  // the CPU writes every page first
        if (k.reg) CK(hipHostRegister(h, down, hipHostRegisterDefault));
        std::vector<float> v, vu;
        for (int r = 0; r < 5; ++r) {
            float t = 0;
            CK(hipEventRecord(b0, s2));
            CK(hipMemcpyAsync(h, dd, down, hipMemcpyDeviceToHost, s2));
            CK(hipEventRecord(b1, s2));
            CK(hipEventSynchronize(b1));
            CK(hipEventElapsedTime(&t, b0, b1));
            if (r) v.push_back(down / (t * 1e-3) / 1e9);
            CK(hipEventRecord(b0, s2));
            CK(hipMemcpyAsync(dd, h, down, hipMemcpyHostToDevice, s2));
            CK(hipEventRecord(b1, s2));
            CK(hipEventSynchronize(b1));
            CK(hipEventElapsedTime(&t, b0, b1));
            if (r) vu.push_back(down / (t * 1e-3) / 1e9);
        }
        printf("{\"probe\": \"pcie_host_kind\", \"kind\": \"%s\", \"d2h_GBps\": %.2f, \"h2d_GBps\": %.2f}\n", k.name, med(v),
               med(vu));
        if (k.reg) {
            CK(hipHostUnregister(h));
            free(h);
        } else {
            CK(hipHostFree(h));
        }
    }
    printf("{\"probe\": \"pcie\", \"h2d_alone_GBps\": %.2f, \"d2h_alone_GBps\": %.2f, \"h2d_with_d2h_GBps\": %.2f, "
           "\"d2h_with_h2d_GBps\": %.2f, \"bytes_up\": %zu, \"bytes_down\": %zu}\n",
           med(h2d), med(d2h), med(both_up), med(both_down), up, down);
    return 0;
}
