// Does work on the null stream (or a device sync, or hipFree) wait for a long-running kernel on a
// CU-masked stream (hipExtStreamCreateWithCUMask has no flags argument: is the stream blocking)?
// The resident one-key reader runs on such a stream for up to 200 ms.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o cumask_block cumask_block.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__global__ void k_spin(uint64_t ticks) {  // one wave, wall-clock bounded
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
__global__ void k_nop(int* p) { if (threadIdx.x == 0 && p) p[0] = 1; }

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
    int khz = 0, ncu = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<uint32_t> mask((ncu + 31) / 32, ~0u);
    if (ncu % 32) mask.back() = (1u << (ncu % 32)) - 1u;
    hipStream_t cm = nullptr, nb = nullptr;
    CK(hipExtStreamCreateWithCUMask(&cm, uint32_t(mask.size()), mask.data()));
    CK(hipStreamCreateWithFlags(&nb, hipStreamNonBlocking));
    unsigned int flags = 99;
    CK(hipStreamGetFlags(cm, &flags));
    printf("cu-mask stream flags %u (hipStreamNonBlocking = %u)\n", flags, unsigned(hipStreamNonBlocking));
    int* d = nullptr;
    CK(hipMalloc(&d, 64));
    const uint64_t spin = uint64_t(khz) * 100;  // 100 ms
    struct Case { const char* what; int kind; };
    const Case cases[] = {{"kernel on a non-blocking stream + its sync", 0}, {"null-stream kernel + null sync", 1},
                          {"hipDeviceSynchronize", 2}, {"hipMalloc + hipFree", 3}, {"hipMemsetAsync null + sync", 4}};
    for (const Case& c : cases) {
        k_spin<<<1, 64, 0, cm>>>(spin);
        CK(hipGetLastError());
        auto t0 = std::chrono::steady_clock::now();
        if (c.kind == 0) { k_nop<<<1, 64, 0, nb>>>(d); CK(hipStreamSynchronize(nb)); }
        if (c.kind == 1) { k_nop<<<1, 64, 0, nullptr>>>(d); CK(hipStreamSynchronize(nullptr)); }
        if (c.kind == 2) CK(hipDeviceSynchronize());
        if (c.kind == 3) { void* p = nullptr; CK(hipMalloc(&p, 1 << 20)); CK(hipFree(p)); }
        if (c.kind == 4) { CK(hipMemsetAsync(d, 0, 64, nullptr)); CK(hipStreamSynchronize(nullptr)); }
        printf("%-45s %8.3f ms (spin 100 ms on the cu-mask stream)\n", c.what, ms_since(t0));
        CK(hipStreamSynchronize(cm));
    }
    // Which stream can host a persistent wave without holding up other streams' kernels: 8
    // non-blocking streams (the library's pool) each run a nop + sync while the wave spins on
    // (a) the CU-masked stream, (b) a plain non-blocking stream, (c) a high-priority non-blocking
    // stream; and whether the null stream waits for (c).
    std::vector<hipStream_t> pool(8);
    for (auto& s : pool) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t plain = nullptr, prio = nullptr;
    CK(hipStreamCreateWithFlags(&plain, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&prio, hipStreamNonBlocking, hi));
    printf("priority range least %d greatest %d\n", lo, hi);
    const hipStream_t hosts[3] = {cm, plain, prio};
    const char* names[3] = {"cu-mask stream", "plain non-blocking stream", "high-priority non-blocking stream"};
    for (int h = 0; h < 3; ++h) {
        k_spin<<<1, 64, 0, hosts[h]>>>(spin);
        CK(hipGetLastError());
        double worst = 0;
        for (auto& s : pool) {
            auto t0 = std::chrono::steady_clock::now();
            k_nop<<<1, 64, 0, s>>>(d);
            CK(hipStreamSynchronize(s));
            worst = std::max(worst, ms_since(t0));
        }
        auto t1 = std::chrono::steady_clock::now();
        CK(hipMemsetAsync(d, 0, 64, nullptr));
        CK(hipStreamSynchronize(nullptr));
        const double null_ms = ms_since(t1);
        printf("spin on %-36s: worst pool-stream nop %8.3f ms, null-stream memset %8.3f ms\n", names[h], worst, null_ms);
        CK(hipStreamSynchronize(hosts[h]));
    }
    // with the wave on the high-priority non-blocking stream: hipMalloc, hipFree, a device sync,
    // and hipMallocAsync / hipFreeAsync on the null stream
    struct Op { const char* what; int kind; };
    const Op ops[] = {{"hipMalloc 64 MiB", 0}, {"hipFree", 1}, {"hipDeviceSynchronize", 2},
                      {"hipMallocAsync + null sync", 3}, {"hipFreeAsync + null sync", 4}};
    void* big = nullptr;
    void* pooled = nullptr;
    for (const Op& o : ops) {
        k_spin<<<1, 64, 0, prio>>>(spin);
        CK(hipGetLastError());
        auto t0 = std::chrono::steady_clock::now();
        if (o.kind == 0) CK(hipMalloc(&big, size_t(64) << 20));
        if (o.kind == 1) CK(hipFree(big));
        if (o.kind == 2) CK(hipDeviceSynchronize());
        if (o.kind == 3) { CK(hipMallocAsync(&pooled, size_t(64) << 20, nullptr)); CK(hipStreamSynchronize(nullptr)); }
        if (o.kind == 4) { CK(hipFreeAsync(pooled, nullptr)); CK(hipStreamSynchronize(nullptr)); }
        printf("wave on the high-priority stream: %-30s %8.3f ms\n", o.what, ms_since(t0));
        CK(hipStreamSynchronize(prio));
    }
    return 0;
}
