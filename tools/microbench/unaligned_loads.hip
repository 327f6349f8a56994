// Does a 16-byte global load at a byte-unaligned address return the bytes at that address on
// gfx950 (the HSA runtime's unaligned access mode), and what does it cost against aligned
// loads?  Probe for the variable-length key hash (murmur_device.hpp: today five aligned chunks +
// a barrel shift).  Usage: ./unaligned_loads   (prints mismatches and GB/s per offset)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ void k_check(const uint8_t* buf, uint32_t off, uint32_t* bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;  // one 16-B load per lane
    const uint8_t* p = buf + off + 16 * i;
    const v4u v = *(const __attribute__((address_space(1))) v4u*)(reinterpret_cast<uintptr_t>(p));
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (int q = 0; q < 16; ++q) {
        const uint8_t got = uint8_t(w[q / 4] >> (8 * (q % 4)));
        const uint8_t want = uint8_t((off + 16 * i + q) * 131u + 7u);
        if (got != want) atomicAdd(bad, 1u);
    }
}

__global__ void k_stream(const uint8_t* buf, uint32_t off, uint64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x) {
        const uint8_t* p = buf + off + 16 * i;
        const v4u v = *(const __attribute__((address_space(1))) v4u*)(reinterpret_cast<uintptr_t>(p));
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const uint64_t bytes = uint64_t(1) << 30;
    std::vector<uint8_t> h(bytes + 64);
    for (uint64_t i = 0; i < h.size(); ++i) h[i] = uint8_t(i * 131u + 7u);
    uint8_t* d = nullptr;
    uint32_t* bad = nullptr;
    CK(hipMalloc(&d, h.size()));
    CK(hipMalloc(&bad, 64));
    CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const uint64_t n16 = bytes / 16 - 1;
    for (uint32_t off = 0; off < 16; ++off) {
        CK(hipMemset(bad, 0, 4));
        k_check<<<4096, 256>>>(d, off, bad);
        CK(hipGetLastError());
        uint32_t nb = 0;
        CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
        float best = 1e9f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(a));
            k_stream<<<8192, 256>>>(d, off, n16, bad + 8);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        printf("offset %2u: mismatching bytes %u of %u; stream %.1f GB/s\n", off, nb, 4096u * 256u * 16u,
               double(n16 * 16) / (best * 1e-3) / 1e9);
    }
    CK(hipFree(d));
    CK(hipFree(bad));
    return 0;
}
