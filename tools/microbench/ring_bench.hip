// Launch times of the C2-shaped ring partition (k_part_ring, the product kernel from
// pebbledb_amd/csrc/ring_kernels.hpp) alone: probe of 20M and build of 10M 16-byte keys, m = 2^30,
// k = 6, geometry as plan_ring picks it.  For A/B builds of the kernel with -D variants.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DVARIANT...] -o ring_bench ring_bench.hip
// Prints per-launch microseconds (hipEvents over 10 launches) and a checksum of the fill counts.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#ifdef OLD_RING  // the round-4 kernel (sources from git, copied under build/r4src)
#include "../../build/r4src/ring_kernels.hpp"
#else
#include "../../pebbledb_amd/csrc/ring_kernels.hpp"
#endif
using namespace pbf;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

template <bool PROBE>
void run(uint8_t* keys, uint64_t n, int reps) {
    const uint64_t nb_bytes = 1ull << 27;
    const uint32_t k = 6, B = 1024, kps = 1024;
    TileMap tm{};
    tm.im.m = nb_bytes * 8;
    tm.im.mode = kPow2;
    tm.im.mask = uint32_t(tm.im.m - 1);
    tm.tb = 20;
    tm.nbuckets = B;
    tm.total_words = nb_bytes / 4;
    PartGeom pg{};  // as plan_ring (pebblebloom.hip)
    const uint64_t G0 = std::min<uint64_t>(256, (n + kps - 1) / kps);
    uint64_t kpw = (n + G0 - 1) / G0;
    kpw = ((kpw + kps - 1) / kps) * kps;
    pg.G = uint32_t((n + kpw - 1) / kpw);
    pg.kps = kps;
    pg.kpw = kpw;
    pg.nsub = uint32_t(kpw / kps);
    pg.nq = uint32_t((kpw + kGroupKeys - 1) / kGroupKeys);
    pg.ring = kRingEntries;
    const double mu = double(kpw) * k / B;
    const uint64_t cap = uint64_t(mu + 8.0 * std::sqrt(mu) + 32.0);
    pg.cap = uint32_t(((cap + 31) / 32) * 32);
    const size_t ring_bytes = size_t(ring_lds_words(B)) * 4, spill_entry = PROBE ? 8 : 4;
#ifdef OLD_RING
    pg.spill_cap = uint32_t(std::min<size_t>(4096, (160 * 1024 - ring_bytes) / spill_entry));
    const size_t lds = ring_bytes + size_t(pg.spill_cap) * spill_entry;
#else
    pg.spill_cap = uint32_t(std::min<size_t>(4096, (size_t(kRingLdsWords) * 4 - ring_bytes) / spill_entry));
    const size_t lds = 0;
#endif
    uint32_t *regions, *fill, *ovf, *cnt, *neg, *bitmap;
    uint16_t* pref;
    CK(hipMalloc(&regions, size_t(pg.G) * B * pg.cap * 4 + size_t(pg.G) * 64));
    CK(hipMalloc(&fill, size_t(pg.G) * B * 4));
    CK(hipMalloc(&pref, size_t(pg.G) * B * (pg.nq + 1) * 2));
    CK(hipMalloc(&ovf, n * k * 4));
    CK(hipMalloc(&cnt, 64));
    CK(hipMalloc(&neg, n / 8 + 64));
    CK(hipMalloc(&bitmap, nb_bytes));
    CK(hipMemset(cnt, 0, 64));
    CK(hipMemset(bitmap, 0xFF, nb_bytes));
    KeySet ks{keys, nullptr, nullptr, 16};
    ProbeSet ps{};
    ps.nf = PROBE ? 1 : 0;
    ps.bm[0] = bitmap;
    ps.neg = neg;
    ps.neg_stride = n / 32 + 1;
    auto kern = k_part_ring<6, kFixed16, PROBE, true, true>;
    if (lds) CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    kern<<<pg.G, kPartThreads, lds>>>(ks, n, int(k), tm, pg, regions, fill, PROBE ? pref : nullptr, ovf, cnt, ps, nullptr);
    CK(hipGetLastError());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        kern<<<pg.G, kPartThreads, lds>>>(ks, n, int(k), tm, pg, regions, fill, PROBE ? pref : nullptr, ovf, cnt, ps, nullptr);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint32_t> hf(size_t(pg.G) * B);
    CK(hipMemcpy(hf.data(), fill, hf.size() * 4, hipMemcpyDeviceToHost));
    uint64_t sum = 0, x = 0;
    for (size_t i = 0; i < hf.size(); ++i) {
        sum += hf[i];
        x = x * 1000003 + hf[i];
    }
    uint32_t ovfc = 0;
    CK(hipMemcpy(&ovfc, cnt, 4, hipMemcpyDeviceToHost));
    printf("%s n=%lu G=%u cap=%u: %.2f us per launch; fill sum %lu (of %lu positions), fill hash %016lx, overflow %u\n",
           PROBE ? "probe" : "build", (unsigned long)n, pg.G, pg.cap, ms * 1e3 / reps, (unsigned long)sum,
           (unsigned long)(n * k), (unsigned long)x, ovfc);
    CK(hipFree(regions));
    CK(hipFree(fill));
    CK(hipFree(pref));
    CK(hipFree(ovf));
    CK(hipFree(cnt));
    CK(hipFree(neg));
    CK(hipFree(bitmap));
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const uint64_t n = 20000000;
    uint8_t* keys;
    CK(hipMalloc(&keys, n * 16));
    k_gen_splitmix_hex<<<4096, 256>>>(keys, 0x5EEDB100, 0, n);
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 2; ++rep) {
        run<true>(keys, n, reps);
        run<false>(keys, n / 2, reps);
    }
    CK(hipFree(keys));
    return 0;
}
