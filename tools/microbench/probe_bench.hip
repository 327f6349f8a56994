// The C2 tiled probe pass alone, from the product kernels (pebbledb_amd/csrc/*.hpp) with the
// geometry pebblebloom.hip's plan_ring / set_gather / run_tiled_probe_set pick: 20M 16-byte keys
// (10M members + 10M absent) against an m = 2^30, k = 6 filter built from the members.  Per
// kernel and per pass times (hipEvents, median of reps) and a check of the hit mask against the
// direct probe (k_probe) bit for bit.  For A/B builds of the kernels with -D variants.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DVARIANT...] -o probe_bench probe_bench.hip
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../pebbledb_amd/csrc/ring_kernels.hpp"
using namespace pbf;

// the gather ANDs straight into the hit mask (n % 32 == 0, aligned: run_tiled_probe_set's hw_is_mask)
#ifndef HW_IS_MASK
#define HW_IS_MASK 1
#endif

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const uint64_t nb = 10000000, n = 20000000, nb_bytes = 1ull << 27;
    const uint32_t k = 6, B = 1024, kps = 1024, tb = 20;
    uint8_t* keys;
    CK(hipMalloc(&keys, n * 16));
    k_gen_splitmix_hex<<<4096, 256>>>(keys, 0x5EEDB100, 0, n);
    TileMap tm{};
    tm.im.m = nb_bytes * 8;
    tm.im.mode = kPow2;
    tm.im.mask = uint32_t(tm.im.m - 1);
    tm.tb = tb;
    tm.nbuckets = B;
    tm.total_words = nb_bytes / 4;
    uint32_t* bitmap;
    CK(hipMalloc(&bitmap, nb_bytes));
    CK(hipMemset(bitmap, 0, nb_bytes));
    KeySet ks{keys, nullptr, nullptr, 16};
    k_build_atomic<6, kFixed16><<<4096, 256>>>(ks, nb, int(k), tm.im, bitmap);
    // plan_ring
    PartGeom pg{};
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
    const uint64_t capx = uint64_t(mu + 8.0 * std::sqrt(mu) + 32.0);
    pg.cap = uint32_t(((capx + 31) / 32) * 32);
    pg.spill_cap = uint32_t(std::min<size_t>(4096, (size_t(kRingLdsWords) * 4 - size_t(ring_lds_words(B)) * 4) / 8));
    const uint32_t G = pg.G, cap = pg.cap;
    // set_gather (nf = 1, 512-thread workgroups, up to 4 per CU)
    const size_t kb = size_t((kpw + 31) / 32) * 4;
    const uint32_t row = pg.nq + 1;
    uint32_t S = 8;
    auto glds = [&](uint32_t sp) { return kb + size_t((B + sp - 1) / sp) * row * 2 + 16; };
    auto per_cu = [](size_t bytes) { return std::min<size_t>(4, (160 * 1024) / bytes); };
    while (glds(S) > 156 * 1024 && S < 64 && S < B) S *= 2;
    while (S < 32 && S < B && per_cu(glds(2 * S)) > per_cu(glds(S))) S *= 2;
    size_t lds_gather = glds(S);
    uint32_t gtq = 0;
    if (row <= 255) {
        const uint32_t tq = cap / 4;
        const size_t with = ((lds_gather + 3) & ~size_t(3)) + size_t((B + S - 1) / S) * tq + 4;
        if (with <= 38 * 1024) {
            gtq = tq;
            lds_gather = with;
        }
    }
    // run_tiled_probe_set
    size_t lds_tile = ((size_t(1) << tb) / 32 + 2 * G + 1 + 16) * 4;
    const size_t table_words = size_t(G) * (cap / 32);
    const int tab = lds_tile + table_words * 5 <= 160 * 1024 ? 2 : (lds_tile + table_words * 2 <= 160 * 1024 ? 1 : 0);
    lds_tile += tab == 2 ? table_words * 5 : (tab == 1 ? table_words * 2 : 0);
    const size_t r_words = size_t(G) * B * (cap / 32);
    const uint64_t neg_words = (n + 31) / 32;
    uint32_t *regions, *fill, *R, *neg, *hw;
    uint16_t* pref;
    uint8_t *hm, *hm_ref;
    CK(hipMalloc(&regions, size_t(G) * B * cap * 4 + size_t(G) * 64));
    CK(hipMalloc(&fill, size_t(G) * B * 4));
    CK(hipMalloc(&pref, size_t(G) * B * row * 2));
    CK(hipMalloc(&R, r_words * 4));
    CK(hipMalloc(&neg, neg_words * 4));
    CK(hipMalloc(&hw, neg_words * 4));
    CK(hipMalloc(&hm, (n + 7) / 8));
    CK(hipMalloc(&hm_ref, (n + 7) / 8));
    ProbeSet ps{};
    ps.nf = 1;
    ps.bm[0] = bitmap;
    ps.neg = neg;
    ps.neg_stride = neg_words;
    auto part = k_part_ring<6, kFixed16, true, true, true>;
    auto tprobe = tab == 2 ? k_tile_probe<2> : (tab == 1 ? k_tile_probe<1> : k_tile_probe<0>);
    CK(hipFuncSetAttribute((const void*)tprobe, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_tile)));
    CK(hipFuncSetAttribute((const void*)k_gather_ring<1>, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_gather)));
    HitMasks hms{};
    hms.hm[0] = hm;
    const dim3 ggrid(G, S), hgrid(std::max<uint32_t>(1, uint32_t(std::min<uint64_t>(4096, (neg_words + 255) / 256))), 1);
    hipEvent_t ev[5];
    for (auto& e : ev) CK(hipEventCreate(&e));
    std::vector<float> t[4];
    for (int r = 0; r < reps + 3; ++r) {
        CK(hipEventRecord(ev[0]));
        part<<<G, kPartThreads, 0>>>(ks, n, int(k), tm, pg, regions, fill, pref, nullptr, nullptr, ps, HW_IS_MASK ? reinterpret_cast<uint32_t*>(hm) : hw);
        CK(hipEventRecord(ev[1]));
        tprobe<<<B, 1024, lds_tile>>>(tm, pg, regions, fill, bitmap, R);
        CK(hipEventRecord(ev[2]));
        k_gather_ring<1><<<ggrid, 512, lds_gather>>>(tm, pg, n, regions, R, fill, pref, neg, hm,
                                                      HW_IS_MASK ? reinterpret_cast<uint32_t*>(hm) : hw, 1, r_words, neg_words, gtq);
        CK(hipEventRecord(ev[3]));
        if (!HW_IS_MASK) k_hw_to_hitmask<<<hgrid, 256>>>(hw, neg_words, n, hms);
        CK(hipEventRecord(ev[4]));
        CK(hipEventSynchronize(ev[4]));
        if (r >= 3)
            for (int x = 0; x < 4; ++x) {
                float ms;
                CK(hipEventElapsedTime(&ms, ev[x], ev[x + 1]));
                t[x].push_back(ms * 1e3f);
            }
    }
    CK(hipGetLastError());
    k_probe<6, kFixed16><<<4096, 256>>>(ks, n, int(k), tm.im, bitmap, hm_ref, 6);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> a((n + 7) / 8), b((n + 7) / 8);
    CK(hipMemcpy(a.data(), hm, a.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), hm_ref, b.size(), hipMemcpyDeviceToHost));
    uint64_t members = 0, fps = 0, diff = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const int x = (a[i >> 3] >> (i & 7)) & 1, y = (b[i >> 3] >> (i & 7)) & 1;
        diff += x != y;
        if (i < nb) members += x;
        else fps += x;
    }
    auto med = [](std::vector<float> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    const float tp = med(t[0]), tt = med(t[1]), tg = med(t[2]), th = med(t[3]);
    const double bytes = double(n) * 16 + double(n) * k * 4 + double(n) / 8;
    printf("probe pass: part %.1f  tile %.1f  gather %.1f  hw %.1f  = %.1f us (%.1f%% of 8 TB/s)  G=%u cap=%u S=%u tab=%d gtq=%u\n",
           tp, tt, tg, th, tp + tt + tg + th, 100.0 * bytes / ((tp + tt + tg + th) * 1e-6) / 8e12, G, cap, S, tab, gtq);
    printf("check: members hit %lu/%lu, absent hits %lu, bits differing from the direct probe %lu\n",
           (unsigned long)members, (unsigned long)nb, (unsigned long)fps, (unsigned long)diff);
    return diff != 0 || members != nb;
}
