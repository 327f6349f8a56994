// Diagnostic: per-phase cycle breakdown of k_part (workgroup 0, wave 0) via s_memtime stamps.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPBF_STAMPS -o part_phases part_phases.hip
// Shares (not absolute times) are what this build is good for: the stamps serialise.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../pebbledb_amd/csrc/tiled_kernels.hpp"
using namespace pbf;

int main(int argc, char** argv) {
    const uint32_t T = argc > 1 ? uint32_t(atoi(argv[1])) : 0;
    const uint64_t n = 10000000, nb_bytes = 1ull << 27;
    const int k = 6;
    uint8_t* keys; hipMalloc(&keys, n * 16);
    k_gen_splitmix_hex<<<4096, 256>>>(keys, 0x5EEDB100, 0, n);
    TileMap tm{};
    tm.im.m = nb_bytes * 8; tm.im.mode = kPow2; tm.im.mask = uint32_t(tm.im.m - 1);
    tm.tb = 20; tm.nbuckets = 1024; tm.total_words = nb_bytes / 4;
    for (int probe = 0; probe < 2; ++probe) {
        const uint32_t B = 1024, kpt = (probe && T > 8) ? 2 : 3, kps = kpt * 1024;
        PartGeom pg{};
        uint64_t kpw = (n + 255) / 256; kpw = (kpw + kps - 1) / kps * kps;
        pg.G = uint32_t((n + kpw - 1) / kpw); pg.kps = kps; pg.kpw = kpw; pg.nsub = uint32_t(kpw / kps);
        pg.cap = 1024; pg.nsup = B;
        uint32_t *regions, *fill, *subcnt, *ovf, *cnt, *neg, *bitmap;
        hipMalloc(&regions, size_t(pg.G) * B * pg.cap * 4); hipMalloc(&fill, size_t(pg.G) * B * 4);
        hipMalloc(&subcnt, size_t(pg.G) * pg.nsub * B * 4); hipMalloc(&ovf, n * k * 4); hipMalloc(&cnt, 64);
        hipMalloc(&neg, n / 8 + 64); hipMalloc(&bitmap, nb_bytes);
        hipMemset(cnt, 0, 64); hipMemset(neg, 0, n / 8 + 64); hipMemset(bitmap, 0, nb_bytes);
        unsigned long long* st; hipMalloc(&st, 64 * 8); hipMemset(st, 0, 64 * 8);
        hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st));
        KeySet ks{keys, nullptr, nullptr, 16};
        const size_t lds = size_t(3 * B + 17) * 4 + size_t(kps) * k * (probe ? 6 : 4);
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipEventRecord(a);
        if (probe) {
            hipFuncSetAttribute((const void*)k_part<8, 0, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            ProbeSet ps{}; ps.nf = 1; ps.bm[0] = bitmap; ps.neg = neg; ps.neg_stride = n / 32 + 1;
            k_part<8, 0, true><<<pg.G, 1024, lds>>>(ks, n, k, tm, pg, regions, fill, subcnt, ovf, cnt, ps);
        } else {
            hipFuncSetAttribute((const void*)k_part<8, 0, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            k_part<8, 0, false><<<pg.G, 1024, lds>>>(ks, n, k, tm, pg, regions, fill, subcnt, ovf, cnt, ProbeSet{});
        }
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        float ms_tile = 0, ms_gather = 0;
        if (probe) {  // the rest of the tiled probe: tile test, then gather (stamped)
            uint32_t* R; uint8_t* hm;
            hipMalloc(&R, size_t(pg.G) * B * (pg.cap / 32) * 4); hipMalloc(&hm, n / 8 + 64);
            const size_t lt = (size_t(1) << 20) / 8 + (2 * pg.G + 17) * 4;
            hipFuncSetAttribute((const void*)k_tile_probe<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lt);
            hipEvent_t c, d; hipEventCreate(&c); hipEventCreate(&d);
            hipEventRecord(c);
            k_tile_probe<false><<<B, 1024, lt>>>(tm, pg, regions, fill, bitmap, R);
            hipEventRecord(d); hipEventSynchronize(d); hipEventElapsedTime(&ms_tile, c, d);
            const size_t lg = size_t((pg.kpw + 31) / 32) * 4 + size_t(B) * (pg.nsub + 1) * 2 + 16;
            hipFuncSetAttribute((const void*)k_gather, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lg);
            hipEventRecord(c);
            k_gather<<<dim3(pg.G, 1), 512, lg>>>(tm, pg, n, regions, R, subcnt, neg, hm, nullptr);
            hipEventRecord(d); hipEventSynchronize(d); hipEventElapsedTime(&ms_gather, c, d);
            printf("k_tile_probe %.1f us, k_gather %.1f us (stamped)\n", ms_tile * 1e3, ms_gather * 1e3);
        }
        std::vector<unsigned long long> h(64);
        hipMemcpy(h.data(), st, 64 * 8, hipMemcpyDeviceToHost);
        const char* names[] = {"zero cnt + barrier", "hash + LDS count", "barrier", "scan", "placement + barrier",
                               "write-out"};
        double tot = 0;
        for (int p = 0; p < 6; ++p) tot += double(h[p + 1] - h[p]);
        printf("k_part<%s> %.1f us (stamped build), nsub=%u kps=%u G=%u\n", probe ? "probe" : "build", ms * 1e3,
               pg.nsub, pg.kps, pg.G);
        for (int p = 0; p < 6; ++p)
            printf("   %-22s %6.1f%%  %10.0f cycles/sub-chunk\n", names[p], 100.0 * double(h[p + 1] - h[p]) / tot,
                   double(h[p + 1] - h[p]) / pg.nsub);
        if (probe) {
            const char* gn[] = {"barrier", "load counts + neg", "barrier", "bucket runs", "barrier", "ballot + store"};
            double gt = 0;
            for (int p = 10; p < 16; ++p) gt += double(h[p + 1] - h[p]);
            printf("k_gather phases:\n");
            for (int p = 10; p < 16; ++p)
                printf("   %-22s %6.1f%%  %10.0f cycles/sub-chunk\n", gn[p - 10], 100.0 * double(h[p + 1] - h[p]) / gt,
                       double(h[p + 1] - h[p]) / pg.nsub);
        }
    }
    return 0;
}
