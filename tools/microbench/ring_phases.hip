// Diagnostic: per-phase cycle shares of k_part_ring (workgroup 0, wave 0) via s_memtime stamps.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPBF_STAMPS -o ring_phases ring_phases.hip
// (without -DPBF_STAMPS: plain launch times; add -DPBF_DIAG_SYNTH_KEYS for keys made in registers)
// Phases: 6-0 hash (incl. the key-load wait), 0-1 barrier, 1-2 LDS atomics + head reads,
// 2-3 ring writes, 3-4 barrier, 4-5 flush, 5-6 loop / key-load issue.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../pebbledb_amd/csrc/ring_kernels.hpp"
using namespace pbf;
#ifdef PBF_STAMPS
constexpr bool kStamped = true;
#else
constexpr bool kStamped = false;
#endif

template <int KMAX, bool PROBE, bool EXACT = false, int RCT = 32, int THREADS = 1024>
void run(const char* name, uint8_t* keys, uint64_t n, int k, uint32_t* alive) {
    const uint64_t nb_bytes = 1ull << 27;
    TileMap tm{};
    tm.im.m = nb_bytes * 8; tm.im.mode = kPow2; tm.im.mask = uint32_t(tm.im.m - 1);
    tm.tb = 20; tm.nbuckets = 1024; tm.total_words = nb_bytes / 4;
    const uint32_t B = 1024;
    PartGeom pg{};
    const uint64_t groups = 256 * (1024 / THREADS);
    uint64_t kpw = (n + groups - 1) / groups; kpw = (kpw + THREADS - 1) / THREADS * THREADS;
    pg.G = uint32_t((n + kpw - 1) / kpw); pg.kps = THREADS; pg.kpw = kpw; pg.nsub = uint32_t(kpw / THREADS);
    pg.nq = (pg.nsub + 3) / 4; pg.ring = RCT; pg.cap = 4096; pg.sb = 0; pg.nsup = B;
    uint32_t *regions, *fill, *pref, *ovf, *cnt, *neg, *bitmap;
    hipMalloc(&regions, size_t(pg.G) * B * pg.cap * 4); hipMalloc(&fill, size_t(pg.G) * B * 4);
    hipMalloc(&pref, size_t(pg.G) * B * (pg.nq + 1) * 4); hipMalloc(&ovf, n * k * 4); hipMalloc(&cnt, 64);
    hipMalloc(&neg, n / 8 + 64); hipMalloc(&bitmap, nb_bytes);
    hipMemset(cnt, 0, 64); hipMemset(neg, 0, n / 8 + 64); hipMemset(bitmap, 0, nb_bytes);
    unsigned long long* st; hipMalloc(&st, 64 * 8); hipMemset(st, 0, 64 * 8);
#ifdef PBF_STAMPS
    hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st));
#endif
    KeySet ks{keys, nullptr, nullptr, 16};
    const size_t lds = size_t((2 * B + 16 * 128 + 3) & ~3u) * 4 + size_t(B) * RCT * 4;
    auto kern = k_part_ring<KMAX, 0, PROBE, true, EXACT, EXACT ? RCT : 0>;
    ProbeSet ps{};
    ps.nf = PROBE ? 1 : 0;
    ps.bm[0] = bitmap;
    ps.neg = neg;
    ps.neg_stride = n / 32 + 1;
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    kern<<<pg.G, THREADS, lds>>>(ks, n, k, tm, pg, regions, fill, pref, ovf, cnt, ps, PROBE ? 1 : 0, alive, nullptr);
    hipMemset(st, 0, 64 * 8);
    hipEventRecord(a);
    kern<<<pg.G, THREADS, lds>>>(ks, n, k, tm, pg, regions, fill, pref, ovf, cnt, ps, PROBE ? 1 : 0, alive, nullptr);
    for (int r = 0; r < 4; ++r)  // unstamped builds: 5 timed launches
        if (!kStamped) kern<<<pg.G, THREADS, lds>>>(ks, n, k, tm, pg, regions, fill, pref, ovf, cnt, ps, PROBE ? 1 : 0, alive, nullptr);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    if (!kStamped) printf("%s: %.1f us per launch (unstamped)\n", name, ms * 1e3 / 5);
    if (kStamped) {
    std::vector<unsigned long long> h(64);
    hipMemcpy(h.data(), st, 64 * 8, hipMemcpyDeviceToHost);
    // phases 0-4 within a sub-chunk; 6->0 = hash; key wait = 9->10 (per batch);
    // rest = total (7->8) minus all of these (loop, load issue, pref)
    const char* names[] = {"barrier A", "atomics+head", "ring writes", "barrier B", "flush", "hash", "key wait", "rest"};
    double d[8];
    for (int p = 0; p < 5; ++p) d[p] = double(h[p + 1] - h[p]);
    d[5] = double(h[0]) - double(h[6]);
    d[6] = double(h[10]) - double(h[9]);
    const double tot = double(h[8]) - double(h[7]);
    d[7] = tot;
    for (int p = 0; p < 7; ++p) d[7] -= d[p];
    printf("%s: %.1f us (stamped), G=%u nsub=%u, wave 0 loop %.0f cycles/sub-chunk\n", name, ms * 1e3, pg.G,
           pg.nsub, tot / pg.nsub);
    for (int p = 0; p < 8; ++p)
        printf("   %-12s %6.1f%%  %8.0f cycles/sub-chunk\n", names[p], 100.0 * d[p] / tot, d[p] / pg.nsub);
    }
    hipFree(regions); hipFree(fill); hipFree(pref); hipFree(ovf); hipFree(cnt); hipFree(neg); hipFree(bitmap); hipFree(st);
}

int main() {
    const uint64_t n = 20000000;
    uint8_t* keys; hipMalloc(&keys, n * 16);
    k_gen_splitmix_hex<<<4096, 256>>>(keys, 0x5EEDB100, 0, n);
    uint32_t* alive; hipMalloc(&alive, n / 8 + 64);
    hipMemset(alive, 0xFF, n / 16);            // first half of the keys alive
    hipMemset((uint8_t*)alive + n / 16, 0, n / 16 + 64);
    hipDeviceSynchronize();
    run<8, false>("build k=6, 10M keys", keys, n / 2, 6, nullptr);
    run<4, true>("probe round 1 (k=1), 20M keys", keys, n, 1, nullptr);
    run<8, true>("probe round 2 (k=5, half alive), 20M keys", keys, n, 5, alive);
    run<8, true>("probe k=6 single round, 20M keys", keys, n, 6, nullptr);
    run<6, false, true>("build k=6 EXACT, 10M keys", keys, n / 2, 6, nullptr);
    run<6, true, true>("probe k=6 EXACT single round, 20M keys", keys, n, 6, nullptr);
    run<6, false, true, 16, 512>("build k=6 EXACT ring 16, 512 threads (2 per CU), 10M keys", keys, n / 2, 6, nullptr);
    run<6, true, true, 16, 512>("probe k=6 EXACT ring 16, 512 threads (2 per CU), 20M keys", keys, n, 6, nullptr);
    return 0;
}
