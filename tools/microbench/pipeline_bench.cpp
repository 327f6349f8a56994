// Native driver of the C-ABI (no Python, no torch): the bench.py step (clear + build 10M keys +
// probe 20M keys, device-resident) timed by wall clock and by hipEvents on the filter's stream.
// Build: hipcc -O3 -std=c++17 -o pipeline_bench pipeline_bench.cpp -L../../pebbledb_amd -lpebblebloom
//        -Wl,-rpath,'$ORIGIN/../../pebbledb_amd'
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../include/pebblebloom.h"

#define CK(x) do { int rc_ = (x); if (rc_) { printf("%s -> %d %s\n", #x, rc_, pbf_last_error()); return 1; } } while (0)

int main(int argc, char** argv) {
    const uint64_t n = 10000000, nb = 1ull << 27;
    const int k = 6, steps = argc > 1 ? atoi(argv[1]) : 20, mode = argc > 2 ? atoi(argv[2]) : 0;
    uint8_t *keys, *hm;
    if (hipMalloc(&keys, 2 * n * 16) || hipMalloc(&hm, 2 * n / 8)) return 1;
    CK(pbf_gen_splitmix_hex(0, nullptr, keys, 0x5EEDB100, 0, 2 * n));
    if (hipDeviceSynchronize()) return 1;
    pbf_filter_t* f;
    CK(pbf_create(0, nb, k, &f));
    CK(pbf_set_build_mode(f, PBF_BUILD_TILED));
    CK(pbf_set_probe_mode(f, PBF_PROBE_TILED));
    hipStream_t s = (hipStream_t)pbf_stream(f);
    auto step = [&]() -> int {
        CK(pbf_clear(f));
        CK(pbf_add_fixed(f, keys, 16, n, 1));
        CK(pbf_probe_fixed(f, keys, 16, 2 * n, hm, 1));
        return 0;
    };
    for (int i = 0; i < 5; ++i) if (step()) return 1;
    CK(pbf_sync(f));
    std::vector<hipEvent_t> ev(steps + 1);
    for (auto& e : ev) hipEventCreate(&e);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < steps; ++i) {
        if (mode == 1) hipEventRecord(ev[i], s);
        if (step()) return 1;
        if (mode == 2) CK(pbf_sync(f));
    }
    if (mode == 1) hipEventRecord(ev[steps], s);
    auto t_enq = std::chrono::steady_clock::now();
    CK(pbf_sync(f));
    auto t1 = std::chrono::steady_clock::now();
    const double wall = std::chrono::duration<double, std::milli>(t1 - t0).count() / steps;
    const double enq = std::chrono::duration<double, std::milli>(t_enq - t0).count() / steps;
    double evms = 0;
    if (mode == 1) { float ms; hipEventElapsedTime(&ms, ev[0], ev[steps]); evms = ms / steps; }
    printf("mode=%d steps=%d wall %.4f ms/step (enqueue %.4f)  events %.4f ms/step  -> %.1f Mkeys/s\n", mode, steps,
           wall, enq, evms, 3.0 * n / wall / 1e3);
    pbf_destroy(f);
    return 0;
}
