// Memory-pattern ceilings of the partition pass: read 20M 16-B keys (320 MB) and write 480 MB of
// region entries, with no compute, in the write shapes a partition can produce.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o wpat wpat.hip
//   mode 0: keys only; 1: + contiguous 1-KB-per-instruction writes; 2: + 64-B segments scattered
//   over 1024 regions of 2.7 KB per workgroup (16 segments per store instruction, the ring
//   flush's shape); 3: + 128-B segments scattered the same way (8 per instruction)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

template <int MODE, bool NT>
__global__ void __launch_bounds__(1024) k_pat(const v4* __restrict__ keys, uint64_t nkeys, v4* __restrict__ out,
                                              uint32_t cap_bytes, uint64_t wg_bytes, uint32_t* sink) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = blockIdx.x;
    const uint64_t kpw = nkeys / gridDim.x;
    const uint64_t k0 = g * kpw;
    char* rgn = reinterpret_cast<char*>(out) + g * wg_bytes;
    v4 acc = {0, 0, 0, 0};
    uint32_t wcur = 0, rnd = g * 2654435761u + tid;
    // per 1024-key sub-chunk: each wave loads 64 keys (1 KB) and stores 1.5 KB (480 MB / 320 MB)
    // keys loaded one sub-chunk ahead (as the partition's batches)
    v4 nx = NT ? __builtin_nontemporal_load(keys + k0 + tid) : keys[k0 + tid];
    for (uint64_t s0 = k0, j = 0; s0 < k0 + kpw; s0 += 1024, ++j) {
        const v4 kv = nx;
        const uint64_t s1 = s0 + 1024 < k0 + kpw ? s0 + 1024 : s0;
        nx = NT ? __builtin_nontemporal_load(keys + s1 + tid) : keys[s1 + tid];
        acc ^= kv;
        if (MODE == 0) continue;
        // 1.5 store instructions per sub-chunk: 3 per two sub-chunks
        const int nst = (j & 1) ? 2 : 1;
        for (int t = 0; t < nst; ++t) {
            char* p;
            if (MODE == 1) {
                p = rgn + ((uint64_t(wave) * 65536 * 16 + wcur) % wg_bytes) + lane * 16;
                wcur += 1024;
            } else if (MODE == 2) {
                rnd = rnd * 1664525u + 1013904223u;
                const uint32_t tile = (wave * 64 + (lane >> 2) * 4 + (rnd >> 28)) & 1023;
                const uint32_t pos = (wcur >> 4) % (cap_bytes / 64);
                p = rgn + uint64_t(tile) * cap_bytes + pos * 64 + (lane & 3) * 16;
                wcur += 64;
            } else {
                rnd = rnd * 1664525u + 1013904223u;
                const uint32_t tile = (wave * 64 + (lane >> 3) * 8 + (rnd >> 29)) & 1023;
                const uint32_t pos = (wcur >> 4) % (cap_bytes / 128);
                p = rgn + uint64_t(tile) * cap_bytes + pos * 128 + (lane & 7) * 16;
                wcur += 64;
            }
            if (NT)
                __builtin_nontemporal_store(kv, reinterpret_cast<v4*>(p));
            else
                *reinterpret_cast<v4*>(p) = kv;
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) sink[0] = tid;
}

template <int MODE, bool NT>
void run(const v4* keys, uint64_t n, v4* out, uint32_t* sink, int reps) {
    const uint32_t G = 256, cap_bytes = 672 * 4;
    const uint64_t wg_bytes = uint64_t(1024) * cap_bytes;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    k_pat<MODE, NT><<<G, 1024>>>(keys, n, out, cap_bytes, wg_bytes, sink);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) k_pat<MODE, NT><<<G, 1024>>>(keys, n, out, cap_bytes, wg_bytes, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps;
    const double bytes = n * 16.0 + (MODE ? n * 16.0 * 1.5 : 0.0);
    printf("mode %d nt %d: %.1f us  (%.2f TB/s of %.0f MB)\n", MODE, NT, us, bytes / us / 1e6, bytes / 1e6);
}

int main() {
    const uint64_t n = 20000000 / 1024 / 256 * 1024 * 256;
    v4 *keys, *out;
    uint32_t* sink;
    CK(hipMalloc(&keys, n * 16));
    CK(hipMalloc(&out, size_t(256) * 1024 * 672 * 4 + 4096));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(keys, 1, n * 16));
    for (int rep = 0; rep < 2; ++rep) {
        run<0, true>(keys, n, out, sink, 10);
        run<1, true>(keys, n, out, sink, 10);
        run<2, true>(keys, n, out, sink, 10);
        run<3, true>(keys, n, out, sink, 10);
        run<1, false>(keys, n, out, sink, 10);
        run<2, false>(keys, n, out, sink, 10);
        run<3, false>(keys, n, out, sink, 10);
    }
    return 0;
}
