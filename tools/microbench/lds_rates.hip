// Microbenchmark: LDS atomic / read rates and random global 4-B reads on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_rates lds_rates.hip ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t xs(uint32_t x) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; }

// mode 0: ds_add_u32 (no return) random in [0, words)
// mode 1: ds_add_rtn_u32 random
// mode 2: ds_or_b32 random bit in [0, words)
// mode 3: ds_read_b32 random (sum)
// mode 4: ds_add_u32 lane-contiguous (no conflicts): address = (lane + it*64) % words
// mode 5: ds_write_b32 random (non-atomic)
template <int MODE>
__global__ void __launch_bounds__(1024) k_lds(uint32_t words, int iters, uint32_t* out) {
    extern __shared__ uint32_t s[];
    for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) s[w] = 0;
    __syncthreads();
    uint32_t x = (blockIdx.x * 1024 + threadIdx.x) * 2654435761u + 1;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            x = xs(x);
            const uint32_t a = (MODE == 4) ? ((threadIdx.x + (it * 8 + u) * 64) & (words - 1)) : (x & (words - 1));
            if (MODE == 0 || MODE == 4) atomicAdd(s + a, 1u);
            if (MODE == 1) acc += atomicAdd(s + a, 1u);
            if (MODE == 2) atomicOr(s + a, 1u << (x >> 27));
            if (MODE == 3) acc += s[a];
            if (MODE == 5) s[a] = x;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = s[acc & (words - 1)] + acc;
}

__global__ void __launch_bounds__(256) k_gather(const uint32_t* __restrict__ t, uint64_t mask, int iters, uint32_t* out) {
    uint32_t x = (blockIdx.x * 256 + threadIdx.x) * 2654435761u + 7;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) { x = xs(x); v[u] = t[(uint64_t(x) * 2654435761ull) & mask]; }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u];
    }
    if (acc == 0x12345678) out[0] = acc;
}

template <int MODE>
float run_lds(uint32_t words, int iters, uint32_t* out, int grid) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    size_t lds = words * 4;
    hipFuncSetAttribute((const void*)k_lds<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    k_lds<MODE><<<grid, 1024, lds>>>(words, iters, out);
    hipEventRecord(a);
    k_lds<MODE><<<grid, 1024, lds>>>(words, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    uint32_t* out; CK(hipMalloc(&out, 1 << 20));
    const int grid = 256 * 2, iters = 256;
    const double ops = double(grid) * 1024 * iters * 8;
    const char* names[] = {"ds_add (no rtn) random", "ds_add_rtn random", "ds_or random", "ds_read random",
                           "ds_add contiguous", "ds_write random"};
    for (uint32_t words : {1024u, 4096u, 32768u}) {
        float t[6] = {run_lds<0>(words, iters, out, grid), run_lds<1>(words, iters, out, grid),
                      run_lds<2>(words, iters, out, grid), run_lds<3>(words, iters, out, grid),
                      run_lds<4>(words, iters, out, grid), run_lds<5>(words, iters, out, grid)};
        for (int m = 0; m < 6; ++m)
            printf("LDS words=%6u %-26s %8.3f ms  %7.2f Gop/s  %6.2f ops/clk/CU(@2.4GHz)\n", words, names[m], t[m],
                   ops / t[m] / 1e6, ops / (t[m] * 1e-3) / 256 / 2.4e9);
    }
    // random global gathers
    for (uint64_t bytes : {uint64_t(4) << 20, uint64_t(32) << 20, uint64_t(128) << 20, uint64_t(1) << 30}) {
        uint32_t* tab; CK(hipMalloc(&tab, bytes)); CK(hipMemset(tab, 1, bytes));
        const int g = 256 * 32, it = 64;
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        k_gather<<<g, 256>>>(tab, bytes / 4 - 1, it, out);
        hipEventRecord(a);
        k_gather<<<g, 256>>>(tab, bytes / 4 - 1, it, out);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        const double n = double(g) * 256 * it * 4;
        printf("global random 4B gather, table %6llu MiB: %8.3f ms  %7.2f G loads/s\n",
               (unsigned long long)(bytes >> 20), ms, n / ms / 1e6);
        hipFree(tab);
    }
    return 0;
}
