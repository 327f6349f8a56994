// Diagnostic: where do the blocks of a 1-workgroup-per-CU launch (1024 threads, 128 KiB LDS,
// the shape of k_tile_build / k_tile_probe) run, and when do they start?  Records each block's
// XCC id and start time (s_memrealtime, 100 MHz).  Checks the "block b and b + 8 share an XCD"
// observation the XCD-aware tile launches rely on (speed only, never correctness).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(1024) k_where(unsigned* xcc, unsigned long long* t0, unsigned long long* t1,
                                                unsigned spin) {
    extern __shared__ unsigned lds[];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned id = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID[3:0]
        xcc[blockIdx.x] = id;
        t0[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    }
    // a bounded busy phase so blocks overlap like a tile pass
    unsigned long long s = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - s < spin) __builtin_amdgcn_s_sleep(1);
    __syncthreads();
    if (threadIdx.x == 0) t1[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    if (lds[(threadIdx.x + 1) & 1023] == 0xFFFFFFFFu) xcc[0] = 99;  // keep the LDS use
}

int main() {
    const unsigned grid = 4096;
    unsigned* xcc;
    unsigned long long *t0, *t1;
    hipMalloc(&xcc, grid * 4);
    hipMalloc(&t0, grid * 8);
    hipMalloc(&t1, grid * 8);
    hipFuncSetAttribute(reinterpret_cast<const void*>(k_where), hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    for (unsigned spin : {0u, 2000u}) {  // 0 / 20 us per block
        k_where<<<grid, 1024, 131072>>>(xcc, t0, t1, spin);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
        std::vector<unsigned> x(grid);
        std::vector<unsigned long long> a(grid), b(grid);
        hipMemcpy(x.data(), xcc, grid * 4, hipMemcpyDeviceToHost);
        hipMemcpy(a.data(), t0, grid * 8, hipMemcpyDeviceToHost);
        hipMemcpy(b.data(), t1, grid * 8, hipMemcpyDeviceToHost);
        unsigned same8 = 0, rr = 0;
        unsigned long long tmin = a[0];
        for (unsigned i = 0; i < grid; ++i) tmin = a[i] < tmin ? a[i] : tmin;
        for (unsigned i = 0; i + 8 < grid; ++i) same8 += x[i] == x[i + 8];
        for (unsigned i = 0; i < grid; ++i) rr += x[i] == ((x[0] + i) & 7);
        // start skew between block b and b+8, b+16, b+24 (the 4 siblings of a super-tile)
        double skew = 0;
        unsigned cnt = 0;
        for (unsigned q = 0; q + 32 <= grid; q += 32)
            for (unsigned r = 0; r < 8; ++r) {
                unsigned long long lo = ~0ull, hi = 0;
                for (unsigned h = 0; h < 4; ++h) {
                    unsigned long long v = a[q + h * 8 + r];
                    lo = v < lo ? v : lo;
                    hi = v > hi ? v : hi;
                }
                skew += double(hi - lo) / 100.0;  // us
                ++cnt;
            }
        printf("spin %u: block i and i+8 on the same XCC: %u/%u; xcc == (xcc0 + i) %% 8: %u/%u; "
               "mean start skew of 4 siblings (b, b+8, b+16, b+24): %.2f us\n",
               spin, same8, grid - 8, rr, grid, skew / cnt);
        printf("  first 24 blocks' XCC:");
        for (unsigned i = 0; i < 24; ++i) printf(" %u", x[i]);
        printf("\n  start (us) of blocks 0,8,16,24,256,264,512: %.2f %.2f %.2f %.2f %.2f %.2f %.2f\n",
               (a[0] - tmin) / 100.0, (a[8] - tmin) / 100.0, (a[16] - tmin) / 100.0, (a[24] - tmin) / 100.0,
               (a[256] - tmin) / 100.0, (a[264] - tmin) / 100.0, (a[512] - tmin) / 100.0);
    }
    return 0;
}
