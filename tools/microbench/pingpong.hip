// Round-trip latency of a one-key request to the GPU, two ways (verdict r4 #6: where do the
// ~12 us of a may_contain go):
//   launch  a 1-wave kernel per request that reads a word of mapped pinned memory and writes
//           the answer back there; the host polls the answer (the shape of k_probe<one key>)
//   serve   ONE resident 1-wave kernel polls the request word in mapped pinned memory (s_sleep
//           between polls) and writes the answer back; the host posts and polls.  The kernel
//           leaves on the stop word, or after 2 s of wall clock whatever happens.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o pingpong pingpong.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

struct Box {
    uint32_t req, ack, stop, served;
    uint32_t key[4];
};

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(64) k_once(Box* b, uint32_t seq) {
    const uint32_t x = ld_sys(&b->key[threadIdx.x & 3]);
    const uint32_t any = __ballot(x & 1) != 0;
    if (threadIdx.x == 0) st_sys(&b->ack, seq + any * 0);
}

template <int SLEEP>
__global__ void __launch_bounds__(64) k_serve(Box* b, uint64_t deadline_ticks) {
    const uint64_t t0 = wall_clock64();
    uint32_t done = 0, served = 0;
    while (true) {
        const uint32_t r = ld_sys(&b->req);
        if (r != done) {
            const uint32_t x = ld_sys(&b->key[threadIdx.x & 3]);
            const uint32_t any = __ballot(x & 1) != 0;
            if (threadIdx.x == 0) st_sys(&b->ack, r + any * 0);
            done = r;
            ++served;
            continue;
        }
        if (ld_sys(&b->stop) || wall_clock64() - t0 > deadline_ticks) break;
        if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    }
    if (threadIdx.x == 0) st_sys(&b->served, served);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void report(const char* what, std::vector<double>& t) {
    std::sort(t.begin(), t.end());
    double s = 0;
    for (double x : t) s += x;
    printf("%-28s mean %6.2f  p50 %6.2f  p90 %6.2f  p99 %6.2f us  (%zu)\n", what, s / t.size(), t[t.size() / 2],
           t[t.size() * 9 / 10], t[t.size() * 99 / 100], t.size());
}

int main() {
    Box* h = nullptr;
    CK(hipHostMalloc(&h, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    Box* d = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int clk_khz = 0;
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0));
    const int n = 5000;
    volatile Box* v = h;
    // launch per request
    {
        std::vector<double> t;
        for (int i = 1; i <= n + 100; ++i) {
            const double a = now_us();
            k_once<<<1, 64, 0, s>>>(d, uint32_t(i));
            while (v->ack != uint32_t(i)) {
            }
            if (i > 100) t.push_back(now_us() - a);
        }
        CK(hipStreamSynchronize(s));
        report("launch + mapped answer", t);
    }
    // resident server, several poll sleeps
    auto serve = [&](auto kern, const char* name) {
        v->req = 0;
        v->ack = 0;
        v->stop = 0;
        v->served = 0;
        const uint64_t ticks = uint64_t(clk_khz) * 2000;  // 2 s
        kern<<<1, 64, 0, s>>>(d, ticks);
        CK(hipGetLastError());
        std::vector<double> t;
        const double t_start = now_us();
        for (int i = 1; i <= n + 100; ++i) {
            const double a = now_us();
            __atomic_store_n(&h->req, uint32_t(i), __ATOMIC_RELEASE);
            bool ok = true;
            while (__atomic_load_n(&h->ack, __ATOMIC_ACQUIRE) != uint32_t(i)) {
                if (now_us() - a > 20000) {
                    ok = false;
                    break;
                }
            }
            if (!ok) {
                printf("%s: no answer to request %d after 20 ms (server started %.0f us ago)\n", name, i,
                       now_us() - t_start);
                break;
            }
            if (i > 100) t.push_back(now_us() - a);
        }
        __atomic_store_n(&h->stop, 1u, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(s));
        if (!t.empty()) report(name, t);
        printf("  served %u\n", v->served);
    };
    serve(k_serve<0>, "resident, no sleep");
    serve(k_serve<1>, "resident, s_sleep 1");
    serve(k_serve<8>, "resident, s_sleep 8");
    CK(hipHostFree(h));
    return 0;
}
