// Multi-filter direct probes for LsmStorage.get (reference src/lsm_storage.py:164-179, each
// `sstable.bloom_filter.may_contain(key)` = bloom_filter.py:67-74), gfx950.
//
// An LSM's SSTable filters all use k = round(-log2 p) = 10 (sstable.py:274 -> bloom_filter.py:
// 109-114) but each has its own nb_bytes (sized from its own key count), and an SSTable of
// 256 MB holds a few million keys: its filter is a few MB.  MurmurHash3 does not depend on m —
// only the floor-mod does — so a key is hashed ONCE (k seeds) and every filter of the set is
// tested from those k hashes:
//   * k_probe_set: one lane per key of a batch; the first two words of every filter of a pass
//     are loaded together (2 x nf loads in flight per lane), the rest only for lanes that are
//     still possible members of that filter (bloom_filter.py:71-73's early exit); one wave64
//     ballot per filter writes that filter's LSB-first hit-mask word.
//   * k_may_contain_set: ONE key against up to 64 filters per launch (the per-key form of
//     LsmStorage.get): every lane hashes the key (a wave's worth of redundant ALU instead of a
//     hash broadcast), lane f tests filter f, one ballot is the answer; key in and answer out
//     through mapped pinned memory.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bloom_kernels.hpp"

namespace pbf {

constexpr int kMaxFilterSet = 64;  // filters per launch (kernel-argument table)
constexpr int kSetPass = 8;        // filters whose first words are in flight together (k_probe_set)

struct FilterSet {
    const uint32_t* bm[kMaxFilterSet];
    IndexMap im[kMaxFilterSet];
    uint8_t* hm[kMaxFilterSet];  // k_probe_set: filter f's hit mask (device memory)
    uint32_t nf;
    uint32_t pad;
};

__device__ __forceinline__ uint32_t test_bit(const uint32_t* __restrict__ bm, uint64_t idx) {
    return (bm[idx >> 5] >> (idx & 31)) & 1u;
}

// fs.hm[f]: filter f's LSB-first hit mask of the n keys.
template <int KMAX, int KM>
__global__ void __launch_bounds__(256) k_probe_set(KeySet ks, uint64_t n, int k, FilterSet fs) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    const uint32_t nf = fs.nf;
    for (uint64_t base = uint64_t(blockIdx.x) * blockDim.x; base < n; base += stride) {
        const uint64_t i = base + threadIdx.x;
        const bool live = i < n;
        uint32_t h[KMAX];
#pragma unroll
        for (int s = 0; s < KMAX; ++s) h[s] = 0;
        if (live) hash_key<KMAX, KM>(ks, i, k, [&](int s, uint32_t hv) { h[s] = hv; });
        const uint64_t key0 = base + (threadIdx.x & ~63u);
        for (uint32_t f0 = 0; f0 < nf; f0 += kSetPass) {
            // stage 1: seeds 0 and 1 of every filter of the pass, all loads issued together
            uint32_t w[kSetPass][2];
#pragma unroll
            for (int q = 0; q < kSetPass; ++q) {
                const uint32_t f = f0 + q;
                if (f < nf) {
                    const IndexMap& im = fs.im[f];
#pragma unroll
                    for (int s = 0; s < 2; ++s)
                        w[q][s] = (live && s < k) ? test_bit(fs.bm[f], py_index(h[s], im)) : 1u;
                }
            }
#pragma unroll
            for (int q = 0; q < kSetPass; ++q) {
                const uint32_t f = f0 + q;
                if (f >= nf) break;
                bool hit = live && (w[q][0] & w[q][1]);
                if (hit) {  // the rest only for lanes still possibly members of filter f
                    const IndexMap& im = fs.im[f];
#pragma unroll
                    for (int s = 2; s < KMAX; ++s)
                        if (s < k) hit &= test_bit(fs.bm[f], py_index(h[s], im)) != 0u;
                }
                const unsigned long long bal = __ballot(hit);
                if ((threadIdx.x & 63) == 0 && key0 < n) store_hit_word(fs.hm[f], n, key0, bal);
            }
        }
    }
}

// One key (len bytes at key) against the nf filters of fs: bit f of the answer = filter f's
// may_contain.  out[0..7]: the answer (u64, filters 0..63); out[8] is set to 1 after it (the
// host polls that byte in mapped memory).
template <int KMAX>
__global__ void __launch_bounds__(64) k_may_contain_set(const uint8_t* __restrict__ key, uint32_t len, int k,
                                                        FilterSet fs, uint8_t* out) {
    const uint32_t f = threadIdx.x;
    uint32_t h[KMAX];
#pragma unroll
    for (int s = 0; s < KMAX; ++s) h[s] = 0;
    murmur_seeds_chunked<KMAX>(key, len, k, [&](int s, uint32_t hv) { h[s] = hv; });
    bool hit = false;
    if (f < fs.nf) {
        const uint32_t* bm = fs.bm[f];
        const IndexMap im = fs.im[f];
        uint32_t acc = 1u;
#pragma unroll
        for (int s = 0; s < KMAX; ++s)
            if (s < k) acc &= test_bit(bm, py_index(h[s], im));  // the AND of bloom_filter.py:71-74
        hit = acc != 0u;
    }
    const unsigned long long bal = __ballot(hit);
    if (f == 0) {
        *reinterpret_cast<volatile unsigned long long*>(out) = bal;
        __threadfence_system();  // the answer is visible to the host before the flag
        *reinterpret_cast<volatile uint8_t*>(out + 8) = 1;
    }
}

}  // namespace pbf
