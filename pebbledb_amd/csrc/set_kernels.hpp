// Multi-filter direct probes for LsmStorage.get (reference src/lsm_storage.py:164-179, each
// `sstable.bloom_filter.may_contain(key)` = bloom_filter.py:67-74), gfx950.
//
// An LSM's SSTable filters all use k = round(-log2 p) = 10 (sstable.py:274 -> bloom_filter.py:
// 109-114) but each has its own nb_bytes (sized from its own key count), and an SSTable of
// 256 MB holds a few million keys: its filter is a few MB.  MurmurHash3 does not depend on m —
// only the floor-mod does — so a key is hashed ONCE (k seeds) and every filter of the set is
// tested from those k hashes:
//   * k_probe_set: one lane per key of a batch, the filters spread over the 8 XCDs (XcdPlan) so
//     each XCD's L2 holds only its own filters; a key is hashed once per XCD slot for all of the
//     slot's filters.  The first two words of every filter of a pass are loaded together, the
//     rest only for lanes that are still possible members of that filter (bloom_filter.py:
//     71-73's early exit); one wave64 ballot per filter writes its LSB-first hit-mask word.
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

// Filters per XCD: workgroups are dealt round-robin over the 8 XCDs in dispatch order (block i
// and block i + 8 run on the same XCD; speed only, never correctness), so the workgroups of
// slot x = blockIdx % 8 share one XCD and its 4 MiB L2.  Slot x tests the filters
// order[first[x] .. first[x] + count[x]) over its part `part[x]` of `nparts[x]` of the batch.
// With fewer than 8 filters a filter spans several slots (keys split between them); with more,
// a slot holds several (each of its keys hashed once for all of them).
struct XcdPlan {
    uint8_t first[8], count[8], part[8], nparts[8];
    uint8_t order[kMaxFilterSet];
};

// fs.hm[f]: filter f's LSB-first hit mask of the n keys.  The direct probe is bound by the rate
// of random 4-B requests; a filter whose requests all come from one XCD stays in that XCD's L2
// (C5mixed: all eight filters tested by every workgroup measured 16.8 ms, one launch per filter
// 12.7 ms, per-XCD slots below).
template <int KMAX, int KM>
__global__ void __launch_bounds__(256) k_probe_set(KeySet ks, uint64_t n, int k, FilterSet fs, XcdPlan xp) {
    const uint32_t x = blockIdx.x & 7, jb = blockIdx.x >> 3, nbx = gridDim.x >> 3;
    const uint32_t nfx = xp.count[x];
    if (nfx == 0) return;
    // the slot's key range, in whole 64-key hit-mask words
    const uint64_t words = (n + 63) >> 6;
    const uint64_t lo = min(n, (words * xp.part[x] / xp.nparts[x]) << 6);
    const uint64_t hi = min(n, (words * (xp.part[x] + 1u) / xp.nparts[x]) << 6);
    for (uint64_t base = lo + uint64_t(jb) * blockDim.x; base < hi; base += uint64_t(nbx) * blockDim.x) {
        const uint64_t i = base + threadIdx.x;
        const bool live = i < hi;
        uint32_t h[KMAX];
#pragma unroll
        for (int s = 0; s < KMAX; ++s) h[s] = 0;
        if (live) hash_key<KMAX, KM>(ks, i, k, [&](int s, uint32_t hv) { h[s] = hv; });
        const uint64_t key0 = base + (threadIdx.x & ~63u);
        for (uint32_t f0 = 0; f0 < nfx; f0 += kSetPass) {
            // stage 1: seeds 0 and 1 of every filter of the pass, all loads issued together
            uint32_t w[kSetPass][2];
#pragma unroll
            for (int q = 0; q < kSetPass; ++q) {
                if (f0 + q < nfx) {
                    const uint32_t f = xp.order[xp.first[x] + f0 + q];
                    const IndexMap& im = fs.im[f];
#pragma unroll
                    for (int s = 0; s < 2; ++s)
                        w[q][s] = (live && s < k) ? test_bit(fs.bm[f], py_index(h[s], im)) : 1u;
                }
            }
#pragma unroll
            for (int q = 0; q < kSetPass; ++q) {
                if (f0 + q >= nfx) break;
                const uint32_t f = xp.order[xp.first[x] + f0 + q];
                bool hit = live && (w[q][0] & w[q][1]);
                if (hit) {  // the rest only for lanes still possibly members of filter f
                    const IndexMap& im = fs.im[f];
#pragma unroll
                    for (int s = 2; s < KMAX; ++s)
                        if (s < k) hit &= test_bit(fs.bm[f], py_index(h[s], im)) != 0u;
                }
                const unsigned long long bal = __ballot(hit);
                if ((threadIdx.x & 63) == 0 && key0 < hi) store_hit_word(fs.hm[f], n, key0, bal);
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
    murmur_seeds_seg<KMAX>(key, len, k, [&](int s, uint32_t hv) { h[s] = hv; });
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
