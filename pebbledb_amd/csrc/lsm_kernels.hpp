// Key-range pre-check of the batched LsmStorage.get (reference src/lsm_storage.py:171-175):
// for every key of a batch and every L>=1 SSTable t, `first_t <= key <= last_t` — Python str
// comparison, which for the UTF-8 bytes the keys are hashed from (bloom_filter.py:43) is plain
// bytewise lexicographic order (UTF-8 preserves code-point order; a proper prefix sorts
// first).  gfx950.
//
// Layout: the 2*T bounds (first_0, last_0, first_1, last_1, ...) are staged once per workgroup
// in LDS, each at a 4-byte-aligned offset and zero-padded to whole words.  One lane per key:
// the key is compared 4 bytes at a time as big-endian words (bswap of the little-endian load),
// the word that holds the end of the shorter string masked to its common bytes.  A wave's 64
// results per table leave as one u64 (wave ballot) of the LSB-first mask [T][ceil(n/8)] — the
// hit-mask layout, so a range mask ANDs directly with that table's filter hit mask.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bloom_kernels.hpp"

namespace pbf {

constexpr uint32_t kRangeLdsBytes = 96 * 1024;  // bound bytes staged per launch (host splits tables)

struct RangeSet {
    const uint8_t* bytes;     // bound bytes (device), concatenated
    const uint64_t* offsets;  // 2*T+1 offsets into bytes (device), relative to offsets[0]
    uint32_t t0, nt;          // tables [t0, t0 + nt) of this launch
    uint32_t lds_words;       // padded words of this launch's bounds
};

// Compare n bytes of key (global, any alignment) with an LDS bound of bl bytes at word w;
// returns <0, 0, >0 as memcmp-then-length.
__device__ __forceinline__ int cmp_key_bound(const uint8_t* key, uint32_t kl, const uint32_t* lb, uint32_t bl) {
    const uint32_t m = min(kl, bl);
    for (uint32_t off = 0; off < m; off += 4) {
        uint32_t a, b = lb[off >> 2];
        if (m - off >= 4) {
            a = load_u32_any(key + off);
        } else {  // the last common bytes: touch only dwords holding them
            a = load_tail(key + off, m - off);
            b &= (1u << (8 * (m - off))) - 1u;
        }
        if (a != b) return __builtin_bswap32(a) < __builtin_bswap32(b) ? -1 : 1;
    }
    return kl < bl ? -1 : (kl > bl ? 1 : 0);
}

template <int KM>
__global__ void __launch_bounds__(256) k_range_mask(KeySet ks, uint64_t n, RangeSet rs, uint8_t* __restrict__ out,
                                                    uint64_t stride) {
    extern __shared__ uint32_t lds[];
    uint32_t* woff = lds;                  // 2*nt+1 word offsets of the bounds
    uint32_t* blen = woff + 2 * rs.nt + 1;  // 2*nt byte lengths
    uint32_t* words = blen + 2 * rs.nt;     // padded bound words
    const uint64_t ob = rs.offsets[0];
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    if (tid == 0) {
        uint32_t w = 0;
        for (uint32_t j = 0; j < 2 * rs.nt; ++j) {
            const uint32_t bl = uint32_t(rs.offsets[2 * rs.t0 + j + 1] - rs.offsets[2 * rs.t0 + j]);
            woff[j] = w;
            blen[j] = bl;
            w += (bl + 3) / 4;
        }
        woff[2 * rs.nt] = w;
    }
    __syncthreads();
    // stage the bounds' bytes (zero padded per bound)
    for (uint32_t j = 0; j < 2 * rs.nt; ++j) {
        const uint8_t* src = rs.bytes + (rs.offsets[2 * rs.t0 + j] - ob);
        const uint32_t bl = blen[j], w0 = woff[j];
        for (uint32_t q = tid; q < (bl + 3) / 4; q += nt) {
            uint32_t v = 0;
            for (uint32_t c = 0; c < 4 && 4 * q + c < bl; ++c) v |= uint32_t(src[4 * q + c]) << (8 * c);
            words[w0 + q] = v;
        }
    }
    __syncthreads();
    const uint64_t gstride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t base = uint64_t(blockIdx.x) * blockDim.x; base < n; base += gstride) {
        const uint64_t i = base + tid;
        const uint8_t* kp = nullptr;
        uint32_t kl = 0;
        if (i < n) {
            if constexpr (KM == kVar) {
                const uint64_t o0 = *ks.off0;
                kp = ks.data + (ks.offsets[i] - o0);
                kl = uint32_t(ks.offsets[i + 1] - ks.offsets[i]);
            } else {
                kp = ks.data + i * uint64_t(ks.key_len);
                kl = ks.key_len;
            }
        }
        const uint64_t key0 = base + (tid & ~63u);
        for (uint32_t t = 0; t < rs.nt; ++t) {
            bool in = false;
            if (i < n)
                in = cmp_key_bound(kp, kl, words + woff[2 * t], blen[2 * t]) >= 0 &&
                     cmp_key_bound(kp, kl, words + woff[2 * t + 1], blen[2 * t + 1]) <= 0;
            const unsigned long long bal = __ballot(in);
            if ((tid & 63) == 0 && key0 < n) store_hit_word(out + uint64_t(rs.t0 + t) * stride, n, key0, bal);
        }
    }
}

}  // namespace pbf
