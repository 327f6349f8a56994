// HIP kernels for the bloom-filter build / probe path (reference src/bloom_filter.py), gfx950.
//
// Bitmap layout in HBM: uint32 words, bit j of the filter = bit (j & 31) of word (j >> 5).  On
// little-endian this is byte-for-byte the reference's to_bytes() bitmap (bloom_filter.py:76-81):
// byte i = (bits >> 8i) & 0xFF.
//
// This file holds the direct (one lane per key) kernels; the LDS-tiled build and probe are in
// tiled_kernels.hpp.
//   * k_build_atomic — one lane per key, k global atomicOr.
//   * k_probe        — one lane per key, k word loads (the first s1 together, the rest only for
//                      lanes still alive: bloom_filter.py:71-73's early exit), wave64 ballot →
//                      one uint64 of the LSB-first hit mask per 64 keys.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "murmur_device.hpp"

namespace pbf {

// ------------------------------------------------------------------ key sets
enum KeyMode : int {
    kFixed16 = 0,  // fixed 16-byte keys, 16-byte aligned base: one dwordx4 load per key
    kFixedN = 1,   // fixed key_len, any alignment
    kVar = 2,      // bytes + uint64 offsets[n+1] (offsets relative to off_base)
};

struct KeySet {
    const uint8_t* data;
    const uint64_t* offsets;  // kVar only: offsets of this batch's keys
    const uint64_t* off0;     // kVar only: offsets[] value that maps to data[0]
    uint32_t key_len;         // kFixed*
};

// Hash key i with seeds sbase..sbase+k-1 and call emit(s, hash_u32), s = 0..k-1.
template <int KMAX, int KM, class Emit>
__device__ __forceinline__ void hash_key(const KeySet& ks, uint64_t i, int k, Emit&& emit, int sbase = 0) {
    if constexpr (KM == kFixed16) {
        const uint4 w = gld(reinterpret_cast<const uint4*>(ks.data) + i);
        if constexpr (KMAX == 0) {
            murmur_seeds_loop(ks.data + i * 16, 16u, k, emit, sbase);
        } else {
            murmur_seeds16<KMAX>(w, k, emit, sbase);
        }
    } else {
        const uint8_t* p;
        uint32_t len;
        if constexpr (KM == kFixedN) {
            p = ks.data + i * uint64_t(ks.key_len);
            len = ks.key_len;
        } else {
            const uint64_t ob = gld(ks.off0);
            const uint64_t a = gld(ks.offsets + i) - ob;
            const uint64_t b = gld(ks.offsets + i + 1) - ob;
            p = ks.data + a;
            len = uint32_t(b - a);
        }
        if constexpr (KMAX == 0) {
            murmur_seeds_loop(p, len, k, emit, sbase);
        } else {
            murmur_seeds_seg<KMAX>(p, len, k, emit, sbase);
        }
    }
}

// ------------------------------------------------------------------ atomic build
template <int KMAX, int KM>
__global__ void __launch_bounds__(256) k_build_atomic(KeySet ks, uint64_t n, int k, IndexMap im,
                                                      uint32_t* __restrict__ bitmap) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        hash_key<KMAX, KM>(ks, i, k, [&](int, uint32_t h) {
            const uint64_t idx = py_index(h, im);
            atomicOr(bitmap + (idx >> 5), 1u << (idx & 31));
        });
    }
}

// ------------------------------------------------------------------ probe
__device__ __forceinline__ void store_hit_word(uint8_t* __restrict__ hitmask, uint64_t n, uint64_t key0,
                                               unsigned long long bits) {
    // key0 is a multiple of 64; hitmask has ceil(n/8) bytes.
    if (key0 + 64 <= n) {
        reinterpret_cast<unsigned long long*>(hitmask)[key0 >> 6] = bits;
    } else {
        const uint64_t nbytes = (n - key0 + 7) >> 3;
        for (uint64_t b = 0; b < nbytes; ++b) hitmask[(key0 >> 3) + b] = uint8_t(bits >> (8 * b));
    }
}

template <int KMAX, int KM>
__global__ void __launch_bounds__(256) k_probe(KeySet ks, uint64_t n, int k, IndexMap im,
                                               const uint32_t* __restrict__ bitmap,
                                               uint8_t* __restrict__ hitmask, int s1) {
    // Whole waves stay in the loop so the ballot sees 64 lanes; lanes past n report 0.
    // The first s1 words are loaded together; the rest only for lanes still possibly members.
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t base = uint64_t(blockIdx.x) * blockDim.x; base < n; base += stride) {
        const uint64_t i = base + threadIdx.x;
        bool hit = false;
        if (i < n) {
            if constexpr (KMAX == 0) {
                hit = true;
                hash_key<0, KM>(ks, i, k, [&](int, uint32_t h) {
                    if (hit) {
                        const uint64_t idx = py_index(h, im);
                        hit = (bitmap[idx >> 5] >> (idx & 31)) & 1u;
                    }
                });
            } else {
                uint64_t idx[KMAX];
                hash_key<KMAX, KM>(ks, i, k, [&](int s, uint32_t h) { idx[s] = py_index(h, im); });
                hit = true;
#pragma unroll
                for (int s = 0; s < KMAX; ++s)
                    if (s < k && s < s1) hit &= ((bitmap[idx[s] >> 5] >> (idx[s] & 31)) & 1u) != 0;
                if (hit) {
#pragma unroll
                    for (int s = 0; s < KMAX; ++s)
                        if (s < k && s >= s1) hit &= ((bitmap[idx[s] >> 5] >> (idx[s] & 31)) & 1u) != 0;
                }
            }
        }
        const unsigned long long bal = __ballot(hit);
        if ((threadIdx.x & 63) == 0) {
            const uint64_t key0 = base + (threadIdx.x & ~63u);
            if (key0 < n) store_hit_word(hitmask, n, key0, bal);
        }
    }
}

// ------------------------------------------------------------------ hash → index (debug/parity)
template <int KMAX, int KM>
__global__ void __launch_bounds__(256) k_hash_indices(KeySet ks, uint64_t n, int k, IndexMap im,
                                                      uint64_t* __restrict__ out) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        hash_key<KMAX, KM>(ks, i, k, [&](int s, uint32_t h) { out[i * uint64_t(k) + s] = py_index(h, im); });
    }
}

// ------------------------------------------------------------------ synthetic key generators
// (bench / test inputs; definitions in pebbledb_amd/keys.py)
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) k_gen_splitmix_hex(uint8_t* __restrict__ out, uint64_t seed, uint64_t start,
                                                          uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t z = splitmix64(seed + start + i);
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t v = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint32_t nib = uint32_t(z >> (60 - 4 * (4 * q + c))) & 0xF;
                const uint32_t ch = nib < 10 ? 48u + nib : 87u + nib;
                v |= ch << (8 * c);
            }
            w[q] = v;
        }
        reinterpret_cast<uint4*>(out)[i] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

__global__ void __launch_bounds__(256) k_gen_varlen(uint8_t* __restrict__ out, const uint64_t* __restrict__ offsets,
                                                    uint64_t seed, uint64_t start, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    const char* alpha = "0123456789abcdefghijklmnopqrstuvwxyz";
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t h = splitmix64((seed << 32) + start + i);
        const uint32_t L = 8u + uint32_t(h % 57u);
        uint8_t* dst = out + (offsets[i] - offsets[0]);
        for (uint32_t p = 0; p < L; p += 8) {
            const uint64_t w = splitmix64(h + 1 + p / 8);
            for (uint32_t c = 0; c < 8 && p + c < L; ++c) dst[p + c] = uint8_t(alpha[((w >> (8 * c)) & 0xFF) % 36]);
        }
    }
}

}  // namespace pbf
