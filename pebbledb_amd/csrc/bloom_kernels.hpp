// HIP kernels for the bloom-filter build / probe path (reference src/bloom_filter.py), gfx950.
//
// Bitmap layout in HBM: uint32 words, bit j of the filter = bit (j & 31) of word (j >> 5).  On
// little-endian this is byte-for-byte the reference's to_bytes() bitmap (bloom_filter.py:76-81):
// byte i = (bits >> 8i) & 0xFF.
//
// Build, two implementations (identical results: OR is commutative and idempotent):
//   * atomic  — one lane per key, k global atomicOr (k_build_atomic).
//   * tiled   — the bitmap is cut into tiles of 2^TB bits that fit one CU's LDS.  The k hash
//               positions of every key are partitioned by tile (k_hist → k_colscan →
//               k_basescan → k_scatter), then one workgroup per tile ORs its positions into
//               an LDS copy of the tile and writes the tile once (k_tile).  HBM sees each
//               position as one coalesced 4-B write + one 4-B read instead of a random 4-B
//               read-modify-write to a 64-B line.
// Probe: one lane per key, k word loads (the first two together, the rest only for lanes still
// alive: bloom_filter.py:71-73's early exit), wave64 ballot → one uint64 of the LSB-first hit
// mask per 64 keys.
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

// Hash key i with seeds 0..k-1 and call emit(seed, hash_u32).
template <int KMAX, int KM, class Emit>
__device__ __forceinline__ void hash_key(const KeySet& ks, uint64_t i, int k, Emit&& emit) {
    if constexpr (KM == kFixed16) {
        const uint4 w = reinterpret_cast<const uint4*>(ks.data)[i];
        if constexpr (KMAX == 0) {
            murmur_seeds_loop(ks.data + i * 16, 16u, k, emit);
        } else {
            murmur_seeds16<KMAX>(w, k, emit);
        }
    } else {
        const uint8_t* p;
        uint32_t len;
        if constexpr (KM == kFixedN) {
            p = ks.data + i * uint64_t(ks.key_len);
            len = ks.key_len;
        } else {
            const uint64_t ob = *ks.off0;
            const uint64_t a = ks.offsets[i] - ob;
            const uint64_t b = ks.offsets[i + 1] - ob;
            p = ks.data + a;
            len = uint32_t(b - a);
        }
        if constexpr (KMAX == 0) {
            murmur_seeds_loop(p, len, k, emit);
        } else {
            murmur_seeds<KMAX>(p, len, k, emit);
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
                                               uint8_t* __restrict__ hitmask) {
    // Whole waves stay in the loop so the ballot sees 64 lanes; lanes past n report 0.
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
                // stage 1: first two bits together; stage 2: the rest, only if still possible.
                hit = true;
#pragma unroll
                for (int s = 0; s < 2 && s < KMAX; ++s)
                    if (s < k) hit &= ((bitmap[idx[s] >> 5] >> (idx[s] & 31)) & 1u) != 0;
                if (hit) {
#pragma unroll
                    for (int s = 2; s < KMAX; ++s)
                        if (s < k) hit &= ((bitmap[idx[s] >> 5] >> (idx[s] & 31)) & 1u) != 0;
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

// ------------------------------------------------------------------ tiled build
// Position space: for m <= 2^32 a position is the bit index itself (u32).  For m > 2^32 only
// [0, 2^31) U [m - 2^31, m) is reachable (|h| <= 2^31); the position is u32(h) and a position
// p >= 2^31 lives at bit p + (m - 2^32).  Tiles are 2^TB positions; tile t → bitmap word
// tile_word0(t).
struct TileMap {
    IndexMap im;
    uint32_t tb;          // log2 positions per tile (<= 20: 128 KiB of LDS)
    uint32_t nbuckets;    // number of tiles
    uint32_t cspace;      // 1 when m > 2^32
    uint32_t pad;
    uint64_t delta_words; // (m - 2^32) / 32 when cspace
    uint64_t total_words; // ceil(nb_bytes / 4)
};

__device__ __forceinline__ uint32_t tile_pos(uint32_t h, const TileMap& tm) {
    return tm.cspace ? h : uint32_t(py_index(h, tm.im));
}

__device__ __forceinline__ uint64_t tile_word0(uint32_t t, const TileMap& tm) {
    const uint64_t p0 = uint64_t(t) << tm.tb;
    uint64_t w = p0 >> 5;
    if (tm.cspace && p0 >= (1ull << 31)) w += tm.delta_words;
    return w;
}

// Block-wide exclusive scan of a[0..B) in LDS into out[0..B], out[B] = total.  Any blockDim
// that is a multiple of 64 (<= 1024).  `warp_sums` needs blockDim/64 entries.
__device__ __forceinline__ void block_exclusive_scan(const uint32_t* a, uint32_t* out, uint32_t B,
                                                     uint32_t* warp_sums) {
    const uint32_t nt = blockDim.x, tid = threadIdx.x;
    const uint32_t per = (B + nt - 1) / nt;
    const uint32_t lo = min(B, tid * per), hi = min(B, lo + per);
    uint32_t sum = 0;
    for (uint32_t j = lo; j < hi; ++j) sum += a[j];
    // inclusive wave scan of `sum`
    uint32_t v = sum;
    const uint32_t lane = tid & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(v, d, 64);
        if (lane >= uint32_t(d)) v += o;
    }
    if (lane == 63) warp_sums[tid >> 6] = v;
    __syncthreads();
    if (tid < 64) {
        const uint32_t nw = nt >> 6;
        uint32_t w = tid < nw ? warp_sums[tid] : 0u;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(w, d, 64);
            if (tid >= uint32_t(d)) w += o;
        }
        if (tid < nw) warp_sums[tid] = w;  // inclusive
    }
    __syncthreads();
    uint32_t run = v - sum + ((tid >> 6) ? warp_sums[(tid >> 6) - 1] : 0u);
    for (uint32_t j = lo; j < hi; ++j) {
        const uint32_t x = a[j];
        out[j] = run;
        run += x;
    }
    if (tid == nt - 1) out[B] = run;
    __syncthreads();
}

// Pass 1: per-workgroup tile histogram over its key range → counts[g * B + b].
template <int KMAX, int KM>
__global__ void __launch_bounds__(1024) k_hist(KeySet ks, uint64_t n, int k, TileMap tm, uint64_t keys_per_wg,
                                               uint32_t* __restrict__ counts) {
    extern __shared__ uint32_t smem[];
    const uint32_t B = tm.nbuckets;
    uint32_t* hist = smem;
    for (uint32_t b = threadIdx.x; b < B; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    const uint64_t k0 = uint64_t(blockIdx.x) * keys_per_wg;
    const uint64_t k1 = min(n, k0 + keys_per_wg);
    for (uint64_t i = k0 + threadIdx.x; i < k1; i += blockDim.x) {
        hash_key<KMAX, KM>(ks, i, k, [&](int, uint32_t h) {
            atomicAdd(hist + (tile_pos(h, tm) >> tm.tb), 1u);
        });
    }
    __syncthreads();
    uint32_t* row = counts + uint64_t(blockIdx.x) * B;
    for (uint32_t b = threadIdx.x; b < B; b += blockDim.x) row[b] = hist[b];
}

// Column scan over workgroups: counts[g][b] ← Σ_{g'<g} counts[g'][b]; total[b] ← Σ_g.
// One block of 1024 threads handles 64 buckets: wave w sums rows [w*G/16, (w+1)*G/16).
__global__ void __launch_bounds__(1024) k_colscan(uint32_t* __restrict__ counts, uint32_t G, uint32_t B,
                                                  uint32_t* __restrict__ total) {
    __shared__ uint32_t part[16][64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t b = blockIdx.x * 64 + lane;
    const uint32_t rows = (G + 15) / 16;
    const uint32_t r0 = min(G, w * rows), r1 = min(G, r0 + rows);
    uint32_t s = 0;
    if (b < B)
        for (uint32_t r = r0; r < r1; ++r) s += counts[uint64_t(r) * B + b];
    part[w][lane] = s;
    __syncthreads();
    uint32_t run = 0;
    for (uint32_t j = 0; j < w; ++j) run += part[j][lane];
    if (b < B) {
        for (uint32_t r = r0; r < r1; ++r) {
            const uint64_t o = uint64_t(r) * B + b;
            const uint32_t c = counts[o];
            counts[o] = run;
            run += c;
        }
        if (w == 15) total[b] = run;
    }
}

// base[0..B] = exclusive scan of total[0..B) (single block).
__global__ void __launch_bounds__(1024) k_basescan(const uint32_t* __restrict__ total, uint32_t B,
                                                   uint32_t* __restrict__ base) {
    extern __shared__ uint32_t smem[];
    uint32_t* a = smem;
    uint32_t* out = a + B;
    uint32_t* ws = out + B + 1;
    for (uint32_t b = threadIdx.x; b < B; b += blockDim.x) a[b] = total[b];
    __syncthreads();
    block_exclusive_scan(a, out, B, ws);
    for (uint32_t b = threadIdx.x; b <= B; b += blockDim.x) base[b] = out[b];
}

// Pass 2: each workgroup re-hashes its key range in sub-chunks of `keys_per_sub` keys, counting-
// sorts the sub-chunk's positions by tile in LDS, and writes each tile's run contiguously at
// its cursor (base[b] + column prefix + what it already wrote).
template <int KMAX, int KM>
__global__ void __launch_bounds__(1024) k_scatter(KeySet ks, uint64_t n, int k, TileMap tm, uint64_t keys_per_wg,
                                                  uint32_t keys_per_sub, const uint32_t* __restrict__ colprefix,
                                                  const uint32_t* __restrict__ base, uint32_t* __restrict__ buf) {
    extern __shared__ uint32_t smem[];
    const uint32_t B = tm.nbuckets;
    uint32_t* cursor = smem;       // B
    uint32_t* lcnt = cursor + B;   // B   (histogram, then running slot)
    uint32_t* lbase = lcnt + B;    // B+1
    uint32_t* ws = lbase + B + 1;  // 16
    uint32_t* stage = ws + 16;     // keys_per_sub * k
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    for (uint32_t b = tid; b < B; b += nt) cursor[b] = base[b] + colprefix[uint64_t(blockIdx.x) * B + b];
    const uint64_t k0 = uint64_t(blockIdx.x) * keys_per_wg;
    const uint64_t k1 = min(n, k0 + keys_per_wg);
    for (uint64_t s0 = k0; s0 < k1; s0 += keys_per_sub) {
        const uint64_t s1 = min(k1, s0 + keys_per_sub);
        for (uint32_t b = tid; b < B; b += nt) lcnt[b] = 0;
        __syncthreads();
        for (uint64_t i = s0 + tid; i < s1; i += nt)
            hash_key<KMAX, KM>(ks, i, k, [&](int, uint32_t h) { atomicAdd(lcnt + (tile_pos(h, tm) >> tm.tb), 1u); });
        __syncthreads();
        block_exclusive_scan(lcnt, lbase, B, ws);
        for (uint32_t b = tid; b < B; b += nt) lcnt[b] = lbase[b];
        __syncthreads();
        for (uint64_t i = s0 + tid; i < s1; i += nt)
            hash_key<KMAX, KM>(ks, i, k, [&](int, uint32_t h) {
                const uint32_t p = tile_pos(h, tm);
                const uint32_t slot = atomicAdd(lcnt + (p >> tm.tb), 1u);
                stage[slot] = p;
            });
        __syncthreads();
        const uint32_t tot = lbase[B];
        for (uint32_t e = tid; e < tot; e += nt) {
            const uint32_t p = stage[e];
            const uint32_t b = p >> tm.tb;
            buf[uint64_t(cursor[b]) + (e - lbase[b])] = p;
        }
        __syncthreads();
        for (uint32_t b = tid; b < B; b += nt) cursor[b] += lbase[b + 1] - lbase[b];
        __syncthreads();
    }
}

// Pass 3: one workgroup per tile.  ORs the tile's positions into LDS and writes the tile.
// `pristine` = the bitmap is logically all-zero (nothing to read back).
__global__ void __launch_bounds__(1024) k_tile(const uint32_t* __restrict__ buf, const uint32_t* __restrict__ base,
                                               TileMap tm, uint32_t* __restrict__ bitmap, int pristine) {
    extern __shared__ uint32_t tile[];
    const uint32_t t = blockIdx.x;
    const uint32_t W = 1u << (tm.tb - 5);
    const uint64_t w0 = tile_word0(t, tm);
    const uint32_t nw = uint32_t(min<uint64_t>(W, tm.total_words - w0));
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    if (pristine) {
        for (uint32_t w = tid; w < W; w += nt) tile[w] = 0;
    } else {
        for (uint32_t w = tid; w < W; w += nt) tile[w] = w < nw ? bitmap[w0 + w] : 0u;
    }
    __syncthreads();
    const uint32_t e0 = base[t], e1 = base[t + 1];
    const uint32_t lmask = (1u << tm.tb) - 1u;
    for (uint32_t e = e0 + tid; e < e1; e += nt) {
        const uint32_t p = buf[e] & lmask;
        atomicOr(tile + (p >> 5), 1u << (p & 31));
    }
    __syncthreads();
    for (uint32_t w = tid; w < nw; w += nt) bitmap[w0 + w] = tile[w];
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
