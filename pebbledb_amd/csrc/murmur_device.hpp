// Device-side hashing for the bloom path: MurmurHash3_x86_32 over UTF-8 key bytes with seeds
// 0..k-1 (mmh3.hash(key, i), reference src/bloom_filter.py:46) and the Python floor-mod
// `hash % bits_size` (bloom_filter.py:47), for gfx950.
//
// A key's 4-byte blocks are mixed (k1 * c1, rotl 15, * c2) independently of the seed, so one
// pass over the key bytes feeds all k seed states at once: the bytes are loaded once and the
// per-block multiply pair is paid once per key, not once per seed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbf {

constexpr uint32_t kC1 = 0xcc9e2d51u;
constexpr uint32_t kC2 = 0x1b873593u;

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return __builtin_rotateleft32(x, r); }

__device__ __forceinline__ uint32_t mix_block(uint32_t k) {
    k *= kC1;
    k = rotl32(k, 15);
    return k * kC2;
}

// h * 5 as one full-rate shift-add: left to itself the compiler folds `h * 5 + c` into a
// 64-bit v_mad_u64_u32 (a quarter-rate instruction), once per 4-byte block and seed — the
// single largest VALU cost of hashing a 16-byte key k times.
__device__ __forceinline__ uint32_t times5(uint32_t h) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 2, %1" : "=v"(r) : "v"(h));
    return r;
}

__device__ __forceinline__ uint32_t round_h(uint32_t h, uint32_t km) {
    h ^= km;
    h = rotl32(h, 13);
    return times5(h) + 0xe6546b64u;
}

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

// Little-endian 4 bytes at an arbitrary byte address.  Only dwords that contain at least one
// requested byte are touched, so the read never leaves the page of a valid byte.
__device__ __forceinline__ uint32_t load_u32_any(const uint8_t* p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const uint32_t sh = uint32_t(a & 3);
    const uint32_t lo = q[0];
    if (sh == 0) return lo;
    const uint32_t hi = q[1];
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// The t (1..3) tail bytes at p, zero-extended, little-endian (MurmurHash3 tail block).
__device__ __forceinline__ uint32_t load_tail(const uint8_t* p, uint32_t t) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const uint32_t sh = uint32_t(a & 3);
    const uint32_t lo = q[0];
    const uint32_t hi = (sh + t > 4) ? q[1] : 0u;
    const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, sh);
    return v & ((1u << (8 * t)) - 1u);
}

// k seeds of MurmurHash3_x86_32 for one key at any byte address, sbase .. sbase+k-1; emit(s,
// hash_u32) is called for s = 0..k-1 (seed sbase + s).  KMAX is the compile-time register budget
// for seed states (k <= KMAX).  The key is read as aligned 16-byte chunks (4 dwordx4 loads in
// flight per 64 bytes) instead of two dword loads per 4-byte block.  Every chunk read holds at
// least one byte of the key (first chunk = floor16(p), last = the one holding p[len-1]), so the
// reads never leave a page the key touches.  Block j = bytes p[4j, 4j+4) = alignbyte(W[w0+j+1],
// W[w0+j], sh) over the chunks' words W (w0 = (p & 15) / 4, sh = p & 3); it is mixed when its
// upper word streams past; the t = len & 3 tail bytes come from W[w0+nb] and W[w0+nb+1].
template <int KMAX, class Emit>
__device__ __forceinline__ void murmur_seeds_chunked(const uint8_t* p, uint32_t len, int k, Emit&& emit,
                                                     int sbase = 0) {
    uint32_t h[KMAX];
#pragma unroll
    for (int s = 0; s < KMAX; ++s) h[s] = uint32_t(sbase + s);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint4* base = reinterpret_cast<const uint4*>(a & ~uintptr_t(15));
    const uint32_t off = uint32_t(a & 15), w0 = off >> 2, sh = off & 3;
    const uint32_t nb = len >> 2, t = len & 3;
    const uint32_t nchunks = len ? (off + len + 15) >> 4 : 0;
    const uint32_t wt = w0 + nb;  // word holding the first tail byte
    uint32_t prev = 0, tlo = 0, thi = 0;
    auto word = [&](uint32_t wi, uint32_t w) {  // word index wi (from base) streams past
        const uint32_t j = wi - 1 - w0;         // block whose upper word this is
        if (wi > w0 && j < nb) {
            const uint32_t km = mix_block(__builtin_amdgcn_alignbyte(w, prev, sh));
#pragma unroll
            for (int s = 0; s < KMAX; ++s) h[s] = round_h(h[s], km);
        }
        if (wi == wt) tlo = w;
        if (wi == wt + 1) thi = w;
        prev = w;
    };
    uint32_t wi = 0;
    for (uint32_t c0 = 0; c0 < nchunks; c0 += 4) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = base[min(c0 + u, nchunks - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (c0 + u < nchunks) {
                word(wi, v[u].x);
                word(wi + 1, v[u].y);
                word(wi + 2, v[u].z);
                word(wi + 3, v[u].w);
                wi += 4;
            }
        }
    }
    // a key ending on a chunk boundary with sh = 0: its last block's upper word is not needed
    if (len) word(wi, 0u);
    if (t) {
        const uint32_t km = mix_block(__builtin_amdgcn_alignbyte(thi, tlo, sh) & ((1u << (8 * t)) - 1u));
#pragma unroll
        for (int s = 0; s < KMAX; ++s) h[s] ^= km;
    }
#pragma unroll
    for (int s = 0; s < KMAX; ++s)
        if (s < k) emit(s, fmix32(h[s] ^ len));
}

// Fixed 16-byte keys from one 16-byte load (the C2/C4/C5 key shape).
// The first round, rotl(seed ^ m0, 13), is rotl(m0, 13) ^ rotl(seed, 13): the key's part is
// rotated once for all seeds, the seed's part is uniform (scalar) — one vector op per seed saved.
template <int KMAX, class Emit>
__device__ __forceinline__ void murmur_seeds16(uint4 w, int k, Emit&& emit, int sbase = 0) {
    const uint32_t m0 = mix_block(w.x), m1 = mix_block(w.y), m2 = mix_block(w.z), m3 = mix_block(w.w);
    const uint32_t r0 = rotl32(m0, 13);
#pragma unroll
    for (int s = 0; s < KMAX; ++s) {
        if (s < k) {
            uint32_t h = times5(r0 ^ rotl32(uint32_t(sbase + s), 13)) + 0xe6546b64u;
            h = round_h(h, m1);
            h = round_h(h, m2);
            h = round_h(h, m3);
            emit(s, fmix32(h ^ 16u));
        }
    }
}

// Runtime-k fallback (k > 32): one seed at a time, key bytes re-read (from L1) per seed.
template <class Emit>
__device__ __forceinline__ void murmur_seeds_loop(const uint8_t* p, uint32_t len, int k, Emit&& emit, int sbase = 0) {
    const uint32_t nb = len >> 2;
    const uint32_t t = len & 3;
    for (int s = 0; s < k; ++s) {
        uint32_t h = uint32_t(sbase + s);
        for (uint32_t b = 0; b < nb; ++b) h = round_h(h, mix_block(load_u32_any(p + 4 * b)));
        if (t) h ^= mix_block(load_tail(p + 4 * nb, t));
        emit(s, fmix32(h ^ len));
    }
}

// ---------------------------------------------------------------- Python floor-mod index
// idx = h % m with h the SIGNED int32 hash and Python's floor semantics (result in [0, m)).
enum IndexMode : uint32_t {
    kPow2 = 0,   // m a power of two, m <= 2^32: idx = u32(h) & (m-1)
    kSmall = 1,  // m < 2^31: a = h>=0 ? h : ~h (< 2^31); r = a mod m; idx = h>=0 ? r : m-1-r
    kLarge = 2,  // m >= 2^31: |h| <= 2^31 <= m, so idx = h>=0 ? h : h + m (64-bit)
};

struct IndexMap {
    uint64_t m;      // bits_size = 8 * nb_bytes
    uint64_t magic;  // Lemire fastmod constant for kSmall: floor((2^64-1)/m) + 1
    uint32_t mode;
    uint32_t mask;   // m-1 for kPow2
};

// a mod d for a, d < 2^32 (Lemire, Kaser & Kurz, "Faster remainder by direct computation").
__device__ __forceinline__ uint32_t fastmod_u32(uint32_t a, uint64_t magic, uint32_t d) {
    const uint64_t low = magic * uint64_t(a);
    return uint32_t(__umul64hi(low, uint64_t(d)));
}

__device__ __forceinline__ uint64_t py_index(uint32_t hu, const IndexMap& im) {
    const int32_t h = int32_t(hu);
    if (im.mode == kPow2) return uint64_t(hu & im.mask);
    if (im.mode == kSmall) {
        const uint32_t a = h >= 0 ? hu : ~hu;
        const uint32_t r = fastmod_u32(a, im.magic, uint32_t(im.m));
        return h >= 0 ? uint64_t(r) : uint64_t(uint32_t(im.m) - 1u - r);
    }
    return h >= 0 ? uint64_t(hu) : uint64_t(int64_t(h) + int64_t(im.m));
}

}  // namespace pbf
