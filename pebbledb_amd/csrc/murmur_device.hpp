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

// A load through the global address space.  Key bytes and offsets (device memory, or mapped
// pinned host memory for the one-key probes) reach the kernels through generic pointers, which
// the compiler loads with flat_* instructions; a flat load's wait also drains every outstanding
// LDS operation (s_waitcnt vmcnt(0) lgkmcnt(0)), which in the partitions serialises the hash's
// key loads with the LDS atomics of the previous keys' positions.  The integer -> global pointer
// cast makes them global_load_*.
template <class T>
__device__ __forceinline__ T gld(const T* p) {
    return *(const __attribute__((address_space(1))) T*)(reinterpret_cast<uintptr_t>(p));
}
// (HIP's uint4 cannot be copied out of an address-space-qualified lvalue: load the vector type)
__device__ __forceinline__ uint4 gld(const uint4* p) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u x = *(const __attribute__((address_space(1))) v4u*)(reinterpret_cast<uintptr_t>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
}

__device__ __forceinline__ uint32_t mix_block(uint32_t k) {
    k *= kC1;
    k = rotl32(k, 15);
    return k * kC2;
}

// h * 5 + c as full-rate ops: left to itself the compiler folds `h * 5 + c` into a 64-bit
// v_mad_u64_u32 (a quarter-rate instruction), once per 4-byte block and seed — the single largest
// VALU cost of hashing a 16-byte key k times.  (h << 2) + (h + c) compiles to v_lshlrev + v_add3;
// the inline-asm v_lshl_add it replaces made the compiler pad every use with an s_nop.
__device__ __forceinline__ uint32_t times5_plus(uint32_t h, uint32_t c) { return (h << 2) + (h + c); }

__device__ __forceinline__ uint32_t round_h(uint32_t h, uint32_t km) {
    h ^= km;
    h = rotl32(h, 13);
    return times5_plus(h, 0xe6546b64u);
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
    const uint32_t lo = gld(q);
    if (sh == 0) return lo;
    const uint32_t hi = gld(q + 1);
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// The t (1..3) tail bytes at p, zero-extended, little-endian (MurmurHash3 tail block).
__device__ __forceinline__ uint32_t load_tail(const uint8_t* p, uint32_t t) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const uint32_t sh = uint32_t(a & 3);
    const uint32_t lo = gld(q);
    const uint32_t hi = (sh + t > 4) ? gld(q + 1) : 0u;
    const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, sh);
    return v & ((1u << (8 * t)) - 1u);
}

// k seeds of MurmurHash3_x86_32 for one key at any byte address, sbase .. sbase+k-1; emit(s,
// hash_u32) is called for s = 0..k-1 (seed sbase + s); KMAX is the compile-time register budget
// for seed states (k <= KMAX).  The key is processed 64 bytes (16 blocks) at a time: the
// segment's window of five aligned 16-byte chunks (every chunk read holds at least one byte of
// the key — first = floor16(p), last = the one holding p[len-1] — so the reads never leave a
// page the key touches) is
// barrel-shifted in registers by the key's word offset (two levels of selects), after which
// block j is alignbyte(W[j+1], W[j], sh) with static register indices — straight-line block
// rounds instead of a per-word state machine (C3 build 5.60 -> 5.39 ms, probe 16.6 -> 16.2 ms
// against the word-by-word chunk walk it replaced; profiles/r03/s4).  The t = len & 3 tail bytes
// come from load_tail (dwords holding key bytes only).
template <int KMAX, class Emit>
__device__ __forceinline__ void murmur_seeds_seg(const uint8_t* p, uint32_t len, int k, Emit&& emit, int sbase = 0) {
    uint32_t h[KMAX];
#pragma unroll
    for (int s = 0; s < KMAX; ++s) h[s] = uint32_t(sbase + s);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint4* base = reinterpret_cast<const uint4*>(a & ~uintptr_t(15));
    const uint32_t off = uint32_t(a & 15), w0 = off >> 2, sh = off & 3;
    const uint32_t nb = len >> 2, t = len & 3;
    const uint32_t nchunks = len ? (off + len + 15) >> 4 : 0;
    // the tail's dwords are loaded up front, beside the first segment's chunks (its latency then
    // overlaps the block rounds instead of following them)
    const uint32_t tail = t ? load_tail(p + 4 * nb, t) : 0u;
    for (uint32_t seg = 0; seg * 16 < nb; ++seg) {
        uint32_t W[20];
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            const uint4 v = gld(base + min(4 * seg + c, nchunks - 1));
            W[4 * c] = v.x;
            W[4 * c + 1] = v.y;
            W[4 * c + 2] = v.z;
            W[4 * c + 3] = v.w;
        }
        // W[i] <- W[i + w0]: the segment's blocks then start at word 0.  Written as masks: as
        // ternaries the compiler recognises a dynamically indexed array and moves W through
        // scratch memory
        const uint32_t m2 = 0u - ((w0 >> 1) & 1u), m1 = 0u - (w0 & 1u);
#pragma unroll
        for (int i = 0; i < 18; ++i) W[i] = (W[i + 2] & m2) | (W[i] & ~m2);
#pragma unroll
        for (int i = 0; i < 17; ++i) W[i] = (W[i + 1] & m1) | (W[i] & ~m1);
        const uint32_t nbs = min(nb - 16 * seg, 16u);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (uint32_t(j) < nbs) {
                const uint32_t km = mix_block(__builtin_amdgcn_alignbyte(W[j + 1], W[j], sh));
#pragma unroll
                for (int s = 0; s < KMAX; ++s) h[s] = round_h(h[s], km);
            }
        }
    }
    if (t) {
        const uint32_t km = mix_block(tail);
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
            uint32_t h = times5_plus(r0 ^ rotl32(uint32_t(sbase + s), 13), 0xe6546b64u);
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
// For m < 2^31 write a = h >= 0 ? h : ~h (a < 2^31); then idx = h >= 0 ? a mod m : m-1-(a mod m).
enum IndexMode : uint32_t {
    kPow2 = 0,   // m a power of two, m <= 2^32: idx = u32(h) & (m-1)
    kSmall = 1,  // m < 2^30: a mod m by a 32-bit reciprocal (below)
    kLarge = 2,  // m >= 2^31: |h| <= 2^31 <= m, so idx = h>=0 ? h : h + m (64-bit)
    kNear = 3,   // 2^30 < m < 2^31: a < 2^31 < 2m, so a mod m = a >= m ? a - m : a (no multiply)
};

struct IndexMap {
    uint64_t m;      // bits_size = 8 * nb_bytes
    uint64_t magic;  // kSmall: M = ceil(2^(31+l) / m), l = ceil(log2 m) (M < 2^32)
    uint32_t mode;
    uint32_t mask;   // kPow2: m-1; kSmall: the shift l-1
};

// a mod m for a < 2^31, m < 2^30 not a power of two: q = floor(a / m) = mulhi(a, M) >> (l-1)
// (Granlund & Montgomery, "Division by invariant integers using multiplication", Thm 4.2 with
// N = 31: 2^(31+l) <= M*m < 2^(31+l) + m <= 2^(31+l) + 2^l), r = a - q*m.  Two quarter-rate
// multiplies instead of the six of a 64-bit Lemire fastmod (C4's product-sized filters hash 10
// positions per key through this).
__device__ __forceinline__ uint32_t mod_small(uint32_t a, uint32_t magic, uint32_t shift, uint32_t m) {
    const uint32_t q = __umulhi(a, magic) >> shift;
    return a - q * m;
}

__device__ __forceinline__ uint64_t py_index(uint32_t hu, const IndexMap& im) {
    const int32_t h = int32_t(hu);
    if (im.mode == kPow2) return uint64_t(hu & im.mask);
    if (im.mode == kLarge) return h >= 0 ? uint64_t(hu) : uint64_t(int64_t(h) + int64_t(im.m));
    const uint32_t m = uint32_t(im.m);
    const uint32_t a = h >= 0 ? hu : ~hu;
    const uint32_t r = im.mode == kNear ? (a >= m ? a - m : a) : mod_small(a, uint32_t(im.magic), im.mask, m);
    return h >= 0 ? uint64_t(r) : uint64_t(m - 1u - r);
}

}  // namespace pbf
