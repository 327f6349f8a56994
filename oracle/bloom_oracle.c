/*
 * ORACLE — test infrastructure only.  CPU restatement of the reference's bloom-filter path
 * (MaudGautier/pebbledb src/bloom_filter.py) used as the parity checker for the HIP engine.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library;
 * the product (pebbledb_amd/, libpebblebloom.so) never links or calls it.
 *
 * Pinned against the real reference: the fixtures in tests/golden/ were produced by importing the
 * reference's own BloomFilter (tools/gen_golden.py) and tests/test_oracle_golden.py checks this
 * file against every one of them.
 *
 * Third-party algorithm restated here: MurmurHash3_x86_32 as provided by mmh3==4.1.0
 * (reference requirements.txt:12, called at src/bloom_filter.py:46).  Restated from the
 * published algorithm (Austin Appleby's public-domain MurmurHash3, x86 32-bit variant):
 * 4-byte little-endian blocks mixed with c1=0xcc9e2d51, c2=0x1b873593, rotl 15 / 13,
 * h = h*5 + 0xe6546b64; tail of 1..3 bytes; h ^= len; fmix32.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

static inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

/* mmh3.hash(key, seed) — returns the signed int32 that mmh3 returns by default
 * (bloom_filter.py:46 uses the default signed=True). */
int32_t oracle_murmur3_x86_32(const uint8_t *key, uint64_t len, uint32_t seed) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h = seed;
    uint64_t nblocks = len / 4;
    for (uint64_t i = 0; i < nblocks; i++) {
        uint32_t k = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) |
                     ((uint32_t)key[4 * i + 2] << 16) | ((uint32_t)key[4 * i + 3] << 24);
        k *= c1;
        k = rotl32(k, 15);
        k *= c2;
        h ^= k;
        h = rotl32(h, 13);
        h = h * 5u + 0xe6546b64u;
    }
    const uint8_t *tail = key + nblocks * 4;
    uint32_t k = 0;
    switch (len & 3) {
        case 3: k ^= (uint32_t)tail[2] << 16; /* fallthrough */
        case 2: k ^= (uint32_t)tail[1] << 8;  /* fallthrough */
        case 1: k ^= tail[0];
            k *= c1;
            k = rotl32(k, 15);
            k *= c2;
            h ^= k;
    }
    h ^= (uint32_t)len;
    return (int32_t)fmix32(h);
}

/* `hashed_key % self.bits_size` with Python floor-mod semantics (bloom_filter.py:47):
 * the result is in [0, m) for a signed h and any m > 0. */
uint64_t oracle_index(int32_t h, uint64_t m) {
    int64_t r = (int64_t)h % (int64_t)m;  /* C truncates toward zero */
    if (r < 0) r += (int64_t)m;
    return (uint64_t)r;
}

/* BloomFilter._hash (bloom_filter.py:38-49): k indices for one UTF-8 key. */
void oracle_hash_indices(const uint8_t *key, uint64_t len, uint32_t k, uint64_t m, uint64_t *out) {
    for (uint32_t i = 0; i < k; i++) out[i] = oracle_index(oracle_murmur3_x86_32(key, len, i), m);
}

static inline void key_span(const uint8_t *keys, const uint64_t *offsets, uint64_t key_len, uint64_t i,
                            const uint8_t **p, uint64_t *len) {
    if (offsets) {
        *p = keys + offsets[i];
        *len = offsets[i + 1] - offsets[i];
    } else {
        *p = keys + i * key_len;
        *len = key_len;
    }
}

/* BloomFilter.add over a batch (bloom_filter.py:60-65, _set_bit :51-54).  `bitmap` holds the
 * filter as to_bytes() lays it out (bloom_filter.py:76-81): byte i = bits >> 8i & 0xFF, i.e.
 * bit j of the filter is bit (j & 7) of byte (j >> 3).  ORs into the existing contents.
 * Fixed-width keys when offsets == NULL (key i = keys[i*key_len, (i+1)*key_len)). */
int oracle_build(uint8_t *bitmap, uint64_t nb_bytes, uint32_t k, const uint8_t *keys,
                 const uint64_t *offsets, uint64_t key_len, uint64_t n) {
    if (nb_bytes == 0) return -1; /* reference: ZeroDivisionError in `% self.bits_size` */
    const uint64_t m = 8 * nb_bytes;
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *p;
        uint64_t len;
        key_span(keys, offsets, key_len, i, &p, &len);
        for (uint32_t s = 0; s < k; s++) {
            uint64_t idx = oracle_index(oracle_murmur3_x86_32(p, len, s), m);
            bitmap[idx >> 3] |= (uint8_t)(1u << (idx & 7));
        }
    }
    return 0;
}

/* BloomFilter.may_contain over a batch (bloom_filter.py:67-74, _is_bit_set :56-58).  The
 * early-exit loop returns the AND over the k bits; the hit mask is LSB-first:
 * bit (i & 7) of hitmask[i >> 3] = may_contain(key i).  hitmask must hold ceil(n/8) bytes. */
int oracle_probe(const uint8_t *bitmap, uint64_t nb_bytes, uint32_t k, const uint8_t *keys,
                 const uint64_t *offsets, uint64_t key_len, uint64_t n, uint8_t *hitmask) {
    if (nb_bytes == 0) return -1;
    const uint64_t m = 8 * nb_bytes;
    memset(hitmask, 0, (size_t)((n + 7) / 8));
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *p;
        uint64_t len;
        key_span(keys, offsets, key_len, i, &p, &len);
        int hit = 1;
        for (uint32_t s = 0; s < k && hit; s++) {
            uint64_t idx = oracle_index(oracle_murmur3_x86_32(p, len, s), m);
            hit = (bitmap[idx >> 3] >> (idx & 7)) & 1;
        }
        if (hit) hitmask[i >> 3] |= (uint8_t)(1u << (i & 7));
    }
    return 0;
}

/* Multi-threaded twins (OpenMP, all host cores) — the "fair" CPU number reported beside the
 * single-core port in bench.py's cpu_baseline leg.  OR is idempotent and commutative, so the
 * result equals oracle_build's bit for bit. */
int oracle_build_omp(uint8_t *bitmap, uint64_t nb_bytes, uint32_t k, const uint8_t *keys,
                     const uint64_t *offsets, uint64_t key_len, uint64_t n) {
    if (nb_bytes == 0) return -1;
    const uint64_t m = 8 * nb_bytes;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        const uint8_t *p;
        uint64_t len;
        key_span(keys, offsets, key_len, (uint64_t)i, &p, &len);
        for (uint32_t s = 0; s < k; s++) {
            uint64_t idx = oracle_index(oracle_murmur3_x86_32(p, len, s), m);
            __atomic_fetch_or(&bitmap[idx >> 3], (uint8_t)(1u << (idx & 7)), __ATOMIC_RELAXED);
        }
    }
    return 0;
}

int oracle_probe_omp(const uint8_t *bitmap, uint64_t nb_bytes, uint32_t k, const uint8_t *keys,
                     const uint64_t *offsets, uint64_t key_len, uint64_t n, uint8_t *hitmask) {
    if (nb_bytes == 0) return -1;
    const uint64_t m = 8 * nb_bytes;
    const int64_t nbytes_out = (int64_t)((n + 7) / 8);
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nbytes_out; b++) {
        uint8_t out = 0;
        for (uint64_t j = 0; j < 8; j++) {
            uint64_t i = (uint64_t)b * 8 + j;
            if (i >= n) break;
            const uint8_t *p;
            uint64_t len;
            key_span(keys, offsets, key_len, i, &p, &len);
            int hit = 1;
            for (uint32_t s = 0; s < k && hit; s++) {
                uint64_t idx = oracle_index(oracle_murmur3_x86_32(p, len, s), m);
                hit = (bitmap[idx >> 3] >> (idx & 7)) & 1;
            }
            out |= (uint8_t)(hit << j);
        }
        hitmask[b] = out;
    }
    return 0;
}

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
