// Per-key call latency from C (no Python): pbf_may_contain on one filter and pbf_may_contain_set
// over 1..16 filters of LsmStorage.get's sizes (20k..170k keys at fp 0.001, k = 10; the bench's
// get_16_filters set), answered by the resident reader.  Splits a get's time between the
// library + device round trip (this program) and the Python above it (bench.py dropin_latency).
//   gcc -O2 -o tools/microbench/get_latency tools/microbench/get_latency.c -Iinclude
//       -Lpebbledb_amd -lpebblebloom -Wl,-rpath,'$ORIGIN/../../pebbledb_amd'
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pebblebloom.h"

static double now_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

#define CK(x)                                                                      \
    do {                                                                           \
        int rc_ = (x);                                                             \
        if (rc_) {                                                                 \
            fprintf(stderr, "%s: %d %s\n", #x, rc_, pbf_last_error());             \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

static void hexkey(uint64_t i, char* out) {  // 16 lowercase hex chars
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    for (int b = 0; b < 16; ++b) out[b] = "0123456789abcdef"[(z >> (60 - 4 * b)) & 15];
}

#ifndef GET_LATENCY_LIB
int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20000;
    enum { NF = 16 };
    pbf_filter_t* fs[NF];
    uint64_t start = 0;
    for (int f = 0; f < NF; ++f) {
        const uint64_t n = 20000 + 10000 * (uint64_t)f;
        const uint64_t nb = (uint64_t)(n * 14.3775 / 8) + 1;  // ~ -n ln(0.001) / ln2^2 bits
        CK(pbf_create(0, nb, 10, &fs[f]));
        char* keys = malloc(n * 16);
        uint64_t* off = malloc((n + 1) * sizeof(uint64_t));
        for (uint64_t i = 0; i < n; ++i) {
            hexkey(start + i, keys + 16 * i);
            off[i] = 16 * i;
        }
        off[n] = 16 * n;
        CK(pbf_add(fs[f], (const uint8_t*)keys, off, n, 0));
        CK(pbf_sync(fs[f]));
        free(keys);
        free(off);
        start += n;
    }
    char key[16];
    int out = 0;
    uint8_t bits[8];
    // warm: the reader wave launched, the filters' lines in the reader's L2
    for (int i = 0; i < 2000; ++i) {
        hexkey(start - 500 + (i % 1000), key);
        CK(pbf_may_contain_set(fs, NF, (const uint8_t*)key, 16, bits));
    }
    double t0 = now_us();
    for (int i = 0; i < reps; ++i) {
        hexkey(start - 500 + (i % 1000), key);
        CK(pbf_may_contain(fs[NF - 1], (const uint8_t*)key, 16, &out));
    }
    printf("may_contain (k=10, 170k-key filter): %.2f us\n", (now_us() - t0) / reps);
    // filter size vs k: which of them makes a one-filter call slower
    const uint64_t nbs[] = {1024, 1024, 1024, 307200, 307200, 307200};
    const uint32_t ks[] = {1, 4, 10, 1, 4, 10};
    for (int v = 0; v < 6; ++v) {
        pbf_filter_t* g;
        CK(pbf_create(0, nbs[v], ks[v], &g));
        char* keys = malloc(1000 * 16);
        uint64_t off[1001];
        for (uint64_t i = 0; i < 1000; ++i) {
            hexkey(i, keys + 16 * i);
            off[i] = 16 * i;
        }
        off[1000] = 16000;
        CK(pbf_add(g, (const uint8_t*)keys, off, 1000, 0));
        CK(pbf_sync(g));
        free(keys);
        for (int i = 0; i < 2000; ++i) {
            hexkey(i % 2000, key);
            CK(pbf_may_contain(g, (const uint8_t*)key, 16, &out));
        }
        t0 = now_us();
        for (int i = 0; i < reps; ++i) {
            hexkey(i % 2000, key);
            CK(pbf_may_contain(g, (const uint8_t*)key, 16, &out));
        }
        printf("may_contain nb_bytes %6llu k %2u: %.2f us\n", (unsigned long long)nbs[v], ks[v], (now_us() - t0) / reps);
        pbf_destroy(g);
    }
    const int sizes[] = {1, 2, 4, 8, 16};
    for (int s = 0; s < 5; ++s) {
        const int nf = sizes[s];
        t0 = now_us();
        for (int i = 0; i < reps; ++i) {
            hexkey(start - 500 + (i % 1000), key);
            CK(pbf_may_contain_set(fs + NF - nf, (uint32_t)nf, (const uint8_t*)key, 16, bits));
        }
        const double per = (now_us() - t0) / reps;
        uint64_t r1 = 0, d1 = 0;
        CK(pbf_resident_stats(0, &r1, &d1));
        static uint64_t r0 = 0, d0 = 0;
        printf("may_contain_set over %2d filters: %.2f us (device %.2f us of it)\n", nf, per,
               r1 > r0 ? (d1 - d0) * 1e-3 / (r1 - r0) : 0.0);
        r0 = r1;
        d0 = d1;
    }
    // the same 16 filters, one key repeated (its bitmap lines stay hot)
    hexkey(start - 1, key);
    t0 = now_us();
    for (int i = 0; i < reps; ++i) CK(pbf_may_contain_set(fs, NF, (const uint8_t*)key, 16, bits));
    printf("may_contain_set over 16 filters, one key: %.2f us\n", (now_us() - t0) / reps);
    uint64_t nreq = 0, dns = 0;
    CK(pbf_resident_stats(0, &nreq, &dns));
    printf("resident reader: %llu requests, %.2f us each on the device (seen -> answered)\n",
           (unsigned long long)nreq, nreq ? dns * 1e-3 / nreq : 0.0);
    for (int f = 0; f < NF; ++f) pbf_destroy(fs[f]);
    return 0;
}
#endif

// Loaded into a Python process (tools/diag/get_stage_check.py): the same call loop over filters
// the Python layer built, keys given as 16-byte records.  Returns microseconds per call.
double loop_set(pbf_filter_t* const* fs, uint32_t nf, const char* keys16, int nkeys, int reps) {
    uint8_t bits[8];
    for (int i = 0; i < 1000; ++i) pbf_may_contain_set(fs, nf, (const uint8_t*)keys16 + 16 * (i % nkeys), 16, bits);
    const double t0 = now_us();
    for (int i = 0; i < reps; ++i) pbf_may_contain_set(fs, nf, (const uint8_t*)keys16 + 16 * (i % nkeys), 16, bits);
    return (now_us() - t0) / reps;
}

// The same loop with a pause of `gap_us` between calls (the caller's own work between gets):
// microseconds per call, the pause excluded.
double loop_set_gap(pbf_filter_t* const* fs, uint32_t nf, const char* keys16, int nkeys, int reps, double gap_us) {
    uint8_t bits[8];
    double inside = 0;
    for (int i = 0; i < reps; ++i) {
        const double g0 = now_us();
        while (now_us() - g0 < gap_us) {
        }
        const double t0 = now_us();
        pbf_may_contain_set(fs, nf, (const uint8_t*)keys16 + 16 * (i % nkeys), 16, bits);
        inside += now_us() - t0;
    }
    return inside / reps;
}
