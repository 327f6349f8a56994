// LDS-tiled bloom build and probe for gfx950 (reference semantics: src/bloom_filter.py:60-74).
//
// Random 4-byte read-modify-writes / reads into a 128 MiB bitmap are bound by the fabric's
// request rate (measured ~55 G 64-B requests/s chip-wide), not by HBM bytes.  The tiled path
// turns them into streams:
//
//   positions   A key's k hash positions.  For m <= 2^32 a position is the bit index (u32).
//               For m > 2^32 only [0, 2^31) U [m - 2^31, m) is reachable (|h| <= 2^31): the
//               position is u32(h) and p >= 2^31 lives at bit p + (m - 2^32).
//   tiles       2^TB positions (TB <= 20: 128 KiB of LDS).  B = number of tiles.
//   regions     Partition workgroup g owns one fixed-capacity region per tile: entries of
//               (g, b) live at regions[(g*B + b)*cap ...].  No histogram pass is needed;
//               entries beyond `cap` (only under heavy key duplication) go to an overflow list
//               that a small fix-up kernel applies with global atomics.
//
// Build:  k_part<build>  hash keys in LDS-sized sub-chunks, counting-sort positions by tile
//                        in LDS, append each tile's run to the workgroup's region.
//         k_tile_build   one workgroup per tile: OR the tile's positions into LDS, write the
//                        tile once (128 KiB, coalesced).
//         k_ovf_build    global atomicOr of overflow positions (usually none).
// Probe:  k_part<probe>  same partition; an entry is (key-in-group << 20 | position in tile)
//                        (a group = 4096 consecutive keys of the workgroup), and the in-region
//                        counts at every group boundary are kept (pref) — the ring
//                        partition's format, so both partitions share one gather.
//         k_tile_probe   one workgroup per tile: load the bitmap tile into LDS, test every
//                        entry, write one result bit per entry (R, parallel to regions).
//         k_gather_ring  (ring_kernels.hpp) workgroup g replays its regions: a failed entry
//                        clears its key's bit in an LDS bitmap, wave64 ballot → hit-mask words.
//         Overflowed probe entries are tested directly against the bitmap inside k_part; a
//         miss sets the key's bit in `neg`, which the gather folds in.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bloom_kernels.hpp"

namespace pbf {

// Streaming access to the region entries and the bitmap tile write-out: each byte is written
// once and read back once or twice by a later kernel, far beyond L2, so those accesses are
// non-temporal.  Choices are the best of the A/B builds on C2 (profiles/r01/s9/nt_ab.txt,
// profiles/r01/s10/nt_ab.txt): region-entry loads, probe-partition stores, the tile build's
// bitmap write-out and the partition's 16-B key loads non-temporal (0.886 -> 0.801 ms/step);
// non-temporal build-partition stores measured 10 us slower, non-temporal bitmap loads into the
// LDS tiles no gain.
constexpr bool kNtLoad = true;        // region entries
constexpr bool kNtBuildPart = false;  // build partition's group stores
constexpr bool kNtProbePart = true;   // probe partition's group stores
constexpr bool kNtTileStore = true;   // k_tile_build's bitmap write-out
constexpr bool kNtKeys = true;        // the partitions' 16-B key loads
constexpr bool kNtTileLoad = false;   // bitmap loads into the LDS tiles
#ifndef PBF_TILE_DMA
#define PBF_TILE_DMA 1
#endif
// Regions of loads in flight per wave: the tile build 4, the tile test 8 words, the gather 4
// (16 loads per wave in the tile test and 8 regions in the gather measured slower).
constexpr int kTileBuildRegionsInFlight = 4;
#ifndef PBF_TILE_PROBE_WORDS
#define PBF_TILE_PROBE_WORDS 8
#endif
constexpr int kTileProbeWordsInFlight = PBF_TILE_PROBE_WORDS;
// The set tile test (k_tile_probe_set: region lines from L2, TAB 1) keeps 12 in flight: C5 6.62
// vs 7.01 ms, while the one-filter test is slower with 12 (profiles/r05/ab/tile_words/)
constexpr int kTileProbeSetWordsInFlight = 12;
constexpr int kGatherRegionsInFlight = 4;
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st_stream(uint32_t* p, uint4 v) {
    if constexpr (NT) {
        const u32x4v x = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(x, reinterpret_cast<u32x4v*>(p));
    } else {
        *reinterpret_cast<uint4*>(p) = v;
    }
}

template <bool NT>
__device__ __forceinline__ uint4 ld_stream_nt(const uint32_t* p) {
    if constexpr (NT) {
        const u32x4v x = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(p));
        return make_uint4(x.x, x.y, x.z, x.w);
    } else {
        return *reinterpret_cast<const uint4*>(p);
    }
}

__device__ __forceinline__ uint4 ld_stream(const uint32_t* p) { return ld_stream_nt<kNtLoad>(p); }

struct TileMap {
    IndexMap im;
    uint32_t tb;           // log2 positions per tile (<= 20)
    uint32_t nbuckets;     // B
    uint32_t cspace;       // 1 when m > 2^32
    uint32_t pad;
    uint64_t delta_words;  // (m - 2^32) / 32 when cspace
    uint64_t total_words;  // ceil(nb_bytes / 4)
};

// The bitmaps a probe partition tests its overflowed (spilled) entries against: one per filter
// of a multi-filter probe (pbf_probe_multi, all with the same m and k); filter f's misses clear
// key bits in neg + f * neg_stride.  A build passes nf = 0.
constexpr int kMaxProbeSet = 8;
struct ProbeSet {
    const uint32_t* bm[kMaxProbeSet];
    uint32_t* neg;
    uint64_t neg_stride;  // u32 words
    uint32_t nf;
    uint32_t pad;
};

// A spilled probe entry: test bit `bit` in every filter of the set, clear `key` where it is 0.
__device__ __forceinline__ void spill_probe(const ProbeSet& ps, uint64_t bit, uint64_t key) {
    for (uint32_t f = 0; f < ps.nf; ++f)
        if (!((ps.bm[f][bit >> 5] >> (bit & 31)) & 1u))
            atomicOr(ps.neg + f * ps.neg_stride + (key >> 5), 1u << (key & 31));
}

// Region (g, b) = partition workgroup g's entries of tile b, workgroup-major (a workgroup's B
// regions back to back: contiguous for the gather; tile-major measured no different).
__device__ __forceinline__ uint64_t region_id(uint32_t g, uint32_t b, uint32_t /*G*/, uint32_t B) {
    return uint64_t(g) * B + b;
}

struct PartGeom {
    uint32_t G;        // partition workgroups
    uint32_t cap;      // region capacity in entries (multiple of 32)
    uint32_t kps;      // keys per sub-chunk (kpt * 1024; <= 4096 for probes)
    uint32_t nsub;     // sub-chunks per workgroup
    uint64_t kpw;      // keys per workgroup (= nsub * kps)
    uint32_t nq;       // pref groups (4096 keys each) per workgroup
    uint32_t ring;     // ring partition: LDS ring entries per tile (0 = counting-sort partition)
    uint32_t spill_cap;  // ring partition: entries of the LDS spill buffer
    uint32_t scap;       // counting-sort partition: stage entries (a sub-chunk is placed in windows of scap)
    uint32_t tabw;       // tile test, TAB 1: words of the per-word table (0 = all of a tile's words)
};

constexpr uint32_t kSlotShift = 20;   // probe entry = key-in-group << 20 | position in tile
constexpr uint32_t kGroupKeys = 4096;  // keys per probe group (12 bits of the entry)

__device__ __forceinline__ uint32_t tile_pos(uint32_t h, const TileMap& tm) {
    return tm.cspace ? h : uint32_t(py_index(h, tm.im));
}

__device__ __forceinline__ uint64_t pos_to_bit(uint32_t p, const TileMap& tm) {
    uint64_t b = p;
    if (tm.cspace && p >= 0x80000000u) b += tm.delta_words * 32;
    return b;
}

__device__ __forceinline__ uint64_t tile_word0(uint32_t t, const TileMap& tm) {
    const uint64_t p0 = uint64_t(t) << tm.tb;
    uint64_t w = p0 >> 5;
    if (tm.cspace && p0 >= (1ull << 31)) w += tm.delta_words;
    return w;
}

// Barrier for LDS hand-offs only: waits for this wave's LDS/scalar operations, not for its
// global stores (which __syncthreads' workgroup-release fence would drain every time).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// s_waitcnt immediate (gfx9 encoding: vmcnt bits 3:0 and 15:14, expcnt 6:4, lgkmcnt 11:8) for
// vmcnt(0) alone.  As a builtin (not inline asm) the compiler's own wait placement sees it.
constexpr unsigned kWaitVmcnt0 = 0x0F70;

// Block-wide exclusive scan of a[0..B) (LDS) into out[0..B] (LDS), out[B] = total.
// blockDim a multiple of 64, <= 1024; warp_sums holds blockDim/64 entries.  Ends synced.
__device__ __forceinline__ void block_exclusive_scan(const uint32_t* a, uint32_t* out, uint32_t B,
                                                     uint32_t* warp_sums) {
    const uint32_t nt = blockDim.x, tid = threadIdx.x;
    const uint32_t per = (B + nt - 1) / nt;
    const uint32_t lo = min(B, tid * per), hi = min(B, lo + per);
    uint32_t sum = 0;
    for (uint32_t j = lo; j < hi; ++j) sum += a[j];
    uint32_t v = sum;
    const uint32_t lane = tid & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(v, d, 64);
        if (lane >= uint32_t(d)) v += o;
    }
    if (lane == 63) warp_sums[tid >> 6] = v;
    lds_barrier();
    if (tid < 64) {
        const uint32_t nw = nt >> 6;
        uint32_t w = tid < nw ? warp_sums[tid] : 0u;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(w, d, 64);
            if (tid >= uint32_t(d)) w += o;
        }
        if (tid < nw) warp_sums[tid] = w;
    }
    lds_barrier();
    uint32_t run = v - sum + ((tid >> 6) ? warp_sums[(tid >> 6) - 1] : 0u);
    for (uint32_t j = lo; j < hi; ++j) {
        const uint32_t x = a[j];
        out[j] = run;
        run += x;
    }
    if (tid == nt - 1) out[B] = run;
    lds_barrier();
}

// Largest b in [0, B) with a[b] <= e (a non-decreasing, a[0] = 0 <= e).
__device__ __forceinline__ uint32_t bucket_of(const uint32_t* a, uint32_t B, uint32_t e) {
    uint32_t lo = 0, len = B;
    while (len > 1) {
        const uint32_t half = len >> 1;
        if (a[lo + half] <= e) lo += half;
        len -= half;
    }
    return lo;
}

// ------------------------------------------------------------------ partition
// One 1024-thread workgroup per CU.  Each thread keeps up to KPT keys' KMAX (position, rank)
// pairs in registers between the counting pass and the LDS placement, so every key is hashed
// once; pg.kps = kpt_eff * 1024 keys per sub-chunk (kpt_eff <= KPT chosen by the host so the
// stage fits LDS).
constexpr int kPartThreads = 1024;
__host__ __device__ constexpr int part_kpt(int kmax, int km, bool probe) {
    // sized so every (KMAX, key mode) variant stays within 128 VGPRs without spilling
    if (km == kFixed16) {
        if (kmax <= 4) return 4;
        if (kmax <= 8) return 3;
        if (kmax <= 10 && !probe) return 3;  // the exact k = 10 build (C4's product sizing)
        return kmax <= 16 ? 2 : 1;
    }
    // variable-length keys (C3): 4 per thread at k = 8 — 4096-key sub-chunks, placed in windows of
    // the stage (longer per-tile runs per write-out than the 2048 / 3072 keys a stage holds)
    return kmax <= 8 ? 4 : 1;
}

// Packed build entries (PK3): a region holds 8-byte words of three 21-bit positions in the tile
// (bits 0-20, 21-41, 42-62), so the partition writes and the tile build reads 8 B per 3 positions
// instead of 12.  Each tile's run of a sub-chunk is padded to a multiple of 3 in the stage: the
// scan writes a pad value of another tile ((b ^ 1) << tb) into the 0-2 slots past the run, and
// the write-out replaces a pad by the word's first position (setting a bit twice is harmless).
// Region cursors and capacities stay in entries (multiples of 3); fill counts are in words.
constexpr uint32_t kPk3Bits = 21;
__device__ __forceinline__ uint32_t div3(uint32_t x) { return __umulhi(x, 0xAAAAAAABu) >> 1; }

// EXACT: k == KMAX at compile time (no per-seed branches; the seeds' LDS atomics issue together).
template <int KMAX, int KM, bool PROBE, bool EXACT = false, bool PK3 = false>
__global__ void __launch_bounds__(kPartThreads) k_part(KeySet ks, uint64_t n, int k, TileMap tm, PartGeom pg,
                                                       uint32_t* __restrict__ regions, uint32_t* __restrict__ fill,
                                                       uint16_t* __restrict__ pref, uint32_t* __restrict__ ovf,
                                                       uint32_t* __restrict__ ovf_count, ProbeSet ps,
                                                       uint32_t* __restrict__ hw_init) {
    constexpr int KPT = part_kpt(KMAX, KM, PROBE);
    extern __shared__ uint32_t smem[];
    if constexpr (EXACT) k = KMAX;
    const uint32_t B = tm.nbuckets;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint32_t kpt = pg.kps / nt;  // <= KPT
    const uint32_t g = blockIdx.x;
    // cb[b] = entries routed to (g, b) before the current sub-chunk - lbase[b] (the write-out's
    // region position of stage entry e is cb[b] + e)
    uint32_t* cb = smem;               // B
    uint32_t* cnt = cb + B;            // B: the next sub-chunk's per-tile count
    uint32_t* lbase = cnt + B;         // B+1: the current sub-chunk's exclusive scan of its counts
    uint32_t* ws = lbase + B + 1;      // 16
    uint32_t* stage = ws + 16;         // scap
    uint16_t* bkt = reinterpret_cast<uint16_t*>(stage + pg.scap);  // scap (probes)
    const uint32_t lmask = (1u << tm.tb) - 1u;
    uint32_t* const rgn = regions + uint64_t(g) * B * pg.cap;  // this workgroup's regions
    // probes: sub-chunks per 4096-key group (kps is 1024, 2048 or 4096 for probes) and the
    // group-boundary counts pref[g][q][b] (q = 0..nq, b fastest), as the ring partition keeps them
    const uint32_t spg = kGroupKeys / pg.kps, nqs = pg.nq + 1;
    for (uint32_t b = tid; b < B; b += nt) {
        cb[b] = 0;
        cnt[b] = 0;
        lbase[b + 1] = 0;
        if constexpr (PROBE) pref[uint64_t(g) * nqs * B + b] = 0;
    }
    const uint64_t k0 = uint64_t(g) * pg.kpw;
    const uint64_t k1 = min(n, k0 + pg.kpw);
    if constexpr (PROBE) {
        // this workgroup's words of every filter's miss bits start at 0 and its gather words
        // (hw_init) at all ones (as k_part_ring)
        for (uint64_t w = (k0 >> 5) + tid; w < ((k1 + 31) >> 5); w += nt) {
            for (uint32_t f = 0; f < ps.nf; ++f) {
                ps.neg[f * ps.neg_stride + w] = 0u;
                if (hw_init) hw_init[f * ps.neg_stride + w] = ~0u;
            }
        }
        __syncthreads();  // before any spill of this workgroup ORs into neg
    }
    // fixed 16-byte keys: a sub-chunk's keys are loaded one sub-chunk ahead; variable-length keys:
    // their byte offsets are (the key bytes then need one dependent load, not two)
    uint4 kw[KM == kFixed16 ? KPT : 1];
    uint64_t koa[KM == kVar ? KPT : 1], kob[KM == kVar ? KPT : 1];
    const uint64_t kvo0 = KM == kVar ? gld(ks.off0) : 0;
    auto load_keys = [&](uint64_t s0) {
        if constexpr (KM == kFixed16) {
#pragma unroll
            for (int u = 0; u < KPT; ++u) {
                const uint64_t i = min(s0 + u * nt + tid, n - 1);
                kw[u] = ld_stream_nt<kNtKeys>(reinterpret_cast<const uint32_t*>(ks.data) + i * 4);
            }
        } else if constexpr (KM == kVar) {
#pragma unroll
            for (int u = 0; u < KPT; ++u) {
                const uint64_t i = min(s0 + u * nt + tid, n - 1);
                koa[u] = gld(ks.offsets + i);
                kob[u] = gld(ks.offsets + i + 1);
            }
        }
    };
    // a sub-chunk's positions and their ranks in their tiles (counted into cnt), kept in
    // registers until the sub-chunk is placed
    // (ranks, then global slots, are < 2^16 — kps * k + pads, checked by the host — and kept as
    // 16-bit halves: entry e in rk2[e / 2] bits 16 * (e % 2))
    uint32_t pos[KPT * KMAX], rk2[(KPT * KMAX + 1) / 2];
#pragma unroll
    for (int e = 0; e < KPT * KMAX; ++e) pos[e] = 0;
#pragma unroll
    for (int e = 0; e < (KPT * KMAX + 1) / 2; ++e) rk2[e] = 0;
    auto rank_of = [&](int e) { return (rk2[e >> 1] >> (16 * (e & 1))) & 0xFFFFu; };
    auto hash_count = [&](uint64_t s0) {
        const uint64_t s1 = min(k1, s0 + pg.kps);
#pragma unroll
        for (int u = 0; u < KPT; ++u) {
            const uint64_t i = s0 + u * nt + tid;
            auto emit = [&](int s, uint32_t h) {
                const uint32_t p = tile_pos(h, tm);
                pos[u * KMAX + s] = p;
                const uint32_t r = atomicAdd(cnt + (p >> tm.tb), 1u);
                const int e = u * KMAX + s;
                rk2[e >> 1] = (e & 1) ? (rk2[e >> 1] & 0xFFFFu) | (r << 16) : r;
            };
            if (uint32_t(u) < kpt && i < s1) {
                if constexpr (KM == kFixed16)
                    murmur_seeds16<KMAX>(kw[u], k, emit);
                else if constexpr (KM == kVar && KMAX > 0)
                    murmur_seeds_seg<KMAX>(ks.data + (koa[u] - kvo0), uint32_t(kob[u] - koa[u]), k, emit);
                else
                    hash_key<KMAX, KM>(ks, i, k, emit);
            }
        }
    };
    // Exclusive scan of cnt into lbase (lbase[B] = the sub-chunk's total) that also moves cb past
    // the previous sub-chunk: cb[b] += lbase_prev[b + 1] - lbase[b] (= its old value + lbase_prev[b]
    // + its count - lbase[b]); a previous sub-chunk that closed a 4096-key group leaves the
    // routed count cb[b] + lbase_prev[b + 1] in pref.  A thread scans <= 4 tiles (B <= 4096).
    // Ends synced.
    auto padded = [](uint32_t c) { return PK3 ? c + (3u - c % 3u) % 3u : c; };
    auto scan_advance = [&](bool group_end, uint32_t q) {
        const uint32_t per = (B + nt - 1) / nt;
        const uint32_t lo = min(B, tid * per), hi = min(B, lo + per);
        uint32_t sum = 0, prevn[4], cn[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            const uint32_t b = lo + x;
            prevn[x] = 0;
            cn[x] = 0;
            if (b < hi) {
                cn[x] = cnt[b];
                sum += padded(cn[x]);
                prevn[x] = lbase[b + 1];
            }
        }
        uint32_t v = sum;
        const uint32_t lane = tid & 63;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(v, d, 64);
            if (lane >= uint32_t(d)) v += o;
        }
        if (lane == 63) ws[tid >> 6] = v;
        lds_barrier();
        if (tid < 64) {
            const uint32_t nw = nt >> 6;
            uint32_t w = tid < nw ? ws[tid] : 0u;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(w, d, 64);
                if (tid >= uint32_t(d)) w += o;
            }
            if (tid < nw) ws[tid] = w;
        }
        lds_barrier();
        uint32_t run = v - sum + ((tid >> 6) ? ws[(tid >> 6) - 1] : 0u);
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            const uint32_t b = lo + x;
            if (b < hi) {
                const uint32_t c = cb[b] + prevn[x];  // routed before this sub-chunk
                if (PROBE && group_end) pref[(uint64_t(g) * nqs + q) * B + b] = uint16_t(min(c, pg.cap));
                cb[b] = c - run;
                lbase[b] = run;
                run += padded(cn[x]);
            }
        }
        if (tid == nt - 1) lbase[B] = run;
        lds_barrier();
    };
    if (k0 < k1) {
        load_keys(k0);
        lds_barrier();  // cnt cleared
        hash_count(k0);
        if (k0 + pg.kps < k1) load_keys(k0 + pg.kps);
    }
    uint32_t j = 0;
    for (uint64_t s0 = k0; s0 < k1; s0 += pg.kps, ++j) {
        const uint64_t s1 = min(k1, s0 + pg.kps);
        lds_barrier();  // this sub-chunk's counts are complete, the previous write-out is done
        scan_advance(PROBE && j > 0 && (j & (spg - 1)) == 0, j / spg);
        // Place the sub-chunk's entries, sorted by tile, and write them out, in windows of the
        // stage: entry (tile b, rank r) has the global slot gs = lbase[b] + r of the sub-chunk's
        // sorted order; window [e_lo, e_lo + scap) is placed into stage[gs - e_lo], then written
        // out.  A sub-chunk's entries (4096 variable-length keys x 8) may thus exceed the stage:
        // its per-tile runs, and so the region writes, are as long as the sub-chunk's.  Usually
        // one or two windows.  (The key's place in its 4096-key group goes into a probe entry.)
        const uint32_t gkey0 = (j & (spg - 1)) * pg.kps;
        const uint32_t tot = lbase[B];
        const uint32_t S = pg.scap;  // (PK3: a multiple of 3)
#pragma unroll
        for (int u = 0; u < KPT; ++u) {
#pragma unroll
            for (int s = 0; s < KMAX; ++s)
                if (s < k) rk2[(u * KMAX + s) >> 1] += lbase[pos[u * KMAX + s] >> tm.tb] << (16 * ((u * KMAX + s) & 1));  // the global slot
        }
        // the scan's tiles of this thread (pads, count reset)
        const uint32_t sper = (B + nt - 1) / nt, slo = min(B, tid * sper), shi = min(B, slo + sper);
        for (uint32_t e_lo = 0;; e_lo += S) {
            const uint32_t e_hi = min(tot, e_lo + S);
            const bool last = e_hi == tot;
#pragma unroll
            for (int u = 0; u < KPT; ++u) {
                const uint32_t slot_key = u * nt + tid;
                if (uint32_t(u) < kpt && s0 + slot_key < s1) {
#pragma unroll
                    for (int s = 0; s < KMAX; ++s) {
                        if (s < k) {
                            const uint32_t p = pos[u * KMAX + s];
                            const uint32_t slot = rank_of(u * KMAX + s) - e_lo;
                            if (slot < S) {
                                stage[slot] = PROBE ? (((gkey0 + slot_key) << kSlotShift) | (p & lmask)) : p;
                                if constexpr (PROBE) bkt[slot] = uint16_t(p >> tm.tb);
                            }
                        }
                    }
                }
            }
            for (uint32_t b = slo; b < shi; ++b) {
                if constexpr (PK3) {
                    // the run's 0-2 pad slots: a position of another tile ((b ^ 1) << tb)
                    const uint32_t c = cnt[b], l0 = lbase[b];
                    for (uint32_t y = c; y < padded(c); ++y)
                        if (l0 + y - e_lo < S) stage[l0 + y - e_lo] = (b ^ 1u) << tm.tb;
                }
                if (last) cnt[b] = 0;
            }
            lds_barrier();
            // The next sub-chunk is hashed and counted while the last window is written out: the
            // hash's VALU work overlaps the write-out's LDS reads and stores (other waves).
            if (last && s1 < k1) {
                hash_count(s1);
                if (s1 + pg.kps < k1) load_keys(s1 + pg.kps);
            }
            // Lane-parallel write-out: window entry e goes to position cb[b] + e_lo + e of region
            // (g, b).  UW entries per thread per batch: the stage reads, then the cursor reads, are
            // issued before any is consumed (one LDS wait each), and the region offsets are 32-bit
            // within the workgroup's regions (B * cap < 2^32; b < 4096, cap < 2^24: one 24-bit
            // multiply-add).  Positions >= cap overflow (rare).
            const uint32_t nw = e_hi - e_lo;
            // (four per batch when the next sub-chunk's KPT x KMAX positions and ranks already hold
            // 60 registers: C4's k = 10 build, which spills at eight)
            constexpr int UW = KPT * KMAX >= 30 ? 4 : 8;
            if constexpr (PK3) {
                // one 8-byte word (three stage entries of one tile) per thread and batch slot
                uint64_t* const rgn64 = reinterpret_cast<uint64_t*>(regions) + uint64_t(g) * B * (pg.cap / 3);
                const uint32_t capw = pg.cap / 3, totw = nw / 3;
                for (uint32_t w0 = tid; w0 < totw; w0 += nt * UW) {
                    uint32_t v0[UW], v1[UW], v2[UW], b[UW], r[UW];
#pragma unroll
                    for (int u = 0; u < UW; ++u) {
                        const uint32_t e = 3 * min(w0 + u * nt, totw - 1);
                        v0[u] = stage[e];
                        v1[u] = stage[e + 1];
                        v2[u] = stage[e + 2];
                        b[u] = v0[u] >> tm.tb;
                    }
#pragma unroll
                    for (int u = 0; u < UW; ++u) r[u] = cb[b[u]] + e_lo + 3 * (w0 + u * nt);
                    uint32_t over = 0;
#pragma unroll
                    for (int u = 0; u < UW; ++u) {
                        const bool live = w0 + u * nt < totw;
                        const uint32_t a = v0[u] & lmask;
                        const uint32_t c1 = (v1[u] >> tm.tb) == b[u] ? (v1[u] & lmask) : a;
                        const uint32_t c2 = (v2[u] >> tm.tb) == b[u] ? (v2[u] & lmask) : a;
                        const uint64_t word = uint64_t(a) | (uint64_t(c1) << kPk3Bits) | (uint64_t(c2) << (2 * kPk3Bits));
                        if (live && r[u] < pg.cap) rgn64[__umul24(b[u], capw) + div3(r[u])] = word;
                        over |= uint32_t(live && r[u] >= pg.cap) << u;
                    }
                    if (over) {  // region overflow: heavy key duplication only
#pragma unroll
                        for (int u = 0; u < UW; ++u) {
                            if ((over >> u) & 1u) {
                                const uint32_t x = atomicAdd(ovf_count, 3u);
                                ovf[x] = v0[u];
                                ovf[x + 1] = (v1[u] >> tm.tb) == b[u] ? v1[u] : v0[u];
                                ovf[x + 2] = (v2[u] >> tm.tb) == b[u] ? v2[u] : v0[u];
                            }
                        }
                    }
                }
            } else {
                for (uint32_t e0 = tid; e0 < nw; e0 += nt * UW) {
                    uint32_t v[UW], b[UW], r[UW];
#pragma unroll
                    for (int u = 0; u < UW; ++u) {
                        const uint32_t e = min(e0 + u * nt, nw - 1);
                        v[u] = stage[e];
                        b[u] = PROBE ? uint32_t(bkt[e]) : (v[u] >> tm.tb);
                    }
#pragma unroll
                    for (int u = 0; u < UW; ++u) r[u] = cb[b[u]] + e_lo + e0 + u * nt;
                    uint32_t over = 0;
#pragma unroll
                    for (int u = 0; u < UW; ++u) {
                        const bool live = e0 + u * nt < nw;
                        if (live && r[u] < pg.cap) rgn[__umul24(b[u], pg.cap) + r[u]] = v[u];
                        over |= uint32_t(live && r[u] >= pg.cap) << u;
                    }
                    if (over) {  // region overflow: heavy key duplication only
#pragma unroll
                        for (int u = 0; u < UW; ++u) {
                            if ((over >> u) & 1u) {
                                if constexpr (PROBE)
                                    spill_probe(ps, pos_to_bit((b[u] << tm.tb) | (v[u] & lmask), tm),
                                                s0 + ((v[u] >> kSlotShift) & (pg.kps - 1)));
                                else
                                    ovf[atomicAdd(ovf_count, 1u)] = v[u];
                            }
                        }
                    }
                }
            }
            if (last) break;
            lds_barrier();  // the window's stage reads are done before the next window is placed
        }
    }
    lds_barrier();
    for (uint32_t b = tid; b < B; b += nt) {
        const uint32_t t = min(cb[b] + lbase[b + 1], pg.cap);
        fill[uint64_t(b) * pg.G + g] = PK3 ? t / 3 : t;
        if constexpr (PROBE)  // the open last group and any the workgroup did not reach
            for (uint32_t q = (j + spg - 1) / spg; q <= pg.nq; ++q) pref[(uint64_t(g) * nqs + q) * B + b] = uint16_t(t);
    }
}

// Copy nw words of the bitmap starting at word w0 into LDS (zero-filling up to W), with every
// thread's loads issued before any is consumed.
__device__ __forceinline__ void load_tile(uint32_t* tile, const uint32_t* __restrict__ bitmap, uint64_t w0,
                                          uint32_t nw, uint32_t W) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    if ((w0 & 3) == 0 && nw == W) {
        // loads are unconditional (clamped index) so the batch stays in registers
        const uint4* src = reinterpret_cast<const uint4*>(bitmap + w0);
        const uint32_t W4 = W / 4;
        for (uint32_t q0 = tid; q0 < W4; q0 += nt * 8) {
            uint4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = ld_stream_nt<kNtTileLoad>(reinterpret_cast<const uint32_t*>(src + min(q0 + u * nt, W4 - 1)));
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (q0 + u * nt < W4) reinterpret_cast<uint4*>(tile)[q0 + u * nt] = v[u];
        }
    } else {
        for (uint32_t w = tid; w < W; w += nt) tile[w] = w < nw ? bitmap[w0 + w] : 0u;
    }
}

__device__ __forceinline__ void store_tile(const uint32_t* tile, uint32_t* __restrict__ bitmap, uint64_t w0,
                                           uint32_t nw) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    if ((w0 & 3) == 0 && (nw & 3) == 0) {
        uint4* dst = reinterpret_cast<uint4*>(bitmap + w0);
        for (uint32_t q = tid; q < nw / 4; q += nt) st_stream<kNtTileStore>(reinterpret_cast<uint32_t*>(dst + q), reinterpret_cast<const uint4*>(tile)[q]);
    } else {
        for (uint32_t w = tid; w < nw; w += nt) bitmap[w0 + w] = tile[w];
    }
}

// OR the in-fill entries of a 4-entry piece into the LDS tile.
__device__ __forceinline__ void or_bits4(uint32_t* tile, uint4 v, uint32_t e, uint32_t f, uint32_t lmask) {
    const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t p = vv[q] & lmask;
        if (e + q < f) atomicOr(tile + (p >> 5), 1u << (p & 31));
    }
}

// OR the in-fill words of a 16-byte piece of packed (PK3) words into the LDS tile: word e
// (positions bits 0-20, 21-41, 42-62) and, when e + 1 < f, word e + 1.
__device__ __forceinline__ void or_bits_pk3(uint32_t* tile, uint4 v, uint32_t e, uint32_t f, uint32_t lmask) {
    const uint32_t lo[2] = {v.x, v.z}, hi[2] = {v.y, v.w};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        if (e + q < f) {
            const uint32_t p0 = lo[q] & lmask;
            const uint32_t p1 = __builtin_amdgcn_alignbit(hi[q], lo[q], kPk3Bits) & lmask;
            const uint32_t p2 = (hi[q] >> (2 * kPk3Bits - 32)) & lmask;
            atomicOr(tile + (p0 >> 5), 1u << (p0 & 31));
            atomicOr(tile + (p1 >> 5), 1u << (p1 & 31));
            atomicOr(tile + (p2 >> 5), 1u << (p2 & 31));
        }
    }
}

// ------------------------------------------------------------------ build: tiles
// One workgroup per tile.  A wave (64 lanes x 16-byte loads = 256 entries, or 128 packed words)
// covers one region per step and keeps kTileBuildRegionsInFlight regions of loads in flight.
// PK3: regions of packed words (k_part's PK3), `fill` in words, region stride cap / 3 words.
template <bool PK3>
__global__ void __launch_bounds__(1024) k_tile_build(TileMap tm, PartGeom pg, const uint32_t* __restrict__ regions,
                                                     const uint32_t* __restrict__ fill, uint32_t* __restrict__ bitmap,
                                                     int pristine) {
    extern __shared__ uint32_t smem[];
    // cap in 4-byte units: entries, or the packed words' dwords
    const uint32_t B = tm.nbuckets, G = pg.G, cap = PK3 ? 2 * (pg.cap / 3) : pg.cap;
    constexpr uint32_t PER = PK3 ? 2 : 4;  // fill units (entries / words) per 16-byte load
    auto or16 = [&](uint32_t* t, uint4 v, uint32_t e, uint32_t f, uint32_t lm) {
        if constexpr (PK3) or_bits_pk3(t, v, e, f, lm);
        else or_bits4(t, v, e, f, lm);
    };
    const uint32_t b = blockIdx.x;
    const uint32_t W = 1u << (tm.tb - 5);
    uint32_t* tile = smem;       // W
    uint32_t* fills = tile + W;  // G
    const uint64_t w0 = tile_word0(b, tm);
    const uint32_t nw = uint32_t(min<uint64_t>(W, tm.total_words - w0));
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    for (uint32_t q = tid; q < G; q += nt) fills[q] = fill[uint64_t(b) * G + q];
    if (pristine) {
        for (uint32_t q = tid; q < W / 4; q += nt) reinterpret_cast<uint4*>(tile)[q] = make_uint4(0, 0, 0, 0);
    } else {
        load_tile(tile, bitmap, w0, nw, W);
    }
    lds_barrier();
    const uint32_t lane = tid & 63, wave = tid >> 6, nwaves = nt >> 6;
    const uint32_t lmask = (1u << tm.tb) - 1u;
    constexpr int U = kTileBuildRegionsInFlight;
    if (cap <= 256) {
        // every region fits one 256-entry chunk (C2: ~230 entries): U regions in flight per wave
        for (uint32_t g0 = wave; g0 < G; g0 += nwaves * U) {
            uint4 v[U];
            uint32_t f[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t q = g0 + u * nwaves;
                f[u] = q < G ? fills[q] : 0u;
                // unconditional loads, clamped to the filled part (idle lanes re-read its last line)
                const uint32_t lc = min(lane, (max(f[u], 1u) - 1) / PER);
                v[u] = ld_stream_nt<kNtLoad>(regions + region_id(min(q, G - 1), b, G, B) * cap + lc * 4);
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (lane * PER < f[u]) or16(tile, v[u], lane * PER, f[u], lmask);
        }
    } else {
        // regions of many chunks (C4: ~2,850 entries, C3: ~760): the wave walks the (region,
        // chunk) sequence of its regions with U chunks in flight — one region's chunk after
        // another, so a long region does not leave the wave with one load in flight at a time.
        // The walk is wave-uniform (fills are in LDS).
        uint32_t q = wave, c = 0;  // next chunk to issue: region q, entries [256c, 256c + 256)
        while (q < G) {
            uint4 v[U];
            uint32_t f[U], e[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                while (q < G && c * 64 * PER >= fills[q]) {
                    q += nwaves;
                    c = 0;
                }
                const bool live = q < G;
                f[u] = live ? fills[q] : 0u;
                e[u] = (c * 64 + lane) * PER;
                const uint32_t qq = live ? q : G - 1, fq = live ? f[u] : 1u;
                // clamped: idle lanes re-read a filled line
                const uint32_t ec = min(e[u] / PER, (fq - 1) / PER) * 4;
                v[u] = ld_stream_nt<kNtLoad>(regions + region_id(qq, b, G, B) * cap + ec);
                if (live) ++c;
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (e[u] < f[u]) or16(tile, v[u], e[u], f[u], lmask);
        }
    }
    lds_barrier();
    store_tile(tile, bitmap, w0, nw);
}

// `reset`: the other of the handle's two overflow counters (the previous build's), zeroed here
// for the next build, so no memset launch precedes a build.
__global__ void __launch_bounds__(256) k_ovf_build(TileMap tm, const uint32_t* __restrict__ ovf,
                                                   const uint32_t* __restrict__ ovf_count, uint32_t* __restrict__ bitmap,
                                                   uint32_t* __restrict__ reset) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *reset = 0u;
    const uint32_t cnt = *ovf_count;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
        const uint64_t bit = pos_to_bit(ovf[i], tm);
        atomicOr(bitmap + (bit >> 5), 1u << (bit & 31));
    }
}

// ------------------------------------------------------------------ probe: tiles
// Result bits R: one 32-bit word per 32-entry word of a region, bit (8t + l) = entry 4l + t
// (l = the entry's 16-byte piece of the word, t = its place in the piece): lane l of a word's
// 8 lanes holds entries 4l..4l+3, so the word's result is the OR of the lanes' bits t << (8t + l).
// One workgroup per tile.  Region words are read 8 per wave instruction: lane = one 16-byte
// piece of a word, so an instruction reads 1 KiB contiguously (words are consecutive within a
// region), U instructions in flight per wave.  Each lane tests its 4 entries in the LDS tile.
// TAB = 2 (the LDS budget allows it): a per-word table gives word c's global index
// wo = region * (cap / 32) + word-in-region — the region word's address / 32 AND its result
// word's index — so a load needs one LDS read and the wave's U loads issue back to back.  TAB = 1
// (4 B per word do not fit, 2 B do: C3's 4096 tiles, C5's 33M-key pipelines): a u16 per word
// holds its region and word-in-region (region << wsh | word), again one LDS read, the index then
// two 24-bit multiply-adds.  TAB = 0: the word's region comes from a binary search over the word
// prefix.  The test does not mask the entries past a region's fill in its last word: the gather
// reads only the filled ones (ring_kernels.hpp), and a stale entry's tile word is in the tile.
// A lane's 4 result bits go to bits 8t + l of the word's result in registers (no ballots): the
// word's 8 lanes OR their pieces with three DPP moves and its first lane stores it.
template <bool NT, int TAB, int U = kTileProbeWordsInFlight>
__device__ __forceinline__ void tile_probe_body(uint32_t* smem, uint32_t b, const TileMap& tm, const PartGeom& pg,
                                                const uint32_t* __restrict__ regions, const uint32_t* __restrict__ fill,
                                                const uint32_t* __restrict__ bitmap, uint32_t* __restrict__ R) {
    const uint32_t B = tm.nbuckets, G = pg.G, cap = pg.cap, wpr = cap / 32;
    const uint32_t wsh = 32u - __builtin_clz(max(wpr, 2u) - 1u);  // TAB 1: bits of a word-in-region
    const uint32_t W = 1u << (tm.tb - 5);
    uint32_t* tile = smem;          // W
    uint32_t* fills = tile + W;     // G
    uint32_t* wpre = fills + G;     // G+1
    uint32_t* ws = wpre + G + 1;    // 16
    uint32_t* wo = ws + 16;                               // G*wpr (TAB 2)
    uint16_t* wq = reinterpret_cast<uint16_t*>(ws + 16);  // G*wpr (TAB 1)
    const uint64_t w0 = tile_word0(b, tm);
    const uint32_t nw = uint32_t(min<uint64_t>(W, tm.total_words - w0));
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    // The region fills are loaded (and waited for) first; then the bitmap tile goes global -> LDS by
    // LDS-DMA while the word scan and the per-word table are built (no global load in between,
    // which would wait for the DMA too), and the stream starts once the DMA has landed.
    // (whole 1 KiB pieces only: tiles of 2^10..2^12 positions, W = 32..128 words, take load_tile)
    const bool dma = PBF_TILE_DMA && (w0 & 3) == 0 && nw == W && W % 256 == 0;
    if (dma) {
        for (uint32_t q = tid; q < G; q += nt) fills[q] = (fill[uint64_t(b) * G + q] + 31) >> 5;  // words
        // (waits for the fill loads only)
        const uint32_t lane = tid & 63, wave = tid >> 6, nwaves = nt >> 6;
        for (uint32_t c = wave; c < W / 256; c += nwaves)  // 1 KiB per wave instruction
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(bitmap + w0 + c * 256 + lane * 4),
                (__attribute__((address_space(3))) void*)(tile + c * 256), 16, 0, 0);
    } else {
        for (uint32_t q = tid; q < G; q += nt) fills[q] = (fill[uint64_t(b) * G + q] + 31) >> 5;  // words
        load_tile(tile, bitmap, w0, nw, W);
    }
    lds_barrier();
    block_exclusive_scan(fills, wpre, G, ws);
    const uint32_t lane = tid & 63, wave = tid >> 6, nwaves = nt >> 6;
    const uint32_t l = lane & 7, wsub = lane >> 3;  // piece of the word, word of the instruction
    const uint32_t stride = nwaves * 8;
    // an entry's tile word: one bit-field extract of bits [5, tb); its bit: one more (the
    // hardware takes the offset's low 5 bits, so no mask)
    const uint32_t wbits = tm.tb - 5;
    auto bit = [&](uint32_t x) { return __builtin_amdgcn_ubfe(tile[__builtin_amdgcn_ubfe(x, 5u, wbits)], x, 1u); };
    // the words [c_lo, c_hi) of the tile's regions; TAB 1's table holds word c at c - c_lo
    auto stream = [&](uint32_t c_lo, uint32_t c_hi) {
        for (uint32_t c0 = c_lo + wave * 8; c0 < c_hi; c0 += stride * U) {
            uint4 v[U];
            uint32_t oo[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t cc = min(c0 + u * stride + wsub, c_hi - 1);  // unconditional loads
                if constexpr (TAB == 2) {
                    oo[u] = wo[cc];
                } else if constexpr (TAB == 1) {
                    const uint32_t e = wq[cc - c_lo];
                    oo[u] = __umul24(__umul24(e >> wsh, B) + b, wpr) + (e & ((1u << wsh) - 1u));
                } else {
                    const uint32_t qq = bucket_of(wpre, G, cc);
                    oo[u] = uint32_t(region_id(qq, b, G, B)) * wpr + (cc - wpre[qq]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ld_stream_nt<NT>(regions + uint64_t(oo[u]) * 32 + l * 4);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint32_t r = (bit(v[u].x) | (bit(v[u].y) << 8) | (bit(v[u].z) << 16) | (bit(v[u].w) << 24)) << l;
                // OR over the word's 8 lanes: swap neighbours, pairs, then the two quads
                r |= uint32_t(__builtin_amdgcn_mov_dpp(int(r), 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
                r |= uint32_t(__builtin_amdgcn_mov_dpp(int(r), 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
                r |= uint32_t(__builtin_amdgcn_mov_dpp(int(r), 0x141, 0xF, 0xF, false));  // row_half_mirror
                if (l == 0 && c0 + u * stride + wsub < c_hi) R[oo[u]] = r;
            }
        }
    };
    if constexpr (TAB == 1) {
        // the table takes the regions in chunks whose words fit it (pg.tabw words; every region's
        // <= wpr words fit): a batch with more regions per tile than the LDS holds a table for
        // (more partition workgroups, e.g. C5's 100M keys in one pipeline) still reads one LDS
        // word per region word, at one more barrier pair per chunk
        const uint32_t tabw = pg.tabw ? pg.tabw : 0xFFFFFFFFu;
        for (uint32_t q0 = 0; q0 < G;) {
            const uint32_t c_lo = wpre[q0];
            const uint32_t q1 = tabw >= wpre[G] - c_lo ? G : max(q0 + 1, bucket_of(wpre, G + 1, c_lo + tabw));
            for (uint32_t q = q0 + tid; q < q1; q += nt)
                for (uint32_t c = wpre[q]; c < wpre[q + 1]; ++c) wq[c - c_lo] = uint16_t((q << wsh) | (c - wpre[q]));
            if (q0 == 0 && dma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's tile pieces landed
            lds_barrier();
            stream(c_lo, wpre[q1]);
            q0 = q1;
            if (q0 < G) lds_barrier();  // every wave is done with this chunk's table
        }
    } else {
        if constexpr (TAB == 2) {
            for (uint32_t q = tid; q < G; q += nt) {
                const uint32_t base = uint32_t(region_id(q, b, G, B)) * wpr;
                for (uint32_t c = wpre[q]; c < wpre[q + 1]; ++c) wo[c] = base + (c - wpre[q]);
            }
        }
        if (dma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's tile pieces landed
        lds_barrier();
        stream(0, wpre[G]);
    }
}

template <int TAB>
__global__ void __launch_bounds__(1024) k_tile_probe(TileMap tm, PartGeom pg, const uint32_t* __restrict__ regions,
                                                     const uint32_t* __restrict__ fill,
                                                     const uint32_t* __restrict__ bitmap, uint32_t* __restrict__ R) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    tile_probe_body<kNtLoad, TAB>(smem, blockIdx.x, tm, pg, regions, fill, bitmap, R);
}

// The tile test of a multi-filter probe in ONE launch: workgroup (tile b, filter f) for every
// filter of the set.  Workgroups are dealt round-robin over the 8 XCDs in dispatch order (speed
// only, never correctness), so block x = ((b / 8) * nf + f) * 8 + b % 8 puts the nf
// workgroups of tile b on one XCD, dispatched together: they stream the same region entries
// (g, b), g = 0..G-1, in the same order, and all but the first read them from that XCD's L2.
template <int TAB>
__global__ void __launch_bounds__(1024) k_tile_probe_set(TileMap tm, PartGeom pg, const uint32_t* __restrict__ regions,
                                                         const uint32_t* __restrict__ fill, ProbeSet ps,
                                                         uint32_t* __restrict__ R, uint64_t r_stride) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t x = blockIdx.x, nf = ps.nf;
    const uint32_t t = x >> 3;
    const uint32_t f = t % nf;
    const uint32_t b = (t / nf) * 8 + (x & 7);
    if (b >= tm.nbuckets) return;
    // the set's other workgroups of tile b read the same lines: temporal loads keep them in L2
    tile_probe_body<false, TAB, kTileProbeSetWordsInFlight>(smem, b, tm, pg, regions, fill, ps.bm[f], R + f * r_stride);
}

// hw (ANDed gather words, one per 32 keys) → the LSB-first hit masks of n keys, for every filter
// of a set in one launch (grid y = filter; filter f's words at hw + f * stride).
struct HitMasks {
    uint8_t* hm[kMaxProbeSet];
};
__global__ void k_hw_to_hitmask(const uint32_t* __restrict__ hw, uint64_t stride, uint64_t n, HitMasks out) {
    const uint64_t nw = (n + 31) / 32;
    const uint32_t* src = hw + uint64_t(blockIdx.y) * stride;
    uint8_t* hitmask = out.hm[blockIdx.y];
    for (uint64_t w = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; w < nw; w += uint64_t(gridDim.x) * blockDim.x) {
        const uint64_t key0 = w * 32;
        const uint32_t bits = src[w];
        const uint64_t nbt = min<uint64_t>(4, (n - key0 + 7) / 8);
        if (nbt == 4 && (reinterpret_cast<uintptr_t>(hitmask + key0 / 8) & 3) == 0)
            *reinterpret_cast<uint32_t*>(hitmask + key0 / 8) = bits;
        else
            for (uint64_t q = 0; q < nbt; ++q) hitmask[key0 / 8 + q] = uint8_t(bits >> (8 * q));
    }
}

}  // namespace pbf
