// Ring-buffer partition for the LDS-tiled build / probe (reference semantics:
// src/bloom_filter.py:60-74), gfx950.  Used when a bitmap has <= 1024 tiles and a 1024-key
// sub-chunk puts only a few positions into each tile (plan_for in pebblebloom.hip), e.g. C2:
// m = 2^30, B = 1024 tiles of 2^20 bits.
//
// Why: the counting-sort partition (k_part) appends each sub-chunk's per-tile run (~18 entries,
// ~72 B at C2) to its region with lane-parallel dword stores.  A run starts and ends inside
// 64-B segments, and the fabric sees every piece as its own write request (measured: 7.0M write
// requests, half of them 32-B partials, for 240 MB of entries).  Here every tile keeps a small
// FIFO ring in LDS; a sub-chunk appends its positions to the rings (one LDS atomic + one LDS
// store per position, no scan, no stage), and a flush phase writes every complete 16-entry group
// with ONE wave store instruction (4 lanes x 16 B), so each region line leaves as whole 64-B
// requests.
//
//   ring      32 entries per tile (RC), groups of GS = 16.  head = entries flushed (= the region
//             write cursor, a multiple of GS), tail = entries appended; packed as the 16-bit
//             halves of one u32 per tile.  Entry e of tile b sits at ring[b*RC + ((e + stagger(b))
//             % RC)] and lands at region position e.
//   sub-chunk kps keys (<= 1024, one per thread).  The host picks the geometry so a tile receives
//             <= GS/2 positions per sub-chunk on average; a position that would overrun the ring
//             (or the region capacity) leaves the stream into an LDS spill buffer, handled once at
//             the end of the kernel (build: copied to the overflow list; probe: tested against the
//             bitmap, a miss sets the key's bit in `neg`); past the buffer's capacity it is
//             handled in place.  (Two 1024-key units per flush — half the barriers and flush
//             scans per key, ~0.2% of positions spilled — measured slower: C2 build 0.199 ->
//             0.212 ms, probe neutral, C5 9.35 -> 9.55 ms; profiles/r03/s7.)
//   probe     entry = key-in-group << 20 | position-in-tile, key-in-group = (j & 3) << 10 |
//             thread (j = sub-chunk; a group = 4096 keys = 4 sub-chunks of 1024).  pref[g][q][b] = in-region entries
//             of (g, b) before group q (b fastest, so a wave's stores of 64 tiles are one
//             contiguous 256-B run), so k_gather_ring finds an entry's group from its region
//             position.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tiled_kernels.hpp"

namespace pbf {

constexpr uint32_t kRingKeysPerSub = 1024;  // = threads; the thread field is 10 bits
constexpr uint32_t kRingEntries = 32;       // RC: LDS ring entries per tile (64-B groups of 16)
static_assert(kSlotShift == 20 && kRingKeysPerSub == 1024 && kGroupKeys == 4 * kRingKeysPerSub,
              "probe entry = ((j & 3) << 10 | thread) << 20 | position");
// Key sub-chunks loaded per batch, one batch ahead: 2 measured best with the non-temporal streams
// (C2 A/B over 1/2/3/4/8: profiles/r01/s11/ab.txt)
constexpr int kRingPrefetch = 2;
constexpr uint32_t kRingDescPerWave = 128;  // flush descriptors per wave (64 tiles x <= 2 groups)

// LDS layout of k_part_ring (u32 words): head|tail per tile [B], flush descriptors [16 waves x
// 128], one dump word (appends that left the stream write there), the spill count, then the rings
// [B x RC], 16-B aligned, then the spill buffer (probe: 2 words per entry, build: 1).
__host__ __device__ constexpr uint32_t ring_lds_base(uint32_t B) { return (B + 16 * kRingDescPerWave + 2 + 3) & ~3u; }
__host__ __device__ constexpr uint32_t ring_lds_words(uint32_t B) { return ring_lds_base(B) + B * kRingEntries; }

// Entry e of tile b sits at ring[b * RC + ((e + ring_stagger(b)) % RC)]: the appends of a
// sub-chunk store to slots e that are close together in every tile (the tails advance alike), so
// without the stagger their LDS banks ((b * RC + e) mod 32 = e mod 32) collide.  A multiple of 4,
// so a flush group (4 entries from e, e a multiple of 4) stays one aligned 16-byte read.
// (C2 0.680-0.681 vs 0.685 ms/step, C5 6.99 vs 7.20 ms: profiles/r04/s8/stagger_*.)
// (A 32-way stagger, b mod 32, with the flush reading 4 single entries: C2 0.700 vs 0.681-0.686,
// C5 7.39 vs 6.98 ms; profiles/r04/s8/st32_*.)
__device__ __forceinline__ uint32_t ring_stagger(uint32_t b) { return (b & 7u) << 2; }
__device__ __forceinline__ uint4 ring_group4(const uint32_t* r, uint32_t e, uint32_t rmask) {
    return *reinterpret_cast<const uint4*>(r + (e & rmask));
}

// Tile position of a hash when m is a power of two <= 2^32 (POW2) or in general.
template <bool POW2>
__device__ __forceinline__ uint32_t ring_pos(uint32_t h, const TileMap& tm) {
    if constexpr (POW2) return h & tm.im.mask;
    return tile_pos(h, tm);
}

// Keys are loaded kRingPrefetch sub-chunks at a time, one batch ahead.  On gfx950 vmcnt also
// counts stores, so the wait for a key load also waits for every flush store issued before it;
// batching pays that wait once per kRingPrefetch sub-chunks instead of once per sub-chunk.
// EXACT: k == KMAX is known at compile time, so the per-seed `s < k` tests vanish and the k LDS
// atomics of a key issue back to back.
// The host keeps cap <= 32768, so a tail never passes cap + one sub-chunk's appends (the flush
// clamps it every sub-chunk) and head / tail fit the 16-bit halves of one u32: the append is a
// 32-bit LDS atomic spread over all 32 banks of a lane group.
template <int KMAX, int KM, bool PROBE, bool POW2, bool EXACT>
__global__ void __launch_bounds__(1024) k_part_ring(KeySet ks, uint64_t n, int k, TileMap tm, PartGeom pg,
                                                    uint32_t* __restrict__ regions, uint32_t* __restrict__ fill,
                                                    uint16_t* __restrict__ pref, uint32_t* __restrict__ ovf,
                                                    uint32_t* __restrict__ ovf_count, ProbeSet ps,
                                                    uint32_t* __restrict__ hw_init) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    if constexpr (EXACT) k = KMAX;
    constexpr uint32_t RC = kRingEntries, GS = RC / 2, rmask = RC - 1;
    constexpr uint32_t SW = PROBE ? 2 : 1;  // spill-buffer words per entry
    const uint32_t B = tm.nbuckets;
    const uint32_t shift = tm.tb;
    const uint32_t kps = pg.kps;  // keys per sub-chunk (<= 1024 threads)
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint32_t lane = tid & 63, wave = tid >> 6;
    const uint32_t g = blockIdx.x;
    const uint32_t cap = pg.cap;
    const uint32_t lmask = (1u << tm.tb) - 1u;
    // ht[b] = head << 16 | tail: one LDS atomic add appends a position and returns the tile's
    // flush cursor with its slot (no separate head read per position)
    uint32_t* const ht = smem;
    uint32_t* const desc = smem + B;                  // 16 waves x 128 group descriptors
    const uint32_t dump = B + 16 * kRingDescPerWave;  // word index of the dump slot
    uint32_t* const nspill = smem + dump + 1;
    uint32_t* const ring = smem + ring_lds_base(B);   // B * RC, 16-B aligned
    uint32_t* const sbuf = ring + B * RC;             // pg.spill_cap entries
    // this workgroup's regions; an entry's offset in them fits 32 bits (B * cap < 2^32), and
    // tb < 4096, cap < 2^20 make it one 24-bit multiply-add
    uint32_t* const rgn = regions + uint64_t(g) * B * cap;
    auto region_at = [&](uint32_t tb, uint32_t e) { return rgn + (__umul24(tb, cap) + e); };
    const uint32_t nqs = pg.nq + 1;  // pref entries per (g, b)
    for (uint32_t b = tid; b < B; b += nt) {
        ht[b] = 0;
        if constexpr (PROBE) pref[uint64_t(g) * nqs * B + b] = 0;
    }
    if (tid == 0) *nspill = 0;
    const uint64_t k0 = uint64_t(g) * pg.kpw;
    const uint64_t k1 = min(n, k0 + pg.kpw);
    if constexpr (PROBE) {
        // this workgroup's words of every filter's miss bits (neg) start at 0 and, when the
        // gather ANDs into words, every filter's gather words (hw_init) at all ones: no memsets
        for (uint64_t w = (k0 >> 5) + tid; w < ((k1 + 31) >> 5); w += nt) {
            for (uint32_t f = 0; f < ps.nf; ++f) {
                ps.neg[f * ps.neg_stride + w] = 0u;
                if (hw_init) hw_init[f * ps.neg_stride + w] = ~0u;
            }
        }
        __syncthreads();  // before any spill of this workgroup ORs into neg
    }
    constexpr int P = kRingPrefetch;
    constexpr bool F16 = KM == kFixed16;
    uint4 kw[F16 ? P : 1];
    auto load_batch = [&](uint64_t c0) {
        if constexpr (F16) {
#pragma unroll
            for (int u = 0; u < P; ++u) {
                const uint64_t i = c0 + uint64_t(u) * kps + tid;
                kw[u] = ld_stream_nt<kNtKeys>(reinterpret_cast<const uint32_t*>(ks.data) + min(i, n - 1) * 4);
            }
        }
    };
    // A position that leaves the stream (its ring or region is full): into the spill buffer, or
    // past its capacity handled here (build: overflow list; probe: tested now).
    auto spill_one = [&](uint32_t p, uint64_t i) {
        const uint32_t x = atomicAdd(nspill, 1u);
        if (x < pg.spill_cap) {
            sbuf[x * SW] = p;
            if constexpr (PROBE) sbuf[x * SW + 1] = uint32_t(i - k0);
        } else if constexpr (PROBE) {
            spill_probe(ps, pos_to_bit(p, tm), i);
        } else {
            ovf[atomicAdd(ovf_count, 1u)] = p;
        }
    };
    load_batch(k0);
    uint32_t j = 0;  // sub-chunks done
    for (uint64_t c0 = k0; c0 < k1; c0 += uint64_t(P) * kps) {
        uint4 cw[F16 ? P : 1];
        if constexpr (F16) {
#pragma unroll
            for (int u = 0; u < P; ++u) cw[u] = kw[u];
        }
        if (c0 + uint64_t(P) * kps < k1) load_batch(c0 + uint64_t(P) * kps);
#pragma unroll
        for (int u = 0; u < P; ++u, ++j) {
            const uint64_t s0 = c0 + uint64_t(u) * kps;
            if (s0 >= k1) break;
            const uint64_t i = s0 + tid;
            const bool live = tid < kps && i < k1;
            uint32_t pos[KMAX], slot[KMAX], hd[KMAX];
            // hash before the barrier: a wave done with its share of the previous flush hashes
            // while the others still flush
            if (live) {
                auto emit = [&](int s, uint32_t h) { pos[s] = ring_pos<POW2>(h, tm); };
                if constexpr (F16)
                    murmur_seeds16<KMAX>(cw[u], k, emit);
                else
                    hash_key<KMAX, KM>(ks, i, k, emit);
            }
            lds_barrier();  // previous flush done: head / tail stable, rings free
            if (live) {
#pragma unroll
                for (int s = 0; s < KMAX; ++s) {
                    if (s < k) {
                        const uint32_t v = atomicAdd(ht + (pos[s] >> shift), 1u);
                        slot[s] = v & 0xFFFFu;
                        hd[s] = v >> 16;
                    }
                }
                uint32_t spill = 0;  // positions that overrun their tile's ring or region
                const uint32_t tag = PROBE ? (((j & 3u) << 30) | (tid << kSlotShift)) : 0u;
#pragma unroll
                for (int s = 0; s < KMAX; ++s) {
                    if (s < k) {
                        const uint32_t p = pos[s], b = p >> shift, e = slot[s];
                        const bool ok = e - hd[s] < RC && e < cap;
                        const uint32_t val = PROBE ? (tag | (p & lmask)) : p;
                        // every lane stores (a position that left the stream into the dump
                        // word): no per-seed exec-mask branch (build 0.196 -> 0.192 ms on C2)
                        smem[ok ? ring_lds_base(B) + b * RC + ((e + ring_stagger(b)) & rmask) : dump] = val;
                        spill |= uint32_t(!ok) << s;
                    }
                }
                if (spill) {  // rare: heavy key duplication
#pragma unroll
                    for (int s = 0; s < KMAX; ++s)
                        if ((spill >> s) & 1u) spill_one(pos[s], i);
                }
            }
            lds_barrier();
            // Flush: each wave owns 64 tiles per pass.  A lane's tile has 0..2 whole groups;
            // the wave lists them (descriptor = tile | region position << 12) and writes
            // 64/(GS/4) groups per store instruction, GS/4 lanes x 16 B per group, each whole.
            uint32_t* wd = desc + wave * kRingDescPerWave;
            constexpr uint32_t lpg = GS / 4;    // lanes per group
            constexpr uint32_t gpi = 64 / lpg;  // groups per store instruction
            for (uint32_t b0 = wave * 64; b0 < B; b0 += nt) {
                const uint32_t b = b0 + lane;
                uint32_t ng = 0, h = 0, t = 0;
                if (b < B) {
                    const uint32_t v = ht[b];
                    h = v >> 16;
                    t = min(v & 0xFFFFu, min(h + RC, cap));  // positions past these left the stream
                    ng = (t - h) / GS;
                }
                const uint64_t m1 = __ballot(ng >= 1), m2 = __ballot(ng >= 2);
                // descriptors of lower lanes: masked bit counts (v_mbcnt), accumulated over m1, m2
                const uint32_t at = __builtin_amdgcn_mbcnt_hi(
                    uint32_t(m2 >> 32), __builtin_amdgcn_mbcnt_lo(
                                            uint32_t(m2), __builtin_amdgcn_mbcnt_hi(
                                                              uint32_t(m1 >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m1), 0u))));
                const uint32_t total = __popcll(m1) + __popcll(m2);
                if (ng >= 1) wd[at] = b | (h << 12);
                if (ng >= 2) wd[at + 1] = b | ((h + GS) << 12);
                __builtin_amdgcn_wave_barrier();
                for (uint32_t c = 0; c < total; c += gpi) {
                    const uint32_t gi = c + lane / lpg, q = lane % lpg;
                    if (gi < total) {
                        const uint32_t d = wd[gi];
                        const uint32_t tb = d & 0xFFFu;
                        const uint32_t e = (d >> 12) + q * 4;  // region position
                        const uint4 v = ring_group4(ring + tb * RC, e + ring_stagger(tb), rmask);
                        st_stream<PROBE ? kNtProbePart : kNtBuildPart>(region_at(tb, e), v);
                    }
                }
                __builtin_amdgcn_wave_barrier();
                if (b < B) {
                    ht[b] = ((h + ng * GS) << 16) | t;
                    if constexpr (PROBE)
                        if (((j + 1) & 3) == 0) pref[(uint64_t(g) * nqs + ((j + 1) >> 2)) * B + b] = uint16_t(t);
                }
            }
        }
    }
    lds_barrier();
    // The last partial group of every tile leaves as a whole group too (entries past the fill
    // count are never read; the region has room: head is a multiple of GS and cap of 32).
    {
        uint32_t* wd = desc + wave * kRingDescPerWave;
        constexpr uint32_t lpg = GS / 4, gpi = 64 / lpg;
        for (uint32_t b0 = wave * 64; b0 < B; b0 += nt) {
            const uint32_t b = b0 + lane;
            uint32_t hh = 0, tt = 0;
            if (b < B) {
                const uint32_t v = ht[b];
                hh = v >> 16;
                tt = v & 0xFFFFu;
            }
            const bool part = tt > hh;
            const uint64_t m1 = __ballot(part);
            const uint32_t at = __popcll(m1 & ((uint64_t(1) << lane) - 1)), total = __popcll(m1);
            if (part) wd[at] = b | (hh << 12);
            __builtin_amdgcn_wave_barrier();
            for (uint32_t c = 0; c < total; c += gpi) {
                const uint32_t gi = c + lane / lpg, q = lane % lpg;
                if (gi < total) {
                    const uint32_t d = wd[gi];
                    const uint32_t tb = d & 0xFFFu;
                    const uint32_t e = (d >> 12) + q * 4;
                    const uint4 v = ring_group4(ring + tb * RC, e + ring_stagger(tb), rmask);
                    st_stream<PROBE ? kNtProbePart : kNtBuildPart>(region_at(tb, e), v);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    // fill counts; the probe's remaining cumulative counts
    for (uint32_t b = tid; b < B; b += nt) {
        const uint32_t t = ht[b] & 0xFFFFu;
        fill[uint64_t(b) * pg.G + g] = t;
        if constexpr (PROBE)
            for (uint32_t q = (j + 3) >> 2; q <= pg.nq; ++q) pref[(uint64_t(g) * nqs + q) * B + b] = uint16_t(t);
    }
    // the buffered spills (every append is done: the barrier above)
    const uint32_t ns = min(*nspill, pg.spill_cap);
    if (ns) {
        if constexpr (PROBE) {
            for (uint32_t x = tid; x < ns; x += nt) spill_probe(ps, pos_to_bit(sbuf[2 * x], tm), k0 + sbuf[2 * x + 1]);
        } else {
            lds_barrier();  // every thread has read nspill before the dump word takes the base
            if (tid == 0) smem[dump] = atomicAdd(ovf_count, ns);
            lds_barrier();
            const uint32_t base = smem[dump];
            for (uint32_t x = tid; x < ns; x += nt) ovf[base + x] = sbuf[x];
        }
    }
}

// Probe gather for the ring partition: workgroup (g, sp) owns the keys [g*kpw, (g+1)*kpw) of
// partition workgroup g and the tiles [sp*B/S, (sp+1)*B/S) of its regions (S = gridDim.y
// splits, so the gather runs several small workgroups per CU instead of one large one), for nf
// filters at once (a multi-filter probe: the region entries are read once, each filter's
// result bits R + f * r_stride).  Entries of sub-chunks 4q..4q+3 lie in [pref[q], pref[q+1]) of
// their region, so a failed entry at position r belongs to sub-chunk 4q + (entry >> 30) with q
// the last group whose pref[q] <= r; its key is that sub-chunk's first key + the entry's slot.
// A failed entry clears its key's bit in the filter's LDS bitmap of the workgroup's keys.
// S = 1 and nf = 1 writes the hit-mask words directly; otherwise the words are ANDed into
// hw + f * neg_stride (one u32 per 32 keys, preset to all ones) and k_hw_to_hitmask writes
// each filter's hit mask.
//   LDS: nf x kbits[kpw/32], pref rows of the split's tiles as u16 ((B/S) x (nq+1)), and with
//   `qtab` (tq = cap/4 bytes per tile, nq < 255) the group of every 4-entry quad's first entry,
//   so a failed quad starts from its group instead of a binary search over the row.
// NFM: compile-time bound on nf (1 for a single filter: no per-filter registers or loops).
template <int NFM>
__device__ __forceinline__ void gather_ring_body(TileMap tm, PartGeom pg, uint64_t n,
                                                     const uint32_t* __restrict__ regions,
                                                     const uint32_t* __restrict__ R, const uint32_t* __restrict__ fill,
                                                     const uint16_t* __restrict__ pref,
                                                     const uint32_t* __restrict__ neg, uint8_t* __restrict__ hitmask,
                                                     uint32_t* __restrict__ hw, uint32_t nf, uint64_t r_stride,
                                                     uint64_t neg_stride, uint32_t tq) {
    extern __shared__ uint32_t smem[];
    if constexpr (NFM == 1) nf = 1;
    const uint32_t B = tm.nbuckets, cap = pg.cap, wpr = cap / 32, nqs = pg.nq + 1;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint32_t wave = tid >> 6, nwaves = nt >> 6, lane = tid & 63;
    const uint32_t g = blockIdx.x;
    const uint32_t S = gridDim.y, sp = blockIdx.y;
    const uint32_t b_lo = uint32_t(uint64_t(B) * sp / S), b_hi = uint32_t(uint64_t(B) * (sp + 1) / S);
    const uint32_t nb = b_hi - b_lo;
    const uint64_t k0 = uint64_t(g) * pg.kpw;
    const uint64_t k1 = min(n, k0 + pg.kpw);
    const uint32_t nkeys = uint32_t(k1 - k0);
    const uint32_t kw = uint32_t((pg.kpw + 31) / 32);
    uint32_t* kbits = smem;                                         // nf x kw words
    uint16_t* lpref = reinterpret_cast<uint16_t*>(kbits + nf * kw);  // nb * nqs (values <= cap < 2^16)
    uint8_t* qtab = reinterpret_cast<uint8_t*>(lpref + ((nb * nqs + 1) & ~1u));  // nb * tq (tq > 0)
    const uint16_t* gp = pref + uint64_t(g) * nqs * B;  // [q][b] in memory, [b][q] in LDS
    // workgroup g's regions and result words; offsets within them fit 32 bits (B * cap < 2^32)
    const uint32_t* const rgn = regions + uint64_t(g) * B * cap;
    const uint32_t* const Rg = R + uint64_t(g) * B * wpr;
    auto entries_at = [&](uint32_t b, uint32_t r) { return rgn + (b * cap + r); };
    auto rword = [&](uint32_t f, uint32_t b, uint32_t r) { return Rg[f * r_stride + (b * wpr + (r >> 5))]; };
    for (uint32_t x = tid; x < nb * nqs; x += nt) {
        const uint32_t q = x / nb, bb = x - q * nb;
        lpref[bb * nqs + q] = gp[uint64_t(q) * B + b_lo + bb];
    }
    if (tq) {
        lds_barrier();
        // quad c of tile bb starts in group q when pref[q] <= 4c < pref[q+1]: each (tile, group)
        // writes the quads whose first entry it holds (pref[nq] = the fill, the last group open)
        for (uint32_t x = tid; x < nb * nqs; x += nt) {
            const uint32_t bb = x / nqs, q = x - bb * nqs;
            const uint16_t* pb = lpref + bb * nqs;
            const uint32_t lo = (uint32_t(pb[q]) + 3) >> 2;
            const uint32_t hi = q + 1 < nqs ? (uint32_t(pb[q + 1]) + 3) >> 2 : tq;
            for (uint32_t c = lo; c < min(hi, tq); ++c) qtab[bb * tq + c] = uint8_t(q);
        }
    }
    for (uint32_t f = 0; f < nf; ++f) {
        for (uint32_t w = tid; w < kw; w += nt) {
            const uint32_t key0 = w * 32;
            uint32_t m = key0 >= nkeys ? 0u : (nkeys - key0 >= 32 ? ~0u : ((1u << (nkeys - key0)) - 1u));
            if (m) m &= ~neg[f * neg_stride + ((k0 + key0) >> 5)];  // k0 is a multiple of 64
            kbits[f * kw + w] = m;
        }
    }
    lds_barrier();
    constexpr int U = kGatherRegionsInFlight;
    for (uint32_t b0 = b_lo + wave; b0 < b_hi; b0 += nwaves * U) {
        // a region's fill is its last group-boundary count (pref[nq]), already in LDS
        uint32_t fillb[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            fillb[u] = b0 + u * nwaves < b_hi ? uint32_t(lpref[(b0 + u * nwaves - b_lo) * nqs + pg.nq]) : 0u;
        uint32_t maxf = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) maxf = max(maxf, fillb[u]);
        for (uint32_t r0 = 0; r0 < maxf; r0 += 256) {
            uint4 v[U];
            uint32_t rw[NFM][U];
            // single filter: result words first; a quad's entries (only their key ids are
            // needed) are loaded only when one of its entries failed, so quads that passed (a
            // probe batch's members) cost their result bits alone (C2 probe 0.517 -> 0.504 ms;
            // re-measured against loading both together: 0.482 vs 0.520 ms, profiles/r03/s11).
            // Multi-filter sets: nearly every quad fails some filter, so entries and result
            // words go out together.
            uint32_t anyq[U];  // one filter: the quad's failed entries as byte-spread bits (0: skip)
            if constexpr (NFM == 1) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t r = min(r0 + lane * 4, (max(fillb[u], 1u) - 1) & ~3u);
                    const uint32_t b = min(b0 + u * nwaves, b_hi - 1);
                    rw[0][u] = rword(0, b, r);
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t b = b0 + u * nwaves;
                    const uint32_t r = r0 + lane * 4;
                    uint32_t a = 0;
                    if (b < b_hi && r < fillb[u]) {
                        // the quad's 4 result bits sit at bits 0, 8, 16, 24 after the shift (the R
                        // layout, tiled_kernels.hpp); entries past the fill masked off
                        const uint32_t cnt = min(fillb[u] - r, 4u);
                        a = (~rw[0][u] >> ((r & 31) >> 2)) & (0x01010101u >> (32 - 8 * cnt));
                    }
                    anyq[u] = a;
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (anyq[u]) v[u] = ld_stream(entries_at(b0 + u * nwaves, r0 + lane * 4));
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    anyq[u] = 1u;
                    const uint32_t b = min(b0 + u * nwaves, b_hi - 1);
                    const uint32_t r = min(r0 + lane * 4, (max(fillb[u], 1u) - 1) & ~3u);
                    v[u] = ld_stream(entries_at(b, r));
#pragma unroll
                    for (int f = 0; f < NFM; ++f)
                        if (uint32_t(f) < nf) rw[f][u] = rword(f, b, r);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t b = b0 + u * nwaves;
                const uint32_t r = r0 + lane * 4;
                if (anyq[u] && b < b_hi && r < fillb[u]) {
                    // failed entries as byte-spread bits: entry r + t at bit 8t (the result word
                    // shifted to the quad's piece; no compaction multiply)
                    const uint32_t lim = 0x01010101u >> (32 - 8 * min(fillb[u] - r, 4u));
                    uint32_t fl[NFM], any = 0;
#pragma unroll
                    for (int f = 0; f < NFM; ++f) {
                        fl[f] = uint32_t(f) < nf ? ((~rw[f][u] >> ((r & 31) >> 2)) & lim) : 0u;
                        any |= fl[f];
                    }
                    if (any) {
                        // q = the last group with pref[q] <= r (pref non-decreasing, pref[0] = 0):
                        // from the quad table, else a fixed-trip binary search
                        const uint16_t* pb = lpref + (b - b_lo) * nqs;
                        uint32_t lo = 0;
                        if (tq) {
                            lo = qtab[(b - b_lo) * tq + (r >> 2)];
                        } else {
                            uint32_t len = nqs;
                            while (len > 1) {
                                const uint32_t half = len >> 1;
                                if (pb[lo + half] <= r) lo += half;
                                len -= half;
                            }
                        }
                        const uint32_t vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                        // the next two groups' first entries: with no second boundary inside the
                        // quad (nearly always: a group holds ~24 entries of a region at C2) an
                        // entry's group is lo or lo + 1 by one compare, no loop
                        const uint32_t nxt1 = lo + 1 < nqs ? uint32_t(pb[lo + 1]) : 0xFFFFFFFFu;
                        const uint32_t nxt2 = lo + 2 < nqs ? uint32_t(pb[lo + 2]) : 0xFFFFFFFFu;
                        if (nxt2 > r + 3) {
#pragma unroll
                            for (int t = 0; t < 4; ++t) {
                                // key = 4096 group + key-in-group (the entry's top 12 bits)
                                const uint32_t key = ((lo + uint32_t(r + t >= nxt1)) << 12) + (vv[t] >> kSlotShift);
#pragma unroll
                                for (int f = 0; f < NFM; ++f)
                                    if ((fl[f] >> (8 * t)) & 1u) atomicAnd(kbits + f * kw + (key >> 5), ~(1u << (key & 31)));
                            }
                        } else {
                            uint32_t nxt = nxt1;
#pragma unroll
                            for (int t = 0; t < 4; ++t) {
                                if ((any >> (8 * t)) & 1u) {
                                    if (r + t >= nxt) {
                                        ++lo;
                                        while (lo + 1 < nqs && pb[lo + 1] <= r + t) ++lo;
                                        nxt = lo + 1 < nqs ? uint32_t(pb[lo + 1]) : 0xFFFFFFFFu;
                                    }
                                    const uint32_t key = (lo << 12) + (vv[t] >> kSlotShift);
#pragma unroll
                                    for (int f = 0; f < NFM; ++f)
                                        if ((fl[f] >> (8 * t)) & 1u) atomicAnd(kbits + f * kw + (key >> 5), ~(1u << (key & 31)));
                                }
                            }
                        }
                    }
                }
            }
        }
    }
    lds_barrier();
    if (S > 1 || nf > 1) {
        for (uint32_t f = 0; f < nf; ++f)
            for (uint32_t w = tid; w * 32 < nkeys; w += nt) {
                const uint32_t bits = kbits[f * kw + w];
                if (bits != ~0u) atomicAnd(hw + f * neg_stride + (k0 >> 5) + w, bits);  // (hw preset to ones)
            }
        return;
    }
    for (uint32_t w = tid; w * 32 < nkeys; w += nt) {
        const uint64_t key0 = k0 + uint64_t(w) * 32;
        const uint32_t bits = kbits[w];
        const uint64_t nbt = min<uint64_t>(4, (n - key0 + 7) / 8);
        if (nbt == 4 && (reinterpret_cast<uintptr_t>(hitmask + key0 / 8) & 3) == 0)
            *reinterpret_cast<uint32_t*>(hitmask + key0 / 8) = bits;
        else
            for (uint64_t q = 0; q < nbt; ++q) hitmask[key0 / 8 + q] = uint8_t(bits >> (8 * q));
    }
}

// One filter: 512 threads, capped at 64 VGPRs so 8 waves per SIMD (4 workgroups per CU, the LDS
// limit) stay resident.  The set gather keeps its registers (one LDS key bitmap and result word
// per filter) and, as its LDS admits one workgroup per CU, runs 1024 threads (16 waves) when
// the host launches it so.
template <int NFM>
__global__ void __launch_bounds__(1024) k_gather_ring(TileMap tm, PartGeom pg, uint64_t n,
                                                     const uint32_t* __restrict__ regions,
                                                     const uint32_t* __restrict__ R, const uint32_t* __restrict__ fill,
                                                     const uint16_t* __restrict__ pref,
                                                     const uint32_t* __restrict__ neg, uint8_t* __restrict__ hitmask,
                                                     uint32_t* __restrict__ hw, uint32_t nf, uint64_t r_stride,
                                                     uint64_t neg_stride, uint32_t tq) {
    gather_ring_body<NFM>(tm, pg, n, regions, R, fill, pref, neg, hitmask, hw, nf, r_stride, neg_stride, tq);
}
template <>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8)))
k_gather_ring<1>(TileMap tm, PartGeom pg, uint64_t n, const uint32_t* __restrict__ regions,
                 const uint32_t* __restrict__ R, const uint32_t* __restrict__ fill, const uint16_t* __restrict__ pref,
                 const uint32_t* __restrict__ neg, uint8_t* __restrict__ hitmask, uint32_t* __restrict__ hw, uint32_t nf,
                 uint64_t r_stride, uint64_t neg_stride, uint32_t tq) {
    gather_ring_body<1>(tm, pg, n, regions, R, fill, pref, neg, hitmask, hw, nf, r_stride, neg_stride, tq);
}

}  // namespace pbf
