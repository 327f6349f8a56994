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
//   ring      32 entries per tile (RC), groups of GS = 16.  ht[b] = lim << 16 | tail, both in
//             BYTES of region position (4 x entries): tail = entries appended to region (g, b),
//             lim = min(head + RC, cap) with head = entries flushed (a multiple of GS).  Region
//             entry e sits in ring slot e mod RC, so an append's LDS byte address is
//             b * 128 + (tail & 124) and its overrun test one compare of the two halves (tail <
//             lim); appends that fail it left the stream (spill below).  Thread b owns tile b in
//             the flush and keeps head in a register.
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
//             contiguous 128-B run), so k_gather_ring finds an entry's group from its region
//             position.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "tiled_kernels.hpp"

namespace pbf {

constexpr uint32_t kRingKeysPerSub = 1024;  // = threads; the thread field is 10 bits
constexpr uint32_t kRingEntries = 32;       // RC: LDS ring entries per tile (64-B groups of 16)
static_assert(kSlotShift == 20 && kRingKeysPerSub == 1024 && kGroupKeys == 4 * kRingKeysPerSub,
              "probe entry = ((j & 3) << 10 | thread) << 20 | position");
// Key sub-chunks loaded per batch, one batch ahead: 2 measured best with the non-temporal streams
// (C2 A/B over 1/2/3/4/8: profiles/r01/s11/ab.txt)
constexpr int kRingPrefetch = 2;
#ifndef PBF_RING_BFE
#define PBF_RING_BFE 1
#endif
constexpr bool kRingBfe = PBF_RING_BFE;  // tile of a power-of-two position by one bit-field extract
#ifndef PBF_GATHER_BRANCH_FREE
#define PBF_GATHER_BRANCH_FREE 1
#endif
constexpr bool kGatherBranchFree = PBF_GATHER_BRANCH_FREE;
// When a flush's two group stores issue (A/B of the round-5 verdict's desynchronised store
// bursts, profiles/r06/ab/): 0 = both after the next sub-chunk's hash; 1 = odd waves before it,
// even waves after (so half the CU's waves reach the store phase at another time); 2 = one store
// before, one after.  The build partition takes 1 (0.186-0.187 vs 0.191 ms per C2 build pass),
// the probe partition 0 (1 and 2 measured 0.475 / 0.473 vs 0.472 ms).  PBF_RING_STORE_PHASE forces
// one for both (A/B builds).
#ifdef PBF_RING_STORE_PHASE
constexpr int kRingStorePhaseBuild = PBF_RING_STORE_PHASE, kRingStorePhaseProbe = PBF_RING_STORE_PHASE;
#else
constexpr int kRingStorePhaseBuild = 1, kRingStorePhaseProbe = 0;
#endif
// Region capacity bound of the ring partition: tail (bytes) must stay below 2^16 although a
// sub-chunk may append up to kps * k <= 8192 positions past lim (all to one tile: a duplicated
// key) before the flush clamps it: 4 * (cap + 8192) < 2^16.
constexpr uint32_t kRingMaxCap = 8160;

// LDS layout of k_part_ring, 4-byte words: ht[1024] (fixed, so the rings start at byte 4096 for
// every B: the ring base is an instruction offset), the rings [B x RC], the dump word (appends
// that left the stream store there), the spill count, two pad words, then the spill buffer
// (probe: 2 words per entry, build: 1).
constexpr uint32_t kRingHtWords = 1024;
constexpr uint32_t kRingDescWords = 16 * 64 * 2;  // per wave 64 write-out descriptors of 8 B
__host__ __device__ constexpr uint32_t ring_lds_words(uint32_t B) { return kRingHtWords + kRingDescWords + B * kRingEntries + 4; }
constexpr uint32_t kRingLdsWords = 160 * 1024 / 4;  // declared statically by k_part_ring

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
//
// Per position the append is one LDS atomic (returns lim | tail), one compare, the slot address
// (b << 7 | tail & 124, or the dump word) and one LDS store (8 VALU with the tile and the entry);
// per sub-chunk each thread flushes its own tile (take_groups / put_groups below).
template <int KMAX, int KM, bool PROBE, bool POW2, bool EXACT>
__global__ void __launch_bounds__(1024) k_part_ring(KeySet ks, uint64_t n, int k, TileMap tm, PartGeom pg,
                                                    uint32_t* __restrict__ regions, uint32_t* __restrict__ fill,
                                                    uint16_t* __restrict__ pref, uint32_t* __restrict__ ovf,
                                                    uint32_t* __restrict__ ovf_count, ProbeSet ps,
                                                    uint32_t* __restrict__ hw_init) {
    // static LDS (the whole CU's 160 KiB): its base is a link-time constant, so the ring base
    // and the region of an append fold into the LDS instructions' offsets
    __shared__ __attribute__((aligned(16))) uint32_t smem[kRingLdsWords];
    if constexpr (EXACT) k = KMAX;
    constexpr uint32_t RC = kRingEntries;
    constexpr uint32_t SW = PROBE ? 2 : 1;  // spill-buffer words per entry
#ifndef PBF_RING_PROBE_NT
#define PBF_RING_PROBE_NT kNtProbePart
#endif
    constexpr bool NT = PROBE ? PBF_RING_PROBE_NT : kNtBuildPart;
    constexpr int kRingStorePhase = PROBE ? kRingStorePhaseProbe : kRingStorePhaseBuild;
    const uint32_t B = tm.nbuckets;  // <= 1024 = blockDim.x (host: ring_kps)
    const uint32_t shift = tm.tb;
    const uint32_t kps = pg.kps;  // keys per sub-chunk (<= 1024 threads)
    const uint32_t tid = threadIdx.x;
    const uint32_t g = blockIdx.x;
    const uint32_t cap = pg.cap, cap4 = 4 * cap;  // cap <= kRingMaxCap (host)
    const uint32_t lmask = (1u << tm.tb) - 1u;
    char* const lds = reinterpret_cast<char*>(smem);
    constexpr uint32_t RING0 = (kRingHtWords + kRingDescWords) * 4;  // byte offset of the rings
    uint32_t* const ht = smem;
    const uint32_t dump = RING0 / 4 + B * RC;  // word index of the dump slot
    uint32_t* const nspill = smem + dump + 1;
    uint32_t* const sbuf = smem + dump + 4;  // pg.spill_cap entries
    // the workgroup's regions; entry offsets within them fit 32 bits (B * cap < 2^32)
    uint32_t* const rgn = regions + uint64_t(g) * B * cap;
    const uint32_t nqs = pg.nq + 1;  // pref entries per (g, b)
    // the flush: thread tid owns tile tid; its region write cursor (head, bytes) in a register
    const bool owner = tid < B;
    uint16_t* const own_pref = PROBE ? pref + uint64_t(g) * nqs * B + (owner ? tid : 0) : nullptr;  // [q * B]
    uint32_t h4 = 0;
    if (owner) {
        ht[tid] = min(4u * RC, cap4) << 16;
        if constexpr (PROBE) own_pref[0] = 0;
    }
    if (tid == 0) *nspill = 0;
    const uint64_t k0 = uint64_t(g) * pg.kpw;
    const uint64_t k1 = min(n, k0 + pg.kpw);
    if constexpr (PROBE) {
        // this workgroup's words of every filter's miss bits (neg) start at 0 and, when the
        // gather ANDs into words, every filter's gather words (hw_init) at all ones: no memsets
        for (uint64_t w = (k0 >> 5) + tid; w < ((k1 + 31) >> 5); w += blockDim.x) {
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
        } else {
            if constexpr (PROBE)
                spill_probe(ps, pos_to_bit(p, tm), i);
            else
                ovf[atomicAdd(ovf_count, 1u)] = p;
            // (rare) this path's global operations complete here, so the waits after the join
            // can still count the flush stores of the common path instead of draining them
            __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
        }
    };
    // Group write-out, dense store instructions: the wave lists the groups its 64 tiles write
    // now (a ballot and a masked bit count give each its descriptor slot: ring byte offset,
    // region byte offset), then each store instruction writes 16 of them, 4 lanes x 16 B per
    // group, so a group leaves as one whole 64-B segment and the instruction is full.  (Each
    // lane writing its own group as four 16-B stores: C2 probe partition 319 vs 251 us, four
    // times the L2 write requests; quads writing their 4 tiles' groups in 4 DPP-broadcast rounds,
    // whole segments but ~6 groups per store instruction: 271 vs 180 us without the stores.)
    // Every call issues exactly two store instructions (32 groups; lanes past the last group
    // rewrite it, the same bytes; with no group at all they write the workgroup's dummy line past
    // the regions) and only a call with more than 32 groups a third: the compiler then counts the
    // flush stores a key load is followed by, and the wait for the next keys lets those stores
    // stay in flight instead of draining them (vmcnt counts loads and stores in issue order).
    const uint32_t lane = tid & 63u, wave = tid >> 6;
    const uint32_t wave_u = __builtin_amdgcn_readfirstlane(wave);  // (wave-uniform branches)
    uint2* const wdesc = reinterpret_cast<uint2*>(lds + kRingHtWords * 4) + wave * 64;
    const uint32_t ring_own = tid << 7;   // ring byte offset of the owned tile
    const uint32_t rgn_own = tid * cap4;  // its region's byte offset in the workgroup's regions (< 2^32)
    const uint32_t q16 = (lane & 3u) << 4;
    // A flush with no group writes the workgroup's 64-B dummy line after all regions (the host
    // allocates G lines there).  Its address is a 64-bit base of its own, chosen per wave (a
    // scalar select), not a 32-bit offset from rgn: the regions of all workgroups may exceed 4 GiB.
    char* const rgn_b = reinterpret_cast<char*>(rgn);
    char* const dummy_b = reinterpret_cast<char*>(regions + uint64_t(pg.G) * B * cap) + uint64_t(g) * 64;
    const uint2 dummy = make_uint2(0u, 0u);
    // A flush's first 32 groups (two store instructions) are read from the rings into registers
    // (take_groups) and stored after the next sub-chunk's hash (put_groups): the chain ht read ->
    // descriptor write -> descriptor read -> ring read -> store no longer holds the wave between
    // the barriers, its LDS latencies run under the hash.  Groups past 32 of a call are written
    // at once (rare).
    struct Pending {
        uint4 x0, x1;    // pieces q of the wave's groups (lane >> 2) and 16 + (lane >> 2)
        uint32_t a0, a1;  // their byte offsets from `base`
        char* base;       // the workgroup's regions, or its dummy line (no group: wave-uniform)
    };
    auto take_groups = [&](bool has, uint32_t hb, Pending& pd) {  // wave-uniform
        const uint64_t m = __builtin_amdgcn_ballot_w64(has);
#ifndef PBF_RING_UNIFORM_TOTAL
#define PBF_RING_UNIFORM_TOTAL 1
#endif
        // (readfirstlane: the group count is known wave-uniform, so the descriptor selects and
        // the loop over groups past 32 are scalar branches; A/B PBF_RING_UNIFORM_TOTAL=0)
        const uint32_t total = PBF_RING_UNIFORM_TOTAL ? __builtin_amdgcn_readfirstlane(uint32_t(__popcll(m)))
                                                      : uint32_t(__popcll(m));
        pd.base = total ? rgn_b : dummy_b;
        if (has) {
            const uint32_t slot = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
            wdesc[slot] = make_uint2(ring_own | (hb & 64u), rgn_own + hb);
        }
        __builtin_amdgcn_wave_barrier();
        auto desc = [&](uint32_t c) { return total ? wdesc[min(c + (lane >> 2), total - 1)] : dummy; };
        const uint2 d0 = desc(0), d1 = desc(16);
        pd.x0 = *reinterpret_cast<const uint4*>(lds + RING0 + d0.x + q16);
        pd.x1 = *reinterpret_cast<const uint4*>(lds + RING0 + d1.x + q16);
        pd.a0 = d0.y + q16;
        pd.a1 = d1.y + q16;
        for (uint32_t c = 32; c < total; c += 16) {
            const uint2 d = desc(c);
            const uint4 x = *reinterpret_cast<const uint4*>(lds + RING0 + d.x + q16);
            st_stream<NT>(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(rgn) + (d.y + q16)), x);
        }
        __builtin_amdgcn_wave_barrier();
    };
    auto put_groups = [&](const Pending& pd) {
        st_stream<NT>(reinterpret_cast<uint32_t*>(pd.base + pd.a0), pd.x0);
        st_stream<NT>(reinterpret_cast<uint32_t*>(pd.base + pd.a1), pd.x1);
    };
    auto write_groups = [&](bool has, uint32_t hb) {
        Pending pd;
        take_groups(has, hb, pd);
        put_groups(pd);
    };
    // pos[s]: with a power-of-two m the raw hash (its tile is one bit-field extract, the entry
    // keeps the low tb bits), else the position in [0, m)
    uint32_t pos[KMAX];
    const uint32_t bbits = 31u - __builtin_clz(B | 1u);  // log2 B (B a power of two when POW2)
    auto tile_of = [&](uint32_t p) {
        if constexpr (POW2 && kRingBfe) return __builtin_amdgcn_ubfe(p, shift, bbits);
        return p >> shift;
    };
    // the positions of sub-chunk s0's key of this thread.  Fixed 16-byte keys are hashed by every
    // lane (a lane past the keys hashes a clamped copy, never appended).  (Issuing the pending
    // flush's two stores between the seeds instead of after the hash measured no different.)
    auto hash_sub = [&](uint64_t s0, const uint4& w) {
        const uint64_t i = s0 + tid;
        if constexpr (F16) {
            auto emit = [&](int s, uint32_t h) { pos[s] = POW2 && kRingBfe ? h : ring_pos<POW2>(h, tm); };
            murmur_seeds16<KMAX>(w, k, emit);
        } else if (tid < kps && i < k1) {
            auto emit = [&](int s, uint32_t h) { pos[s] = POW2 && kRingBfe ? h : ring_pos<POW2>(h, tm); };
            hash_key<KMAX, KM>(ks, i, k, emit);
        }
    };
    // the first batch's keys are taken before the loop; inside it a batch's keys are taken at the
    // end of the previous batch, after that batch's flush stores, which the wait lets stay in flight
    load_batch(k0);
    uint4 cw[F16 ? P : 1];
    if constexpr (F16) {
#pragma unroll
        for (int u = 0; u < P; ++u) cw[u] = kw[u];
    }
    hash_sub(k0, cw[0]);
    // Nothing in flight at the loop's entry: otherwise the wait the compiler places at the loop
    // header, merging the entry path (the first batch's second key load pending) with the back
    // edge, is a full vmcnt(0) that drains every batch's flush stores
    __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
    uint32_t j = 0;  // sub-chunks done
    for (uint64_t c0 = k0; c0 < k1; c0 += uint64_t(P) * kps) {
        if (c0 + uint64_t(P) * kps < k1) load_batch(c0 + uint64_t(P) * kps);
        // the batch's sub-chunks, u = 0 .. P-1 at compile time (cw[u] register-indexed)
        auto sub = [&](auto U) {
            constexpr int u = decltype(U)::value;
            // (a batch's second sub-chunk past the workgroup's keys still runs, empty: every
            // batch then issues the same stores, which the compiler's wait for the next keys counts)
            const uint64_t s0 = c0 + uint64_t(u) * kps;
            const uint64_t i = s0 + tid;
            const bool live = tid < kps && i < k1;
            lds_barrier();  // previous flush done: ht stable, rings free
            if (live) {
                uint32_t v[KMAX];
#pragma unroll
                for (int s = 0; s < KMAX; ++s)
                    if (s < k) v[s] = atomicAdd(ht + tile_of(pos[s]), 4u);
                const uint32_t tag = PROBE ? (((j & 3u) << 30) | (tid << kSlotShift)) : 0u;
                bool bad = false;  // a position overran its tile's ring or region
#pragma unroll
                for (int s = 0; s < KMAX; ++s) {
                    if (s < k) {
                        const uint32_t b = tile_of(pos[s]);
                        const bool ok = (v[s] & 0xFFFFu) < (v[s] >> 16);
                        // every lane stores (a position that left the stream into the dump word):
                        // no per-seed exec-mask branch
                        const uint32_t off = ok ? ((b << 7) | (v[s] & 124u)) : (dump * 4 - RING0);
                        *reinterpret_cast<uint32_t*>(lds + RING0 + off) = PROBE ? (tag | (pos[s] & lmask)) : pos[s];
                        bad |= !ok;
                    }
                }
                if (bad) {  // rare: heavy key duplication
#pragma unroll
                    for (int s = 0; s < KMAX; ++s)
                        if (s < k && (v[s] & 0xFFFFu) >= (v[s] >> 16)) spill_one(POW2 && kRingBfe ? pos[s] & tm.im.mask : pos[s], i);
                }
            }
            lds_barrier();
            // Flush: every tile's complete groups (<= 2) leave, the owner clamps its tail
            Pending pd;
            {
                const uint32_t v = owner ? ht[tid] : 0u;
                const uint32_t t4 = min(v & 0xFFFFu, v >> 16);  // positions past lim left the stream
                bool more = h4 + 64 <= t4;
                take_groups(more, h4, pd);  // always: its two stores on every path (put_groups below)
                h4 += more ? 64u : 0u;
                more = h4 + 64 <= t4;
                while (__builtin_amdgcn_ballot_w64(more)) {  // wave-uniform: a second group is rare
                    write_groups(more, h4);
                    h4 += more ? 64u : 0u;
                    more = h4 + 64 <= t4;
                }
                if (owner) {
                    ht[tid] = (min(h4 + 4 * RC, cap4) << 16) | t4;
                    if constexpr (PROBE)
                        if (((j + 1) & 3) == 0) own_pref[__umul24((j + 1) >> 2, B)] = uint16_t(t4 >> 2);
                }
            }
            // the next sub-chunk's hash (the next batch's keys, at a batch's end), then this
            // flush's stores (kRingStorePhase: when they issue)
            if constexpr (kRingStorePhase == 1) {
                if (wave_u & 1u) put_groups(pd);
            } else if constexpr (kRingStorePhase == 2) {
                st_stream<NT>(reinterpret_cast<uint32_t*>(pd.base + pd.a0), pd.x0);
            }
            if constexpr (u + 1 < P) {
                hash_sub(s0 + kps, cw[F16 ? u + 1 : 0]);
            } else {
                if constexpr (F16) {
#pragma unroll
                    for (int x = 0; x < P; ++x) cw[x] = kw[x];
                }
                hash_sub(c0 + uint64_t(P) * kps, cw[0]);
            }
            if constexpr (kRingStorePhase == 1) {
                if (!(wave_u & 1u)) put_groups(pd);
            } else if constexpr (kRingStorePhase == 2) {
                st_stream<NT>(reinterpret_cast<uint32_t*>(pd.base + pd.a1), pd.x1);
            } else {
                put_groups(pd);
            }
            ++j;
        };
        static_assert(P == 2, "two sub-chunks per batch");
        sub(std::integral_constant<int, 0>{});
        sub(std::integral_constant<int, 1>{});
    }
    lds_barrier();
    {
        // the last partial group leaves as a whole group too (entries past the fill count are
        // never read; the region has room: head is a multiple of GS and cap of 32)
        const uint32_t t4 = owner ? ht[tid] & 0xFFFFu : 0u;
        write_groups(t4 > h4, h4);
    }
    if (owner) {
        const uint32_t t4 = ht[tid] & 0xFFFFu;
        // fill counts; the probe's remaining cumulative counts
        fill[uint64_t(tid) * pg.G + g] = t4 >> 2;
        if constexpr (PROBE)
            for (uint32_t q = (j + 3) >> 2; q <= pg.nq; ++q) own_pref[uint64_t(q) * B] = uint16_t(t4 >> 2);
    }
    // the buffered spills (every append is done: the barrier above)
    const uint32_t ns = min(*nspill, pg.spill_cap);
    if (ns) {
        if constexpr (PROBE) {
            for (uint32_t x = tid; x < ns; x += blockDim.x) spill_probe(ps, pos_to_bit(sbuf[2 * x], tm), k0 + sbuf[2 * x + 1]);
        } else {
            lds_barrier();  // every thread has read nspill before the dump word takes the base
            if (tid == 0) smem[dump] = atomicAdd(ovf_count, ns);
            lds_barrier();
            const uint32_t base = smem[dump];
            for (uint32_t x = tid; x < ns; x += blockDim.x) ovf[base + x] = sbuf[x];
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
                                if constexpr (NFM == 1 && kGatherBranchFree) {
                                    // every entry's LDS AND, a passing one's with all ones (no
                                    // per-entry branch; most entries of a failed quad failed)
                                    atomicAnd(kbits + (key >> 5), ~(((fl[0] >> (8 * t)) & 1u) << (key & 31)));
                                } else {
#pragma unroll
                                    for (int f = 0; f < NFM; ++f)
                                        if ((fl[f] >> (8 * t)) & 1u) atomicAnd(kbits + f * kw + (key >> 5), ~(1u << (key & 31)));
                                }
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
