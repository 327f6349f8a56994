// Resident one-key reader for the per-key calls of LsmStorage.get (reference src/lsm_storage.py:
// 164-179: `sstable.bloom_filter.may_contain(key)` = bloom_filter.py:67-74, per filter), gfx950.
//
// A launch per key costs the host's launch path and the GPU's dispatch on every call (~9 us of
// the ~12 us a may_contain took).  Instead ONE wave stays resident on a stream of its own while
// keys arrive: host threads post requests into slots of a board in mapped, coherent pinned host
// memory and the wave polls the slots' 128-byte heads over the bus (one load round trip per
// poll: 8 lanes per slot, the control line beside them), answers every posted request and writes
// the answer and the request's sequence number back.  The wave leaves after `idle` ticks without
// a request (and after `life` ticks whatever happens, so it never holds its queue for long), and
// on the board's stop word; the host relaunches it when a request finds it gone (pebblebloom.hip:
// ResidentReader).
//
// Filters travel as 16-bit indexes into the board's descriptor table (bitmap pointer + index map,
// written by the host once per filter), so a get's 16 filters fit in the request head next to the
// key; the wave keeps the descriptors it has read in an LDS cache.  The cache is valid for one
// `epoch` of the table: the host bumps the epoch whenever it frees an index (a destroyed filter)
// and every request carries the epoch it was posted under, so a request never meets a descriptor
// cached for an index's earlier owner.
//
// Per request (one key against up to 64 filters sharing k): the key (from the head when it has at
// most 76 bytes, else one 16-B load per lane from the slot body) goes into LDS, lane s hashes seed
// s (MurmurHash3_x86_32, seeds 0..k-1), and the nf x k (filter, seed) pairs are dealt over the
// lanes -- one index computation and one bitmap load per pair, all loads of a round of 64 pairs
// in flight together -- and a filter hits when none of its pairs found a clear bit.  Every load
// of host memory bypasses the caches (the board changes under the kernel), and the bitmap words
// are read with device-scope atomic loads, so a filter rebuilt on another XCD since the wave
// started is never read from a stale line of this XCD's L2 (the host only posts keys for a filter
// with no work still queued on its stream).
#pragma once
#ifndef PBF_SVC_TICK_AT
#define PBF_SVC_TICK_AT 0
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "murmur_device.hpp"

namespace pbf {

constexpr uint32_t kSvcSlots = 64;       // host threads with a slot (one lane each)
constexpr uint32_t kSvcKeyMax = 1024;    // longer keys take the launch path
constexpr uint32_t kSvcFilters = 64;     // filters per request
constexpr uint32_t kSvcInlineKey = 76;   // keys up to this many bytes travel in the head lines
constexpr uint32_t kSvcInlineIds = 16;   // filter indexes in the head (the rest in the slot body)
constexpr uint32_t kSvcDescs = 65536;    // descriptor table entries (index 0 unused)
constexpr uint32_t kSvcCache = 256;      // LDS descriptor cache entries (direct-mapped by index)

struct SvcFilter {  // 32 B
    const uint32_t* bm;
    IndexMap im;
};
static_assert(sizeof(SvcFilter) == 32, "SvcFilter layout");

// Slot s's request head: two 64-B lines, each written by the host with its sequence tag last
// (req in line 0, req2 in line 1; x86 keeps stores in order, and a read of one line over the bus
// returns a snapshot of it).  The wave reads both lines in its poll (8 lanes x 16 B per slot), and
// a request is complete when req == req2: for up to 16 filters and a key of up to kSvcInlineKey
// bytes -- may_contain's and a get's -- the poll has brought everything but the descriptors.
struct alignas(64) SvcHead {
    uint32_t req;        // line 0: sequence number of the posted request (never 0)
    uint32_t shape;      // nf | k << 8 | len << 16 (nf 1..64, k 1..32, len <= kSvcKeyMax); 0 = retracted
    uint32_t epoch;      // the descriptor table's epoch the indexes belong to
    uint32_t pad;
    uint16_t ids[kSvcInlineIds];  // descriptor indexes of filters [0, 16)
    uint8_t key0[16];    // key bytes [0, 16) (len <= kSvcInlineKey)
    uint32_t req2;       // line 1: the same sequence number
    uint8_t key1[60];    // key bytes [16, 76)
};
static_assert(sizeof(SvcHead) == 128, "SvcHead layout: two lines");

struct SvcSlot {
    uint32_t ack;      // device: the sequence answered, stored with `bits`
    uint32_t ticks;    // device: wall-clock ticks from seeing the request to answering it
    uint64_t bits;     // device: bit f = filters[f] may contain the key
    uint8_t pad1[48];  // the body starts on its own 64-B line
    uint16_t ids[kSvcFilters];            // indexes of filters [16, nf)
    alignas(16) uint8_t key[kSvcKeyMax];  // keys longer than kSvcInlineKey
};

struct SvcBoard {
    uint32_t stop;    // host: nonzero, the wave leaves at its next poll
    uint32_t nused;   // host: slots [0, nused) may hold requests (the lanes that poll)
    uint32_t state;   // device: launch id while serving, 0 once the wave has left
    uint32_t served;  // device: requests answered by the last launch
    uint32_t pad[12];
    SvcHead head[kSvcSlots];
    SvcSlot slot[kSvcSlots];
    SvcFilter desc[kSvcDescs];  // host: descriptor of index i (written before any request names i)
};

typedef uint32_t svc_v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 vload16(const void* p) {
    const svc_v4u x = *reinterpret_cast<const volatile svc_v4u*>(p);
    return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ uint32_t vload4(const void* p) { return *reinterpret_cast<const volatile uint32_t*>(p); }

// Loads of host memory that go out together: a volatile load is followed by a wait for it, so a
// poll's control line and head lines would cost one bus round trip each.  These issue the load
// (cache-bypassing, like the volatile form) without a wait; svc_wait() waits for all of them and
// svc_touch() then orders every use of a loaded value after that wait.
__device__ __forceinline__ svc_v4u svc_issue16(const void* p) {
    svc_v4u v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ void svc_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint4 svc_touch(svc_v4u v) {
    asm volatile("" : "+v"(v));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// The answer: ack and bits in ONE 16-byte store to the slot's first 16 bytes (a single bus write,
// so the host never sees the new ack with the old bits) -- not a release at system scope, which
// compiles to an L2 write-back (buffer_wbl2) of this XCD's whole L2 per answer: with ~200k gets/s
// that slowed a concurrent batched probe by 40% (profiles/r06/s3).  The board is coherent host
// memory, which the GPU does not cache.
// (The second word carries the wall-clock ticks from the request's detection to the answer: the
// host's pbf_resident_stats.)
__device__ __forceinline__ void svc_ack(SvcSlot* sl, uint32_t req, uint64_t bits, uint32_t ticks) {
    const svc_v4u x = {req, ticks, uint32_t(bits), uint32_t(bits >> 32)};
    *reinterpret_cast<volatile svc_v4u*>(sl) = x;
}

// LDS of the resident wave.
struct SvcLds {
    uint32_t kw[kSvcKeyMax / 4 + 4];   // the key
    uint32_t hb[32];                   // the request's head lines
    uint32_t hs[32];                   // hash of seed s
    SvcFilter rq[kSvcFilters];         // the request's descriptors, by filter
    uint32_t miss[kSvcFilters];        // filter f met a clear bit
    uint32_t ctag[kSvcCache];          // cached index (0: empty)
    SvcFilter cdesc[kSvcCache];
};

// One request of slot s, its head lines in LDS (hb, 32 words).
__device__ __forceinline__ void svc_answer(SvcBoard* b, uint32_t s, uint32_t req, uint32_t nf, uint32_t len, uint32_t k,
                                           SvcLds& L, uint64_t t_seen) {
    const uint32_t lane = threadIdx.x;
    SvcSlot* sl = b->slot + s;
    // the key and the filters' indexes: from the head, or (a longer key, filters past 16) the body
    if (len <= kSvcInlineKey) {
        // key words 0..3 at head bytes 48..63, words 4..18 at bytes 68..127
        if (lane < 19) L.kw[lane] = L.hb[lane < 4 ? 12 + lane : 17 + (lane - 4)];
    } else if (lane * 16 < len) {  // 16 B per lane (the body's key buffer is 16-B aligned)
        const uint4 w = vload16(sl->key + lane * 16);
        L.kw[lane * 4] = w.x;
        L.kw[lane * 4 + 1] = w.y;
        L.kw[lane * 4 + 2] = w.z;
        L.kw[lane * 4 + 3] = w.w;
    }
    uint32_t id = 0;
    if (lane < nf) {
        id = lane < kSvcInlineIds ? (L.hb[4 + (lane >> 1)] >> (16 * (lane & 1))) & 0xFFFFu
                                  : uint32_t(*reinterpret_cast<const volatile uint16_t*>(sl->ids + lane));
    }
    // the descriptors: the LDS cache, else one load round trip over the bus for every lane missing
    const uint32_t ce = id & (kSvcCache - 1);
    const bool miss = lane < nf && L.ctag[ce] != id;
    svc_v4u m0 = {0u, 0u, 0u, 0u}, m1 = m0;
    if (miss) {
        const uint8_t* p = reinterpret_cast<const uint8_t*>(b->desc + id);
        m0 = svc_issue16(p);
        m1 = svc_issue16(p + 16);
    }
    svc_wait();
    const uint4 d0 = svc_touch(m0), d1 = svc_touch(m1);
    if (lane < nf) {
        SvcFilter fd;
        if (miss) {
            fd.bm = reinterpret_cast<const uint32_t*>(uint64_t(d0.x) | (uint64_t(d0.y) << 32));
            fd.im.m = uint64_t(d0.z) | (uint64_t(d0.w) << 32);
            fd.im.magic = uint64_t(d1.x) | (uint64_t(d1.y) << 32);
            fd.im.mode = d1.z;
            fd.im.mask = d1.w;
        } else {
            fd = L.cdesc[ce];
        }
        L.rq[lane] = fd;
        L.miss[lane] = 0u;
    }
    __syncthreads();
#if PBF_SVC_TICK_AT == 1  // (A/B: the wave's time to this point instead of to the answer)
    const uint64_t t_mark = wall_clock64();
#endif
    // into the cache: of the lanes whose indexes share an entry, the one whose tag landed writes it
    if (miss) L.ctag[ce] = id;
    __syncthreads();
    if (miss && L.ctag[ce] == id) L.cdesc[ce] = L.rq[lane];
    // lane s: MurmurHash3_x86_32(key, seed s) (bloom_filter.py:46, mmh3.hash(key, s))
    uint32_t h = lane;
    const uint32_t nb = len >> 2, t = len & 3;
    for (uint32_t i = 0; i < nb; ++i) h = round_h(h, mix_block(L.kw[i]));
    if (t) h ^= mix_block(L.kw[nb] & ((1u << (8 * t)) - 1u));
    h = fmix32(h ^ len);
    if (lane < k) L.hs[lane] = h;
    __syncthreads();
#if PBF_SVC_TICK_AT == 2
    const uint64_t t_mark = wall_clock64();
#endif
    // the AND of bloom_filter.py:71-74 for every filter, without its early exit: pair p = (filter
    // p / k, seed p % k); up to 4 rounds of 64 pairs issue their loads before any is used
    const uint32_t np = nf * k;
    const uint32_t inv = (65536u + k - 1u) / k;  // p / k = (p * inv) >> 16, exact for p < 2048, k <= 32
    for (uint32_t p0 = 0; p0 < np; p0 += 256) {
        uint32_t w[4], sh[4], fr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            w[r] = ~0u;
            sh[r] = 0;
            fr[r] = 0;
            if (p0 + 64u * r < np) {  // (wave-uniform)
                const uint32_t p = min(p0 + 64u * r + lane, np - 1u);  // past the end: a repeat of the last pair
                const uint32_t f = (p * inv) >> 16;
                const uint32_t sd = p - f * k;
                const SvcFilter fd = L.rq[f];
                const uint64_t idx = py_index(L.hs[sd], fd.im);
                sh[r] = uint32_t(idx & 31);
                fr[r] = f;
                // through a global (not flat) pointer: a flat load counts on the LDS counter too,
                // so the next round's LDS reads would wait for this round's bitmap load
                const __attribute__((address_space(1))) uint32_t* gw =
                    (const __attribute__((address_space(1))) uint32_t*)(fd.bm + (idx >> 5));
                w[r] = __hip_atomic_load(gw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (!((w[r] >> sh[r]) & 1u)) L.miss[fr[r]] = 1u;
    }
    __syncthreads();
#if PBF_SVC_TICK_AT == 3
    const uint64_t t_mark = wall_clock64();
#endif
    const bool hit = lane < nf && L.miss[lane] == 0u;
    const unsigned long long bal = __ballot(hit);
#if PBF_SVC_TICK_AT >= 1
    if (lane == 0) svc_ack(sl, req, uint64_t(bal), uint32_t(t_mark - t_seen));
#else
    if (lane == 0) svc_ack(sl, req, uint64_t(bal), uint32_t(wall_clock64() - t_seen));
#endif
    __syncthreads();  // kw, hb, rq and miss are rewritten by the next request
}

// The resident wave (one workgroup of 64 threads).  `id` is the launch's id (state while it
// serves); ticks are wall-clock ticks (hipDeviceAttributeWallClockRate).  Each poll is ONE bus
// round trip: the control line and the used slots' head lines are loaded together (lane l reads
// piece l & 7 of slot 8i + (l >> 3) in load i; the slot count of the previous poll decides how
// many loads go out).
__global__ void __launch_bounds__(64) k_reader_service(SvcBoard* b, uint32_t id, uint64_t idle_ticks, uint64_t life_ticks) {
    __shared__ SvcLds L;
    const uint32_t lane = threadIdx.x, grp = lane >> 3, piece = lane & 7;
    constexpr int NI = kSvcSlots / 8;
    for (uint32_t i = lane; i < kSvcCache; i += 64) L.ctag[i] = 0u;
    uint32_t cepoch = 0;  // (the cache starts empty: any epoch may fill it)
    // a relaunch resumes from the answered sequences
    uint32_t done[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) done[i] = vload4(&b->slot[8 * i + grp].ack);
    uint32_t nused = min(vload4(&b->nused), kSvcSlots);
    if (lane == 0) __hip_atomic_store(&b->state, id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    const uint64_t t0 = wall_clock64();
    uint64_t t_last = t0;
    uint32_t served = 0;
    while (true) {
        const uint32_t ni = (nused + 7) >> 3;  // (wave-uniform)
        svc_v4u raw[NI];
        const svc_v4u rctl = svc_issue16(&b->stop);  // stop, nused
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            raw[i] = svc_v4u{0u, 0u, 0u, 0u};
            if (uint32_t(i) < ni) raw[i] = svc_issue16(reinterpret_cast<const uint8_t*>(&b->head[8 * i + grp]) + 16 * piece);
        }
        svc_wait();
        const uint4 ctl = svc_touch(rctl);
        uint4 hv[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) hv[i] = svc_touch(raw[i]);
        if (ctl.x) break;
        nused = min(ctl.y, kSvcSlots);
        bool any = false;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if (uint32_t(i) >= ni) break;
            // the group's req (piece 0) and req2 (piece 4): complete when equal
            const uint32_t req = __shfl(hv[i].x, int(lane & ~7u), 64);
            const uint32_t req2 = __shfl(hv[i].x, int((lane & ~7u) | 4u), 64);
            uint64_t pend = __ballot(piece == 0 && req != done[i] && req == req2);
            while (pend) {
                const uint32_t g = uint32_t(__builtin_ctzll(pend)) >> 3;
                pend &= pend - 1;
                const uint64_t t_seen = wall_clock64();
                if (grp == g) reinterpret_cast<uint4*>(L.hb)[piece] = hv[i];
                __syncthreads();
                const uint32_t rq = L.hb[0], shape = L.hb[1], epoch = L.hb[2];
                const uint32_t nf = shape & 0xFFu, k = (shape >> 8) & 0xFFu, len = shape >> 16;
                const uint32_t s = 8 * uint32_t(i) + g;
                // a malformed head (a request retracted by its host thread: shape = 0) is
                // acknowledged with no hits, without reading any memory
                if (nf >= 1 && nf <= kSvcFilters && len <= kSvcKeyMax && k >= 1 && k <= 32) {
                    if (epoch != cepoch) {  // indexes were freed since the cache was filled
                        for (uint32_t c = lane; c < kSvcCache; c += 64) L.ctag[c] = 0u;
                        cepoch = epoch;
                        __syncthreads();
                    }
                    svc_answer(b, s, rq, nf, len, k, L, t_seen);
                } else {
                    if (lane == 0) svc_ack(b->slot + s, rq, 0, 0);
                    __syncthreads();
                }
                if (grp == g) done[i] = rq;
                ++served;
                any = true;
            }
        }
        if (any) {
            t_last = wall_clock64();
            continue;
        }
        const uint64_t now = wall_clock64();
        if (now - t_last > idle_ticks || now - t0 > life_ticks) break;
        __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) {
        __hip_atomic_store(&b->served, served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&b->state, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace pbf
