// Resident one-key reader for the per-key calls of LsmStorage.get (reference src/lsm_storage.py:
// 164-179: `sstable.bloom_filter.may_contain(key)` = bloom_filter.py:67-74, per filter), gfx950.
//
// A launch per key costs the host's launch path and the GPU's dispatch on every call (~9 us of
// the ~12 us a may_contain took).  Instead ONE wave stays resident on a stream of its own while
// keys arrive: host threads post requests into slots of a board in mapped, coherent pinned host
// memory and the wave polls the slots' 128-byte heads over the bus (one load round trip per
// poll: 8 lanes per slot, the stop word beside them), answers every posted request and writes the
// answer and the request's sequence number back.  The wave
// leaves after `idle` ticks without a request (and after `life` ticks whatever happens, so it
// never holds its queue for long), and on the board's stop word; the host relaunches it when a
// request finds it gone (pebblebloom.hip: ResidentReader).
//
// Per request (one key against up to 64 filters sharing k, like k_may_contain_set): the key
// (from the head when it has at most 76 bytes, else one 16-B load per lane from the slot body)
// goes into LDS, lane s hashes seed s (MurmurHash3_x86_32, seeds
// 0..k-1), lane f gathers the k hashes from the other lanes and tests filter f's k bits, one
// ballot is the answer.  Every load of host memory is volatile (the board changes under the
// kernel: no load may be hoisted out of the poll loop or served from a cache), and the bitmap
// words are read with device-scope atomic loads, so a filter rebuilt on another XCD since the
// wave started is never read from a stale line of this XCD's L2 (the host only posts keys for a
// filter with no work still queued on its stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "murmur_device.hpp"

namespace pbf {

constexpr uint32_t kSvcSlots = 64;     // host threads with a slot (one lane each)
constexpr uint32_t kSvcKeyMax = 1024;  // longer keys take the launch path
constexpr uint32_t kSvcFilters = 64;   // filters per request (one lane each)
constexpr uint32_t kSvcInlineKey = 76; // keys up to this many bytes travel in the head lines

struct SvcFilter {  // 32 B
    const uint32_t* bm;
    IndexMap im;
};
static_assert(sizeof(SvcFilter) == 32, "SvcFilter layout");

// Slot s's request head: two 64-B lines, each written by the host with its sequence tag last
// (req in line 0, req2 in line 1; x86 keeps stores in order, and a read of one line over the bus
// returns a snapshot of it).  The wave reads both lines in its poll (8 lanes x 16 B per slot), and
// a request is complete when req == req2: for a one-filter request with a key of up to
// kSvcInlineKey bytes -- may_contain's -- the poll has brought everything the answer needs.
struct alignas(64) SvcHead {
    uint32_t req;        // line 0: sequence number of the posted request (never 0)
    uint32_t nf;         // filters (1..kSvcFilters)
    uint32_t len;        // key bytes (<= kSvcKeyMax)
    uint32_t k;          // hash functions (1..32), shared by the request's filters
    SvcFilter f0;        // filters[0]
    uint8_t key0[16];    // key bytes [0, 16) (len <= kSvcInlineKey)
    uint32_t req2;       // line 1: the same sequence number
    uint8_t key1[60];    // key bytes [16, 76)
};
static_assert(sizeof(SvcHead) == 128, "SvcHead layout: two lines");

struct SvcSlot {
    uint32_t ack;      // device: the sequence answered, stored after `bits`
    uint32_t pad0;
    uint64_t bits;     // device: bit f = filters[f] may contain the key
    uint8_t pad1[48];  // the body starts on its own 64-B line
    SvcFilter f[kSvcFilters];  // filters[1..nf) (filters[0] is in the head)
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
};

__device__ __forceinline__ uint4 vload16(const void* p) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u x = *reinterpret_cast<const volatile v4u*>(p);
    return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ uint32_t vload4(const void* p) { return *reinterpret_cast<const volatile uint32_t*>(p); }

// The answer: ack and bits in ONE 16-byte store to the slot's first 16 bytes (a single bus write,
// so the host never sees the new ack with the old bits) -- not a release at system scope, which
// compiles to an L2 write-back (buffer_wbl2) of this XCD's whole L2 per answer: with ~200k gets/s
// that slowed a concurrent batched probe by 40% (profiles/r06/s3).  The board is coherent host
// memory, which the GPU does not cache.
__device__ __forceinline__ void svc_ack(SvcSlot* sl, uint32_t req, uint64_t bits) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u x = {req, 0u, uint32_t(bits), uint32_t(bits >> 32)};
    *reinterpret_cast<volatile v4u*>(sl) = x;
}

// Filter fd's k bits (lanes f < nf) for the hashes held by lanes 0..k-1 (k <= KMAX): every
// lane takes part in the shuffles (a lane reading an inactive lane's register gets no data), then
// the k loads of a filter go out together.
template <int KMAX>
__device__ __forceinline__ bool svc_test(uint32_t h, uint32_t k, bool active, const SvcFilter& fd) {
    uint32_t hv[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; ++q) hv[q] = __shfl(h, q, 64);
    if (!active) return false;
    uint32_t w[KMAX], sh[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
        const uint64_t idx = py_index(hv[q], fd.im);
        sh[q] = uint32_t(idx & 31);
        w[q] = uint32_t(q) < k ? __hip_atomic_load(fd.bm + (idx >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0u;
    }
    uint32_t acc = 1u;
#pragma unroll
    for (int q = 0; q < KMAX; ++q) acc &= w[q] >> sh[q];
    return (acc & 1u) != 0u;
}

// One request of slot s, its head lines in LDS (hb, 32 words): the key into LDS (from the head,
// or for a longer key one 16-B load per lane from the slot body), one seed per lane, filter f on
// lane f (filter 0 from the head, the others from the slot body).
__device__ __forceinline__ void svc_answer(SvcBoard* b, uint32_t s, uint32_t req, uint32_t nf, uint32_t len, uint32_t k,
                                           uint32_t* kw, const uint32_t* hb) {
    const uint32_t lane = threadIdx.x;
    SvcSlot* sl = b->slot + s;
    if (len <= kSvcInlineKey) {
        // key words 0..3 at head bytes 48..63, words 4..18 at bytes 68..127
        if (lane < 19) kw[lane] = hb[lane < 4 ? 12 + lane : 17 + (lane - 4)];
    } else if (lane * 16 < len) {  // 16 B per lane (the body's key buffer is 16-B aligned)
        const uint4 w = vload16(sl->key + lane * 16);
        kw[lane * 4] = w.x;
        kw[lane * 4 + 1] = w.y;
        kw[lane * 4 + 2] = w.z;
        kw[lane * 4 + 3] = w.w;
    }
    uint4 d0 = make_uint4(0, 0, 0, 0), d1 = d0;
    if (lane == 0) {
        d0 = make_uint4(hb[4], hb[5], hb[6], hb[7]);
        d1 = make_uint4(hb[8], hb[9], hb[10], hb[11]);
    } else if (lane < nf) {  // (issued beside the key loads)
        d0 = vload16(&sl->f[lane]);
        d1 = vload16(reinterpret_cast<const uint8_t*>(&sl->f[lane]) + 16);
    }
    __syncthreads();
    // lane s: MurmurHash3_x86_32(key, seed s) (bloom_filter.py:46, mmh3.hash(key, s))
    uint32_t h = lane;
    const uint32_t nb = len >> 2, t = len & 3;
    for (uint32_t i = 0; i < nb; ++i) h = round_h(h, mix_block(kw[i]));
    if (t) h ^= mix_block(kw[nb] & ((1u << (8 * t)) - 1u));
    h = fmix32(h ^ len);
    SvcFilter fd;
    fd.bm = reinterpret_cast<const uint32_t*>(uint64_t(d0.x) | (uint64_t(d0.y) << 32));
    fd.im.m = uint64_t(d0.z) | (uint64_t(d0.w) << 32);
    fd.im.magic = uint64_t(d1.x) | (uint64_t(d1.y) << 32);
    fd.im.mode = d1.z;
    fd.im.mask = d1.w;
    // the AND of bloom_filter.py:71-74, without its early exit: the k loads go out together
    const bool act = lane < nf;
    const bool hit = k <= 4    ? svc_test<4>(h, k, act, fd)
                     : k <= 8  ? svc_test<8>(h, k, act, fd)
                     : k <= 16 ? svc_test<16>(h, k, act, fd)
                               : svc_test<32>(h, k, act, fd);
    const unsigned long long bal = __ballot(hit);
    if (lane == 0) svc_ack(sl, req, uint64_t(bal));
    __syncthreads();  // kw and hb are rewritten by the next request
}

// The resident wave (one workgroup of 64 threads).  `id` is the launch's id (state while it
// serves); ticks are wall-clock ticks (hipDeviceAttributeWallClockRate).  Each poll is ONE bus
// round trip: the stop word and the used slots' head lines are loaded together (lane l reads
// piece l & 7 of slot 8i + (l >> 3) in load i; the slot count of the previous poll decides how
// many loads go out).
__global__ void __launch_bounds__(64) k_reader_service(SvcBoard* b, uint32_t id, uint64_t idle_ticks, uint64_t life_ticks) {
    __shared__ uint32_t kw[kSvcKeyMax / 4 + 4];
    __shared__ uint32_t hb[32];
    const uint32_t lane = threadIdx.x, grp = lane >> 3, piece = lane & 7;
    constexpr int NI = kSvcSlots / 8;
    // a relaunch resumes from the answered sequences
    uint32_t done[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) done[i] = vload4(&b->slot[8 * i + grp].ack);
    uint32_t nused = min(vload4(&b->nused), kSvcSlots);
    if (lane == 0) __hip_atomic_store(&b->state, id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t t0 = wall_clock64();
    uint64_t t_last = t0;
    uint32_t served = 0;
    while (true) {
        const uint32_t ni = (nused + 7) >> 3;  // (wave-uniform)
        const uint4 ctl = vload16(&b->stop);   // stop, nused
        uint4 hv[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i)
            hv[i] = uint32_t(i) < ni ? vload16(reinterpret_cast<const uint8_t*>(&b->head[8 * i + grp]) + 16 * piece)
                                     : make_uint4(0, 0, 0, 0);
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
                if (grp == g) reinterpret_cast<uint4*>(hb)[piece] = hv[i];
                __syncthreads();
                const uint32_t rq = hb[0], nf = hb[1], len = hb[2], k = hb[3];
                const uint32_t s = 8 * uint32_t(i) + g;
                // a malformed head (a request retracted by its host thread: nf = 0) is
                // acknowledged with no hits, without reading any memory
                if (nf >= 1 && nf <= kSvcFilters && len <= kSvcKeyMax && k >= 1 && k <= 32) {
                    svc_answer(b, s, rq, nf, len, k, kw, hb);
                } else {
                    if (lane == 0) svc_ack(b->slot + s, rq, 0);
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
