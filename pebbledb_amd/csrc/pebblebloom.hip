// libpebblebloom.so — C-ABI (include/pebblebloom.h) over the HIP bloom kernels.
//
// Reference surface replaced: MaudGautier/pebbledb src/bloom_filter.py —
//   pbf_create        ← BloomFilter.__init__            (bloom_filter.py:26-31)
//   pbf_add[_fixed]   ← BloomFilter.add / _set_bit       (:60-65, :51-54)
//   pbf_probe[_fixed] ← BloomFilter.may_contain / _is_bit_set (:67-74, :56-58)
//   pbf_hash_indices  ← BloomFilter._hash                (:38-49)
//   pbf_get_bitmap    ← BloomFilter.to_bytes (bitmap part) (:76-81)
//   pbf_set_bitmap    ← BloomFilter.from_bytes (bitmap part) (:83-90)
// There is no CPU fallback in this library: every entry point runs on the GPU or fails.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <atomic>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/pebblebloom.h"
#include "bloom_kernels.hpp"
#include "tiled_kernels.hpp"
#include "ring_kernels.hpp"
#include "sstable_kernels.hpp"
#include "lsm_kernels.hpp"
#include "set_kernels.hpp"
#include "reader_service.hpp"

using namespace pbf;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(PBF_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
    } while (0)

#define CHECK_LAUNCH() HIP_TRY(hipGetLastError())
// after a launch on f's stream: checks it and names it as the stream's last kernel (reported by
// wait_stream when the stream does not finish in time)
#define LAUNCHED(f, name)           \
    do {                            \
        (f)->last_kernel = (name);  \
        (f)->pending = true;        \
        CHECK_LAUNCH();             \
    } while (0)

// Every stream the library queues work on (the filter and reader stream pools, the encoder's),
// per device: a buffer's users are done once these are (not a device-wide sync, which would also
// wait for the resident reader's wave, up to its 200 ms life).
std::mutex g_lib_streams_mu;
std::map<int, std::vector<hipStream_t>> g_lib_streams;
void register_stream(int device, hipStream_t s) {
    std::lock_guard<std::mutex> lock(g_lib_streams_mu);
    g_lib_streams[device].push_back(s);
}
hipError_t sync_library_streams() {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::vector<hipStream_t> ss;
    {
        std::lock_guard<std::mutex> lock(g_lib_streams_mu);
        ss = g_lib_streams[dev];
    }
    for (hipStream_t s : ss)
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    return hipStreamSynchronize(nullptr);
}

// Device working memory from the device's stream-ordered pool (hipMallocAsync / hipFreeAsync on
// the null stream): hipFree and hipDeviceSynchronize wait for every kernel on the device, the
// resident reader's too (measured: tools/microbench/cumask_block.hip), the pool's calls do not.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool pooled = false;
    hipError_t ensure(size_t want) {
        if (want <= bytes) return hipSuccess;
        if (p) {
            // growth only: the old buffer may still be read by queued work on the library's streams
            hipError_t s = sync_library_streams();
            if (s != hipSuccess) return s;
            release();
        }
        hipError_t e = hipMallocAsync(&p, want, nullptr);
        pooled = e == hipSuccess;
        if (pooled) {
            e = hipStreamSynchronize(nullptr);  // usable from every stream
        } else {
            (void)hipGetLastError();
            e = hipMalloc(&p, want);
        }
        if (e == hipSuccess) bytes = want;
        return e;
    }
    void release() {
        if (p) {
            if (pooled) {
                (void)hipFreeAsync(p, nullptr);
                (void)hipStreamSynchronize(nullptr);
            } else {
                (void)hipFree(p);
            }
        }
        p = nullptr;
        bytes = 0;
        pooled = false;
    }
};

struct PinBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipEvent_t done = nullptr;  // last async copy out of this buffer
    hipError_t ensure(size_t want) {
        if (want <= bytes) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) bytes = want;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        if (done) (void)hipEventDestroy(done);
        p = nullptr;
        done = nullptr;
        bytes = 0;
    }
};

// host→device staging chunk (PBF_STAGE_BYTES overrides, for tests of the chunked path)
size_t stage_bytes() {
    static const size_t v = [] {
        const char* e = std::getenv("PBF_STAGE_BYTES");
        const long long x = e ? std::atoll(e) : 0;
        return x > 0 ? size_t(x) : (size_t(256) << 20);
    }();
    return v;
}
// Positions per tiled pipeline: the partition counts them in u32 (fill, overflow list).  Round 3
// capped pipelines at 2^30 positions: C4's 125M-key filters (1.25G positions) ran as 107M + 18M
// keys, and the second pipeline's tile pass streamed the whole 225 MB bitmap again for 18M keys.
constexpr uint64_t kMaxPositions = (uint64_t(1) << 32) - (uint64_t(1) << 26);
// Probes keep 2^30 per pipeline: C3's 200M keys in ONE pipeline (G = 512, a 390K-key gather key
// bitmap per workgroup) measured 14.8 vs 12.9 ms for two of 100M (profiles/r04/s4): the gather's
// LDS then admits half the workgroups per CU.
constexpr uint64_t kMaxProbePositions = uint64_t(1) << 30;

// Words loaded in the direct probe's first stage (k_probe): 2 measured best of 1/2/6
// (profiles/r02/s1, the direct probe is the small-batch path).
constexpr int kProbeStage1 = 2;

// Most partition workgroups of one pipeline (PBF_PART_G overrides; default 256 = one per CU).
// More workgroups mean fewer keys each: smaller gather key bitmaps and run tables.
// Measured (profiles/r02/s5): the counting-sort PROBE partition prefers 512 (C3 probe 17.4 ->
// 16.0 ms: the gather's per-workgroup key bitmap and run tables halve, more gather workgroups
// fit a CU), the ring partition 256 (C2 probe 0.586 -> 0.604 ms at 512).
bool resident_live(int device);  // (the resident one-key reader below)

uint64_t part_max_groups(bool sort_probe) {
    static const long long v = [] {
        const char* e = std::getenv("PBF_PART_G");
        return e ? std::atoll(e) : 0LL;
    }();
    if (v > 0) return uint64_t(std::min<long long>(v, 8192));
    return sort_probe ? 512 : 256;
}

// Tile-range splits of the ring probe's gather (PBF_GATHER_SPLIT overrides; 1 = one workgroup
// per partition workgroup, writing the hit mask directly).
uint32_t gather_splits() {
    static const uint32_t v = [] {
        const char* e = std::getenv("PBF_GATHER_SPLIT");
        const int x = e ? std::atoi(e) : 0;
        // 16 measured ~1% faster on C2 alone but 7% slower on C5's 8-filter gather
        // (profiles/r01/s11/ab.txt, profiles/r01/s11/final_split16/): 8
        return x > 0 ? uint32_t(std::min(x, 64)) : 8u;
    }();
    return v;
}

int kmax_for(uint32_t k) {
    if (k <= 4) return 4;
    if (k <= 8) return 8;
    if (k <= 16) return 16;
    if (k <= 32) return 32;
    return 0;
}

template <class F>
void dispatch(int kmax, int km, F&& f) {
    auto g = [&](auto KM) {
        switch (kmax) {
            case 4: f(std::integral_constant<int, 4>{}, KM); break;
            case 8: f(std::integral_constant<int, 8>{}, KM); break;
            case 16: f(std::integral_constant<int, 16>{}, KM); break;
            case 32: f(std::integral_constant<int, 32>{}, KM); break;
            default: f(std::integral_constant<int, 0>{}, KM); break;
        }
    };
    switch (km) {
        case kFixed16: g(std::integral_constant<int, kFixed16>{}); break;
        case kFixedN: g(std::integral_constant<int, kFixedN>{}); break;
        default: g(std::integral_constant<int, kVar>{}); break;
    }
}

IndexMap make_index_map(uint64_t m) {
    IndexMap im{};
    im.m = m;
    const bool pow2 = (m & (m - 1)) == 0;
    if (pow2 && m <= (uint64_t(1) << 32)) {
        im.mode = kPow2;
        im.mask = uint32_t(m - 1);
    } else if (m < (uint64_t(1) << 30)) {
        // mod_small's reciprocal: l = ceil(log2 m), M = ceil(2^(31+l) / m) < 2^32, shift l-1
        uint32_t l = 0;
        while ((uint64_t(1) << l) < m) ++l;
        im.mode = kSmall;
        im.magic = ((uint64_t(1) << (31 + l)) + m - 1) / m;
        im.mask = l - 1;
    } else if (m < (uint64_t(1) << 31)) {
        im.mode = kNear;
    } else {
        im.mode = kLarge;
    }
    return im;
}

// Dynamic LDS above 64 KiB must be allowed per kernel (gfx950 has 160 KiB per CU).  The
// attribute call is slow (~0.5 ms): do it once per (device, kernel) at the largest size seen.
template <class K>
hipError_t allow_lds(K kernel, size_t bytes) {
    if (bytes <= 65536) return hipSuccess;
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, size_t> done;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const auto key = std::make_pair(dev, reinterpret_cast<const void*>(kernel));
    std::lock_guard<std::mutex> lock(mu);
    auto it = done.find(key);
    if (it != done.end() && it->second >= bytes) return hipSuccess;
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int(bytes));
    if (e == hipSuccess) done[key] = bytes;
    return e;
}

uint32_t ceil_log2(uint64_t x) {
    uint32_t r = 0;
    while ((uint64_t(1) << r) < x) ++r;
    return r;
}

}  // namespace

namespace {

// Transient working memory of the tiled pipelines and the host staging path.  It is not owned
// by a filter: an LSM keeps one filter per SSTable alive for the SSTable's lifetime, and each
// needs only its bitmap once built.  A device keeps a small pool of these sets; a call leases
// one for the duration of its host-side enqueue, and the GPU-side reuse across streams is
// ordered by the set's `last` event (the next user's stream waits on it).
struct Scratch {
    DevBuf regions, fill, ovf, ovf_count, pref, rbits, neg, hw;
    uint32_t ovf_phase = 0;  // which of the two overflow counters the next build uses
    bool ovf_init = false;
    DevBuf dkeys, doffs, dout;
    DevBuf svals, splan, ssec, serr;  // pbf_build_sstable: values + value offsets, block plan, section
    PinBuf pin[2];
    int pin_next = 0;
    hipEvent_t last = nullptr;          // completion of the last user's work
    hipStream_t last_stream = nullptr;  // ... on this stream
    bool leased = false;
    void release_all() {
        for (DevBuf* d : {&regions, &fill, &ovf, &ovf_count, &pref, &rbits, &neg, &hw, &dkeys, &doffs, &dout,
                          &svals, &splan, &ssec, &serr})
            d->release();
        pin[0].release();
        pin[1].release();
        ovf_init = false;
    }
};

struct DevicePool {
    std::mutex mu;
    std::vector<Scratch*> sets;
};

DevicePool& device_pool(int device) {
    static std::mutex mu;
    static std::map<int, DevicePool*> pools;
    std::lock_guard<std::mutex> lock(mu);
    auto& p = pools[device];
    if (!p) p = new DevicePool();
    return *p;
}

// Sets kept per device before a lease waits for an idle one (PBF_SCRATCH_SETS overrides).
size_t max_scratch_sets() {
    static const size_t v = [] {
        const char* e = std::getenv("PBF_SCRATCH_SETS");
        const int x = e ? std::atoi(e) : 0;
        return x > 0 ? size_t(x) : size_t(8);
    }();
    return v;
}

}  // namespace

struct alignas(128) pbf_filter {
    // The fields a per-key probe reads (or writes) of every filter it tests, together in the first
    // 128 bytes (two lines of each filter instead of four; measured neutral for a 16-filter get,
    // tools/diag/get_stage_check.py, kept as the layout the per-key path reads).
    //
    // Writers (builds, from_bytes, batch probes: anything that touches the handle's state or
    // queues work on its stream) hold mu exclusively; one-key probes of a built filter hold it
    // shared and run on a reader stream, so concurrent readers do not queue behind each other
    // (the reference's get probes a published filter from any thread, lsm_storage.py:153-179).
    std::shared_mutex mu;
    int device = 0;
    uint32_t k = 0;
    std::atomic<uint32_t> svc_id{0};  // index in the device reader's descriptor table (0: none yet)
    // work may be queued on the stream since its last completed wait; set by writers (lock held
    // exclusively), cleared by a wait or by a reader whose stream query found the stream drained
    // (lock held shared: concurrent readers may clear it together, hence atomic)
    std::atomic<bool> pending{false};
    bool pristine = true;  // logically all-zero; reachable words not yet materialised
    std::atomic<int> last_probe_mode{0};          // (written by concurrent readers too)
    std::atomic<uint32_t> last_probe_detail{0};   // PBF_DETAIL_* of the last probe
    uint32_t* bitmap = nullptr;
    IndexMap im{};
    // the rest
    hipStream_t stream = nullptr;
    uint64_t nb_bytes = 0;
    uint64_t words = 0;  // logical words ceil(nb_bytes / 4)
    uint64_t alloc_words = 0;
    bool middle_dirty = false;  // m > 2^32: unreachable middle written by set_bitmap
    int mode = PBF_BUILD_AUTO;
    int last_mode = 0;
    TileMap tm{};
    bool tiled_ok = false;
    int probe_mode = PBF_PROBE_AUTO;
    uint32_t last_build_detail = 0;  // PBF_DETAIL_* | (kps / 256) << 12 of the last tiled build
    Scratch* sc = nullptr;           // leased for the current call
    bool spare_cu = false;           // the current tiled call plans around a resident reader (groups_cap)
    uint64_t* dpop = nullptr;
    hipEvent_t ev = nullptr;       // stream joins of multi-filter probes
    hipEvent_t wait_ev = nullptr;  // pbf_wait_stream: the caller's stream -> this stream
    hipEvent_t sig_ev = nullptr;   // pbf_signal_stream: this stream -> the caller's stream
    const char* last_kernel = "";  // the last kernel enqueued on the stream (wait_stream's report)
};
static_assert(offsetof(pbf_filter, im) + sizeof(IndexMap) <= 128, "per-key fields in the first 128 bytes");

namespace {

int enter(pbf_filter_t* f) {
    if (!f) return fail(PBF_ERR_INVALID, "null filter handle");
    HIP_TRY(hipSetDevice(f->device));
    return PBF_OK;
}

// hipEventQuery / hipStreamQuery report "not ready" as an error code, and HIP keeps it as the
// thread's last error; the launch checks (hipGetLastError) must not see it.
bool event_done(hipEvent_t e) {
    const hipError_t r = hipEventQuery(e);
    if (r != hipSuccess) (void)hipGetLastError();
    return r == hipSuccess;
}

// Bitmap allocations (bitmap words + the popcount slot) are recycled per device and size:
// an LSM creates a filter per flushed / compacted SSTable and drops it with the SSTable, and a
// hipMalloc + hipFree pair cost milliseconds per filter.  At most PBF_BITMAP_CACHE_MB (default
// 1024) of freed bitmaps are kept; pbf_trim releases them.
size_t bitmap_alloc_bytes(uint64_t alloc_words) { return size_t(alloc_words) * 4 + 16; }

struct BitmapCache {
    std::mutex mu;
    std::map<std::pair<int, size_t>, std::vector<void*>> free;
    std::map<void*, bool> from_pool;  // allocation -> came from hipMallocAsync
    size_t bytes = 0;
};

void bitmap_free_now(BitmapCache& c, void* p) {  // c.mu held
    auto it = c.from_pool.find(p);
    const bool pooled = it != c.from_pool.end() && it->second;
    if (it != c.from_pool.end()) c.from_pool.erase(it);
    if (pooled) {
        (void)hipFreeAsync(p, nullptr);
        (void)hipStreamSynchronize(nullptr);
    } else {
        (void)hipFree(p);
    }
}
BitmapCache& bitmap_cache() {
    static BitmapCache c;
    return c;
}
size_t bitmap_cache_cap() {
    static const size_t v = [] {
        const char* e = std::getenv("PBF_BITMAP_CACHE_MB");
        const long long x = e ? std::atoll(e) : -1;
        return x >= 0 ? size_t(x) << 20 : size_t(1024) << 20;
    }();
    return v;
}

// A miss allocates from the device's stream-ordered memory pool (hipMallocAsync, with the
// pool's release threshold raised so freed blocks stay in it): a plain hipMalloc of a 1.8 MB
// bitmap measured ~10 ms on the box; the pool suballocates.
hipError_t bitmap_alloc(int device, size_t bytes, void** out, hipStream_t stream) {
    BitmapCache& c = bitmap_cache();
    {
        std::lock_guard<std::mutex> lock(c.mu);
        auto it = c.free.find({device, bytes});
        if (it != c.free.end() && !it->second.empty()) {
            *out = it->second.back();
            it->second.pop_back();
            c.bytes -= bytes;
            return hipSuccess;
        }
    }
    static std::mutex mu;
    static std::map<int, bool> pool_ok;
    bool use_pool;
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = pool_ok.find(device);
        if (it == pool_ok.end()) {
            hipMemPool_t pool = nullptr;
            bool ok = hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess;
            if (ok) {
                uint64_t keep = ~uint64_t(0);
                ok = hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep) == hipSuccess;
            }
            if (!ok) (void)hipGetLastError();
            it = pool_ok.emplace(device, ok).first;
        }
        use_pool = it->second;
    }
    if (use_pool) {
        if (hipMallocAsync(out, bytes, stream) == hipSuccess) {
            std::lock_guard<std::mutex> lock(c.mu);
            c.from_pool[*out] = true;
            return hipSuccess;
        }
        (void)hipGetLastError();
    }
    return hipMalloc(out, bytes);
}

// The caller has synchronised the filter's stream (no queued work reads the buffer).
void bitmap_release(int device, size_t bytes, void* p) {
    BitmapCache& c = bitmap_cache();
    {
        std::lock_guard<std::mutex> lock(c.mu);
        if (c.bytes + bytes <= bitmap_cache_cap()) {
            c.free[{device, bytes}].push_back(p);
            c.bytes += bytes;
            return;
        }
        bitmap_free_now(c, p);
    }
}

void bitmap_cache_trim(int device) {
    BitmapCache& c = bitmap_cache();
    std::lock_guard<std::mutex> lock(c.mu);
    for (auto& kv : c.free) {
        if (kv.first.first != device) continue;
        for (void* p : kv.second) {
            bitmap_free_now(c, p);
            c.bytes -= kv.first.second;
        }
        kv.second.clear();
    }
}

// Streams are per device, dealt round-robin to filters (PBF_STREAMS, default 8), so filters
// built or probed together (C4's eight) run on distinct streams, while filters sharing a
// stream only order their work.  Creating a HIP stream costs 3-15 ms
// (profiles/r02/s9/create_in_flush.txt): the whole set is created at a device's first filter
// (which also pays the runtime's start-up), not one per early SSTable.
hipError_t pooled_stream(int device, hipStream_t* out) {
    static std::mutex mu;
    static std::map<int, std::pair<std::vector<hipStream_t>, size_t>> pools;
    static const size_t nstreams = [] {
        const char* e = std::getenv("PBF_STREAMS");
        const int x = e ? std::atoi(e) : 0;
        return x > 0 ? size_t(std::min(x, 64)) : size_t(8);
    }();
    std::lock_guard<std::mutex> lock(mu);
    auto& pool = pools[device];
    while (pool.first.size() < nstreams) {
        hipStream_t st = nullptr;
        const hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        if (e != hipSuccess) {
            if (pool.first.empty()) return e;
            (void)hipGetLastError();  // fewer streams than asked for: share the ones there are
            break;
        }
        pool.first.push_back(st);
        register_stream(device, st);
    }
    *out = pool.first[pool.second++ % pool.first.size()];
    return hipSuccess;
}

// Lease a scratch set of f's device for work enqueued on f's stream (RAII).  Prefers a set
// whose previous work is done or was on this same stream; creates one while fewer than
// max_scratch_sets() exist; otherwise takes a free set and orders this stream after its
// previous user.
class Lease {
   public:
    Lease(pbf_filter_t* f) : f_(f) {}
    int acquire() {
        DevicePool& pool = device_pool(f_->device);
        Scratch* pick = nullptr;
        {
            std::lock_guard<std::mutex> lock(pool.mu);
            Scratch* any = nullptr;
            for (Scratch* s : pool.sets) {
                if (s->leased) continue;
                if (!any) any = s;
                if (!s->last || s->last_stream == f_->stream || event_done(s->last)) {
                    pick = s;
                    break;
                }
            }
            if (!pick && (pool.sets.size() < max_scratch_sets() || !any)) {
                pick = new Scratch();
                pool.sets.push_back(pick);
            }
            if (!pick) pick = any;
            pick->leased = true;
        }
        s_ = pick;
        if (!s_->last) HIP_TRY(hipEventCreateWithFlags(&s_->last, hipEventDisableTiming));
        if (s_->last_stream && s_->last_stream != f_->stream) HIP_TRY(hipStreamWaitEvent(f_->stream, s_->last, 0));
        f_->sc = s_;
        return PBF_OK;
    }
    ~Lease() {
        if (!s_) return;
        // stream-order the set's next user after everything this call enqueued
        if (hipEventRecord(s_->last, f_->stream) == hipSuccess) s_->last_stream = f_->stream;
        f_->sc = nullptr;
        DevicePool& pool = device_pool(f_->device);
        std::lock_guard<std::mutex> lock(pool.mu);
        s_->leased = false;
    }

   private:
    pbf_filter_t* f_;
    Scratch* s_ = nullptr;
};

#define LEASE(f)                        \
    Lease lease_(f);                    \
    do {                                \
        int lrc_ = lease_.acquire();    \
        if (lrc_) return lrc_;          \
    } while (0)

// Bring a pristine bitmap to its explicit all-zero form (before atomics / reads).
int materialise(pbf_filter_t* f) {
    if (!f->pristine) return PBF_OK;
    f->pending = true;
    HIP_TRY(hipMemsetAsync(f->bitmap, 0, f->alloc_words * 4, f->stream));
    f->pristine = false;
    return PBF_OK;
}

struct Batch {
    KeySet ks;
    int km;
    uint64_t n;
};

Batch make_batch(const uint8_t* keys, const uint64_t* offsets, uint32_t key_len, uint64_t n) {
    Batch b{};
    b.ks.data = keys;
    b.ks.offsets = offsets;
    b.ks.off0 = offsets;
    b.ks.key_len = key_len;
    b.n = n;
    if (offsets)
        b.km = kVar;
    else if (key_len == 16 && (reinterpret_cast<uintptr_t>(keys) & 15) == 0)
        b.km = kFixed16;
    else
        b.km = kFixedN;
    return b;
}

// Keys [i0, i0 + n) of a batch (offsets stay relative to off0, so a slice needs no rebasing).
Batch slice(const Batch& b, uint64_t i0, uint64_t n) {
    Batch c = b;
    c.n = n;
    if (b.km == kVar)
        c.ks.offsets = b.ks.offsets + i0;
    else
        c.ks.data = b.ks.data + i0 * b.ks.key_len;
    return c;
}

uint32_t grid_for(uint64_t n, uint32_t block, uint32_t cap = 16384) {
    uint64_t g = (n + block - 1) / block;
    return uint32_t(std::max<uint64_t>(1, std::min<uint64_t>(g, cap)));
}

int run_atomic(pbf_filter_t* f, const Batch& b) {
    int rc = materialise(f);
    if (rc) return rc;
    const uint32_t grid = grid_for(b.n, 256);
    dispatch(kmax_for(f->k), b.km, [&](auto KMAX, auto KM) {
        k_build_atomic<decltype(KMAX)::value, decltype(KM)::value>
            <<<grid, 256, 0, f->stream>>>(b.ks, b.n, int(f->k), f->im, f->bitmap);
    });
    LAUNCHED(f, "k_build_atomic");
    return PBF_OK;
}

// Geometry of the partition pass for a batch of n keys (see tiled_kernels.hpp).
struct PartPlan {
    PartGeom pg;
    bool pk3;           // counting-sort build with packed entries (k_part / k_tile_build PK3)
    size_t lds_part;
    size_t lds_gather;  // probes: per gather workgroup
    uint32_t gsplit;    // probes: gather splits over tile ranges (grid G x gsplit)
    uint32_t gtq;       // ring gather: quad-table bytes per tile (0 = binary search)
};

// Partition strategy: PBF_PART=sort|ring|sort_build forces one (tests, measurements); default auto.
int part_override() {
    static const int v = [] {
        const char* e = std::getenv("PBF_PART");
        if (!e) return 0;
        if (!std::strcmp(e, "sort")) return 1;
        if (!std::strcmp(e, "ring")) return 2;
        if (!std::strcmp(e, "sort_build")) return 3;  // counting sort for builds only
        return 0;
    }();
    return v;
}

// Ring partition (ring_kernels.hpp) when there are many tiles: a 1024-key sub-chunk then puts
// only a few positions into each tile (<= GS/2 = 8 on average), which is what the ring's 16-entry
// groups need, while the counting-sort partition's per-tile runs get too short to write well.
// The 32-entry rings of B tiles take B * 128 B of LDS: up to 1024 tiles.  (Rings for more tiles
// — super-tiles of 2^sb tiles, or 16-entry rings — measured slower than the counting sort for
// C3 / C4 and were removed: profiles/r02/s2, profiles/r02/s9.)
bool ring_pow2(const TileMap& tm) { return tm.im.mode == kPow2 && !tm.cspace; }

// Keys per sub-chunk of a ring partition of B tiles and k hashes (0 = the ring does not apply):
// the largest of 1024 / 512 / 256 with kps * k <= B * GS / 2.  Probes keep 1024 (the entry's
// thread field), builds may take smaller sub-chunks (k = 10 over 1024 tiles: 512).
uint32_t ring_kps(uint32_t B, uint32_t k, bool probe, uint32_t tb) {
    const int ov = part_override();
    if (ov == 1 || (ov == 3 && !probe) || k == 0 || k > 16 || B > 1024 || (probe && tb > kSlotShift)) return 0;
    for (uint32_t kp = kRingKeysPerSub; kp >= (probe ? kRingKeysPerSub : 256u); kp /= 2)
        if (uint64_t(kp) * k * 4 <= uint64_t(B) * kRingEntries) return kp;
    return ov == 2 ? (probe ? kRingKeysPerSub : 256u) : 0u;
}

// Gather LDS = the key bitmap of a partition workgroup + one u16 run-boundary row (`row`
// entries) per tile of the split.  Splits start at gather_splits() and double (up to 64) while
// the workgroup does not fit, so large batches stay in one pipeline.
void set_gather(PartPlan& pl, uint32_t B, uint32_t row, uint32_t nf = 1) {
    const size_t kb = size_t((pl.pg.kpw + 31) / 32) * 4 * nf;  // one key bitmap per fused filter
    uint32_t S = gather_splits();
    auto lds = [&](uint32_t sp) { return kb + size_t((B + sp - 1) / sp) * row * 2 + 16; };
    auto per_cu = [](size_t bytes) { return std::min<size_t>(4, (160 * 1024) / bytes); };  // 512-thread WGs
    while (lds(S) > 156 * 1024 && S < 64 && S < B) S *= 2;
    // more splits while they raise the workgroups per CU (the gather waits on memory; each split
    // ANDs its key words into hw once): C3 (4096 tiles, 65 boundary counts per tile) 8 -> 32
    // splits, probe 14.42 -> 13.40 ms; C2 / C5 keep 8 (profiles/r03/s12)
    while (S < 32 && S < B && per_cu(lds(2 * S)) > per_cu(lds(S))) S *= 2;
    pl.gsplit = S;
    pl.lds_gather = lds(S);
    pl.gtq = 0;
    // the ring gather's quad table, when groups fit a byte and the workgroup stays small enough
    // for 4 per CU (measured neutral against the binary search, kept for the shorter path:
    // profiles/r02/s3/gsweep_*)
    if (row <= 255) {
        const uint32_t tq = pl.pg.cap / 4;
        const size_t with = ((pl.lds_gather + 3) & ~size_t(3)) + size_t((B + S - 1) / S) * tq + 4;
        if (with <= 38 * 1024) {
            pl.gtq = tq;
            pl.lds_gather = with;
        }
    }
}

// Partition workgroups each take a whole CU (all of its LDS).  Workgroups are dealt round-robin
// over the 8 XCDs (32 CUs each): while the device's resident one-key reader holds a CU slot
// (reader_service.hpp), 256 workgroups put 32 on its XCD, and one of them waits for a second
// round.  `spare`: plan for 31 per XCD then.
uint64_t groups_cap(bool sort_probe, bool spare) {
    const uint64_t g = part_max_groups(sort_probe);
    return spare && g >= 256 ? g / 256 * 248 : g;
}

PartPlan plan_ring_g(uint32_t B, uint32_t k, uint64_t n, uint32_t kps, bool probe, double share, uint32_t nf,
                     uint64_t gcap) {
    PartPlan pl{};
    const uint64_t G0 = std::min<uint64_t>(gcap, std::max<uint64_t>(1, (n + kps - 1) / kps));
    uint64_t kpw = (n + G0 - 1) / G0;
    kpw = ((kpw + kps - 1) / kps) * kps;
    pl.pg.G = uint32_t(std::max<uint64_t>(1, (n + kpw - 1) / kpw));
    pl.pg.kps = kps;
    pl.pg.kpw = kpw;
    pl.pg.nsub = uint32_t(kpw / kps);
    pl.pg.nq = uint32_t((kpw + kGroupKeys - 1) / kGroupKeys);
    pl.pg.ring = kRingEntries;
    const double mu = double(kpw) * k * share;
    const uint64_t cap = uint64_t(mu + 8.0 * std::sqrt(mu) + 32.0);
    pl.pg.cap = uint32_t(((cap + 31) / 32) * 32);
    // the rest of the CU's 160 KiB of LDS (up to 4096 entries) buffers spilled positions
    const size_t ring_bytes = size_t(ring_lds_words(B)) * 4, spill_entry = probe ? 8 : 4;
    pl.pg.spill_cap = uint32_t(std::min<size_t>(4096, (size_t(kRingLdsWords) * 4 - ring_bytes) / spill_entry));
    pl.lds_part = 0;  // k_part_ring declares the CU's whole LDS statically (kRingLdsWords)
    set_gather(pl, B, pl.pg.nq + 1, nf);
    return pl;
}

// A multi-filter probe's gather keeps one key bitmap per filter of its partition workgroup's keys
// in LDS, which caps a pipeline at ~33M keys with one workgroup per CU (C5's 100M keys: 3
// pipelines, each streaming every filter's bitmap through the set tile test).  So while the
// gather does not fit, a multi-filter probe plans 2, 3 or 4 rounds of partition workgroups
// (smaller key bitmaps, one pipeline for the batch); the tile test's per-word table then walks
// the regions in chunks (PartGeom::tabw).
PartPlan plan_ring(uint32_t B, uint32_t k, uint64_t n, uint32_t kps, bool probe, double share, uint32_t nf = 1,
                   bool spare = false) {
    const uint64_t gcap = groups_cap(false, spare);
    PartPlan pl = plan_ring_g(B, k, n, kps, probe, share, nf, gcap);
    static const bool g_forced = std::getenv("PBF_PART_G") != nullptr;  // (A/B: the count as given)
    if (probe && nf > 1 && !g_forced) {
        for (uint64_t mult = 2; mult <= 4 && pl.lds_gather > 156 * 1024; ++mult) {
            const PartPlan p2 = plan_ring_g(B, k, n, kps, probe, share, nf, gcap * mult);
            if (p2.pg.G <= pl.pg.G) break;  // (too few keys for more workgroups)
            pl = p2;
        }
    }
    return pl;
}

// The KMAX of the counting-sort kernel with_part_kernel launches for (k, key layout): the
// exact-k variants (6, 8, 10) or the register bucket.
int part_kmax(uint32_t k, int km) {
    if (km != kFixedN && (k == 6 || k == 8 || k == 10)) return int(k);
    return kmax_for(k);
}

// Packed build entries (PBF_PK3=0 disables them, for A/B measurements).
bool pk3_enabled() {
    static const bool v = [] {
        const char* e = std::getenv("PBF_PK3");
        return !(e && e[0] == '0');
    }();
    return v;
}

PartPlan plan_partition(uint32_t B, uint32_t k, int km, uint64_t n, bool probe, double share, uint32_t nf,
                        bool spare = false) {
    PartPlan pl{};
    const size_t per_entry = probe ? 6 : 4;  // stage u32 (+ u16 tile id for probes)
    const size_t fixed = size_t(3 * B + 1 + 16) * 4;
    const uint64_t smax = (156 * 1024 - fixed) / per_entry;  // stage entries the LDS holds
    // keys per thread per sub-chunk: as many as the registers allow (part_kpt), placed in at most
    // two windows of the stage
    uint64_t kpt = uint64_t(part_kpt(part_kmax(k, km), km, probe));
    // (and k_part keeps ranks and slots as 16-bit halves: kps * k + pads < 2^16)
    while (kpt > 1 && (kpt * kPartThreads * k > 2 * smax || kpt * kPartThreads * k + 2 * std::min<uint64_t>(B, kpt * kPartThreads * k) >= 65536)) --kpt;
    // probe sub-chunks tile the 4096-key groups of the entry format: 1, 2 or 4 keys per thread
    if (probe) kpt = kpt >= 4 ? 4 : (kpt >= 2 ? 2 : 1);
    const uint64_t kps = kpt * kPartThreads;
    // packed build entries (tiled_kernels.hpp PK3) for the exact-k kernels; their runs are padded
    // (<= 2 pad slots per tile)
    pl.pk3 = !probe && pk3_enabled() && km != kFixedN && (k == 6 || k == 8 || k == 10);
    const uint64_t need = kps * k + (pl.pk3 ? 2 * std::min<uint64_t>(B, kps * k) : 0);
    uint64_t scap = std::min(need, smax);
    if (pl.pk3) scap -= scap % 3;  // windows hold whole packed words
    pl.pg.scap = uint32_t(scap);
    pl.lds_part = fixed + size_t(scap) * per_entry;
    const uint64_t G0 = std::min<uint64_t>(groups_cap(probe, spare), std::max<uint64_t>(1, (n + kps - 1) / kps));
    uint64_t kpw = (n + G0 - 1) / G0;
    kpw = ((kpw + kps - 1) / kps) * kps;
    pl.pg.G = uint32_t(std::max<uint64_t>(1, (n + kpw - 1) / kpw));
    pl.pg.kps = uint32_t(kps);
    pl.pg.kpw = kpw;
    pl.pg.nsub = uint32_t(kpw / kps);
    pl.pg.nq = uint32_t((kpw + kGroupKeys - 1) / kGroupKeys);
    const double mu = double(kpw) * k * share;
    const uint64_t cap = uint64_t(mu + 8.0 * std::sqrt(mu) + 32.0);
    // (k_part addresses an entry by a 24-bit multiply-add within its workgroup's regions)
    pl.pg.cap = uint32_t(std::min<uint64_t>(((cap + 31) / 32) * 32, ((uint64_t(1) << 32) - 1) / std::max<uint32_t>(B, 1) & ~uint64_t(31)));
    pl.pg.cap = std::min<uint32_t>(pl.pg.cap, (1u << 24) - 32);
    if (pl.pk3) {
        // + the pads (<= 2 per sub-chunk), in whole 32-word units of 3 entries
        const uint64_t c3 = uint64_t(pl.pg.cap) + 2 * pl.pg.nsub;
        pl.pg.cap = uint32_t(std::min<uint64_t>(((c3 + 95) / 96) * 96, ((1u << 24) - 96) / 96 * 96));
    }
    set_gather(pl, B, pl.pg.nq + 1, nf);
    return pl;
}

// Expected share of one hash in the busiest tile.  The reference's floor-mod of a signed 32-bit
// hash (bloom_filter.py:47) is uniform only for power-of-two m: for m < 2^31 a position has
// 2*floor(2^31/m) or 2*ceil(2^31/m) preimages (the first and last 2^31 mod m positions get the
// extra ones), for 2^31 <= m < 2^32 the overlap [m - 2^31, 2^31) gets 2; above 2^32 the tile
// space is the 2^32 reachable positions, one preimage each.  Region capacity is sized for the
// densest tile so edge tiles of a non-power-of-two filter do not overflow.
double busiest_tile_share(const TileMap& tm) {
    const double tile = double(uint64_t(1) << tm.tb);
    const uint64_t m = tm.im.m;
    double max_pre;
    if (tm.cspace)
        max_pre = 1.0;
    else if (tm.im.mode == kPow2)
        max_pre = 4294967296.0 / double(m);
    else if (m < (uint64_t(1) << 31))
        max_pre = 2.0 * double(((uint64_t(1) << 31) + m - 1) / m);
    else
        max_pre = 2.0;
    return std::min(1.0, max_pre * tile / 4294967296.0);
}

// nf: filters one ring gather serves at once (a multi-filter probe).
// spare: leave a CU per XCD to the resident reader (groups_cap), decided once per call
// (pbf_filter::spare_cu) so a probe's batch split and its pipelines plan alike.
PartPlan plan_for(const TileMap& tm, uint32_t k, int km, uint64_t n, bool probe, uint32_t nf = 1, bool spare = false) {
    const uint32_t B = tm.nbuckets;
    const double share = busiest_tile_share(tm);
    if (const uint32_t kps = ring_kps(B, k, probe, tm.tb)) {
        const PartPlan pl = plan_ring(B, k, n, kps, probe, share, probe ? nf : 1, spare);
        // lim / tail are 16-bit byte counts in LDS (cap <= kRingMaxCap); entry offsets within a
        // workgroup's regions are 32-bit (B * cap < 2^32)
        if (pl.pg.cap <= kRingMaxCap && uint64_t(B) * pl.pg.cap < (uint64_t(1) << 32)) return pl;
    }
    return plan_partition(B, k, km, n, probe, share, probe ? nf : 1, spare);
}

// The ring partition kernel for (k, key layout): with the seed count fixed at compile time
// where it pays (k equal to the register bucket, or k = 6 — C2/C5's k), its k LDS atomics per
// key issue back to back; other k take the runtime-k kernel of their bucket.
template <int KX, int KMD, bool PROBE, class L>
void with_ring_kernel(uint32_t k, bool pow2, L&& launch) {
    if constexpr (KMD != kFixedN) {
        if constexpr (KX == 8) {
            if (k == 6) {
                launch(pow2 ? k_part_ring<6, KMD, PROBE, true, true> : k_part_ring<6, KMD, PROBE, false, true>);
                return;
            }
        }
        if (k == uint32_t(KX)) {
            launch(pow2 ? k_part_ring<KX, KMD, PROBE, true, true> : k_part_ring<KX, KMD, PROBE, false, true>);
            return;
        }
    }
    launch(pow2 ? k_part_ring<KX, KMD, PROBE, true, false> : k_part_ring<KX, KMD, PROBE, false, false>);
}

// The counting-sort partition kernel for (k, key layout): exact-k variants for the k the
// configurations use (6: C2/C5 shapes, 8: C3, 10: the fp = 0.001 product sizing of C4 / SSTables).
template <int KX, int KMD, bool PROBE, class L>
void with_part_kernel(uint32_t k, L&& launch, bool pk3 = false) {
    if constexpr (KMD != kFixedN) {
        if constexpr (KX == 8) {
            if constexpr (!PROBE) {
                if (pk3 && k == 6) return launch(k_part<6, KMD, PROBE, true, true>);
                if (pk3 && k == 8) return launch(k_part<8, KMD, PROBE, true, true>);
            }
            if (k == 6) return launch(k_part<6, KMD, PROBE, true>);
            if (k == 8) return launch(k_part<8, KMD, PROBE, true>);
        }
        if constexpr (KX == 16) {
            if constexpr (!PROBE) {
                if (pk3 && k == 10) return launch(k_part<10, KMD, PROBE, true, true>);
            }
            if (k == 10) return launch(k_part<10, KMD, PROBE, true>);
        }
    }
    launch(k_part<KX, KMD, PROBE>);
}

int run_tiled(pbf_filter_t* f, const Batch& b) {
    const TileMap& tm = f->tm;
    const uint32_t B = tm.nbuckets;
    const uint32_t k = f->k;
    const PartPlan pl = plan_for(tm, k, b.km, b.n, false, 1, f->spare_cu);
    const PartGeom& pg = pl.pg;
    // (+ the ring partition's 64-B dummy line per workgroup after the regions)
    HIP_TRY(f->sc->regions.ensure(size_t(pg.G) * B * pg.cap * 4 + size_t(pg.G) * 64));
    HIP_TRY(f->sc->fill.ensure(size_t(pg.G) * B * 4));
    HIP_TRY(f->sc->ovf.ensure(std::max<uint64_t>(b.n * k, 1) * 4));
    HIP_TRY(f->sc->ovf_count.ensure(64));
    if (!f->sc->ovf_init) {  // two counters, used alternately; each build's k_ovf_build zeroes the other
        HIP_TRY(hipMemsetAsync(f->sc->ovf_count.p, 0, 64, f->stream));
        f->sc->ovf_init = true;
    }
    auto* regions = static_cast<uint32_t*>(f->sc->regions.p);
    auto* fill = static_cast<uint32_t*>(f->sc->fill.p);
    auto* ovf = static_cast<uint32_t*>(f->sc->ovf.p);
    auto* ovf_count = static_cast<uint32_t*>(f->sc->ovf_count.p) + f->sc->ovf_phase;
    uint32_t* ovf_next = static_cast<uint32_t*>(f->sc->ovf_count.p) + (f->sc->ovf_phase ^ 1);
    f->sc->ovf_phase ^= 1;
    hipStream_t s = f->stream;
    const KeySet pks = b.ks;
    hipError_t err = hipSuccess;
    dispatch(kmax_for(k), b.km, [&](auto KMAX, auto KM) {
        if constexpr (decltype(KMAX)::value > 0) {  // tiled path only for k <= 32
            constexpr int KX = decltype(KMAX)::value, KMD = decltype(KM)::value;
            if (pg.ring) {
                if constexpr (KX <= 16) {
                    with_ring_kernel<KX, KMD, false>(k, ring_pow2(tm), [&](auto kern) {
                        err = allow_lds(kern, pl.lds_part);
                        if (err == hipSuccess)
                            kern<<<pg.G, kPartThreads, pl.lds_part, s>>>(b.ks, b.n, int(k), tm, pg, regions, fill,
                                                                 nullptr, ovf, ovf_count, ProbeSet{}, nullptr);
                    });
                }
            } else {
                with_part_kernel<KX, KMD, false>(k, [&](auto kern) {
                    err = allow_lds(kern, pl.lds_part);
                    if (err == hipSuccess)
                        kern<<<pg.G, kPartThreads, pl.lds_part, s>>>(pks, b.n, int(k), tm, pg, regions, fill, nullptr,
                                                             ovf, ovf_count, ProbeSet{}, nullptr);
                }, pl.pk3);
            }
        }
    });
    HIP_TRY(err);
    LAUNCHED(f, pg.ring ? "k_part_ring<build>" : "k_part<build>");
    const size_t lds_tile = ((size_t(1) << tm.tb) / 32 + pg.G) * 4;
    if (pl.pk3) {
        HIP_TRY(allow_lds(k_tile_build<true>, lds_tile));
        k_tile_build<true><<<B, 1024, lds_tile, s>>>(tm, pg, regions, fill, f->bitmap, f->pristine ? 1 : 0);
    } else {
        HIP_TRY(allow_lds(k_tile_build<false>, lds_tile));
        k_tile_build<false><<<B, 1024, lds_tile, s>>>(tm, pg, regions, fill, f->bitmap, f->pristine ? 1 : 0);
    }
    LAUNCHED(f, "k_tile_build");
    f->last_build_detail = (pg.ring ? PBF_DETAIL_RING : PBF_DETAIL_SORT) | (pl.pk3 ? PBF_DETAIL_PACKED : 0u) |
                           ((pg.kps / 256) << 12);
    k_ovf_build<<<256, 256, 0, s>>>(tm, ovf, ovf_count, f->bitmap, ovf_next);
    LAUNCHED(f, "k_ovf_build");
    f->pristine = false;
    return PBF_OK;
}

// Tiled probe of one key batch against nf filters sharing (m, k) (nf = 1: a plain probe).  The
// keys are hashed and partitioned once, on f's stream with f's scratch (f = the set's first
// filter, also for every later group of a large set); the tile test runs once per filter and
// (ring partition) ONE gather serves every filter.  hitmasks[i] + hm_off is filter i's output.
int run_tiled_probe_set(pbf_filter_t* f, pbf_filter_t* const* fs, uint32_t nf, const Batch& b,
                        uint8_t* const* hitmasks, uint64_t hm_off) {
    Scratch* const sc = f->sc;
    const TileMap& tm = f->tm;
    const uint32_t B = tm.nbuckets;
    const uint32_t k = f->k;
    const PartPlan pl = plan_for(tm, k, b.km, b.n, true, nf, f->spare_cu);
    const PartGeom& pg = pl.pg;
    f->last_probe_detail = (pg.ring ? PBF_DETAIL_RING : PBF_DETAIL_SORT) | (nf << 8);
    HIP_TRY(sc->regions.ensure(size_t(pg.G) * B * pg.cap * 4 + size_t(pg.G) * 64));
    HIP_TRY(sc->fill.ensure(size_t(pg.G) * B * 4));
    // both partitions: in-region counts at every 4096-key group boundary
    HIP_TRY(sc->pref.ensure(size_t(pg.G) * B * (pg.nq + 1) * 2));  // u16 (cap < 2^16)
    const size_t r_words = size_t(pg.G) * B * (pg.cap / 32);
    HIP_TRY(sc->rbits.ensure(r_words * 4 * nf));
    const uint64_t neg_words = (b.n + 31) / 32;
    const size_t neg_bytes = neg_words * 4;
    HIP_TRY(sc->neg.ensure(neg_bytes * nf));
    auto* regions = static_cast<uint32_t*>(sc->regions.p);
    auto* fill = static_cast<uint32_t*>(sc->fill.p);
    auto* pref = static_cast<uint16_t*>(sc->pref.p);
    auto* R = static_cast<uint32_t*>(sc->rbits.p);
    auto* neg = static_cast<uint32_t*>(sc->neg.p);
    hipStream_t s = f->stream;
    // gather split over S tile ranges (several small workgroups per CU)
    const uint32_t S = pl.gsplit;
    const bool use_hw = S > 1 || nf > 1;
    uint32_t* hw = nullptr;
    // one filter, whole 32-key words, a 4-byte aligned mask: the gather's ANDed words ARE the
    // LSB-first hit mask (bit i of word w = key 32w + i, little-endian), so it ANDs into the
    // caller's mask directly and no conversion kernel runs
    const bool hw_is_mask = use_hw && nf == 1 && b.n % 32 == 0 &&
                            (reinterpret_cast<uintptr_t>(hitmasks[0] + hm_off) & 3) == 0;
    if (hw_is_mask) {
        hw = reinterpret_cast<uint32_t*>(hitmasks[0] + hm_off);
    } else if (use_hw) {
        HIP_TRY(sc->hw.ensure(neg_bytes * nf));
        hw = static_cast<uint32_t*>(sc->hw.p);
    }
    ProbeSet ps{};
    ps.nf = nf;
    ps.neg = neg;
    ps.neg_stride = neg_words;
    for (uint32_t i = 0; i < nf; ++i) ps.bm[i] = fs[i]->bitmap;
    size_t lds_tile = ((size_t(1) << tm.tb) / 32 + 2 * pg.G + 1 + 16) * 4;
    // the tile test's per-word table: the u32 global word index per word (TAB 2), else a u16 of
    // region << wsh | word-in-region (TAB 1: when both fit 16 bits and region * B + tile 24
    // bits), else a binary search (TAB 0)
    const uint32_t wpr = pg.cap / 32;
    const size_t table_words = size_t(pg.G) * wpr;
    const uint32_t wsh = 32u - uint32_t(__builtin_clz(std::max(wpr, 2u) - 1u));
    const bool tab1_fits = (uint64_t(pg.G - 1) << wsh) < 65536 && uint64_t(pg.G) * B < (uint64_t(1) << 24);
    // TAB 1 in chunks of whole regions when the whole table does not fit beside the tile (at
    // least one region's words per chunk)
    const size_t tab1_room = lds_tile < 160 * 1024 ? (160 * 1024 - lds_tile) / 2 & ~size_t(1) : 0;
    const int tab = lds_tile + table_words * 4 <= 160 * 1024 ? 2 : (tab1_fits && tab1_room >= wpr ? 1 : 0);
    PartGeom tpg = pg;  // (the tile test's copy: tabw)
    tpg.tabw = tab == 1 && table_words > tab1_room ? uint32_t(tab1_room) : 0u;
    lds_tile += tab == 2 ? table_words * 4 : (tab == 1 ? (tpg.tabw ? size_t(tpg.tabw) : table_words) * 2 : 0);
    // a region word's global index (region * cap/32 + word) is 32-bit
    if (uint64_t(pg.G) * B * (pg.cap / 32) >= (uint64_t(1) << 32)) return fail(PBF_ERR_INVALID, "probe scratch too large");
    auto tprobe = tab == 2 ? k_tile_probe<2> : (tab == 1 ? k_tile_probe<1> : k_tile_probe<0>);
    auto tprobe_set = tab == 2 ? k_tile_probe_set<2> : (tab == 1 ? k_tile_probe_set<1> : k_tile_probe_set<0>);
    HIP_TRY(allow_lds(tprobe, lds_tile));
    // the partition zeroes neg (and presets hw for the gather) itself
    const KeySet pks = b.ks;
    hipError_t err = hipSuccess;
    dispatch(kmax_for(k), b.km, [&](auto KMAX, auto KM) {
        if constexpr (decltype(KMAX)::value > 0) {
            constexpr int KX = decltype(KMAX)::value, KMD = decltype(KM)::value;
            if (pg.ring) {
                if constexpr (KX <= 16) {
                    with_ring_kernel<KX, KMD, true>(k, ring_pow2(tm), [&](auto kern) {
                        err = allow_lds(kern, pl.lds_part);
                        if (err == hipSuccess)
                            kern<<<pg.G, kPartThreads, pl.lds_part, s>>>(b.ks, b.n, int(k), tm, pg, regions, fill, pref,
                                                                 nullptr, nullptr, ps, use_hw ? hw : nullptr);
                    });
                }
            } else {
                with_part_kernel<KX, KMD, true>(k, [&](auto kern) {
                    err = allow_lds(kern, pl.lds_part);
                    if (err == hipSuccess)
                        kern<<<pg.G, kPartThreads, pl.lds_part, s>>>(pks, b.n, int(k), tm, pg, regions, fill, pref,
                                                             nullptr, nullptr, ps, use_hw ? hw : nullptr);
                });
            }
        }
    });
    HIP_TRY(err);
    LAUNCHED(f, pg.ring ? "k_part_ring<probe>" : "k_part<probe>");
    const dim3 grid(pg.G, S);
    auto gather = nf > 1 ? k_gather_ring<kMaxProbeSet> : k_gather_ring<1>;
    HIP_TRY(allow_lds(gather, pl.lds_gather));
    // every filter's tile test (one XCD-aware launch for a set), then ONE gather over the shared
    // region entries
    if (nf == 1) {
        tprobe<<<B, 1024, lds_tile, s>>>(tm, tpg, regions, fill, fs[0]->bitmap, R);
    } else {
        HIP_TRY(allow_lds(tprobe_set, lds_tile));
        const uint32_t tgrid = ((B + 7) / 8) * 8 * nf;
        tprobe_set<<<tgrid, 1024, lds_tile, s>>>(tm, tpg, regions, fill, ps, R, r_words);
    }
    LAUNCHED(f, nf == 1 ? "k_tile_probe" : "k_tile_probe_set");
    // the set gather: 1024 threads when its LDS admits one workgroup per CU (C5's 8 key bitmaps)
    const uint32_t gthreads = nf > 1 && pl.lds_gather > 80 * 1024 ? 1024 : 512;
    gather<<<grid, gthreads, pl.lds_gather, s>>>(tm, pg, b.n, regions, R, fill, pref, neg, hitmasks[0] + hm_off, hw, nf,
                                           r_words, neg_words, pl.gtq);
    LAUNCHED(f, "k_gather_ring");
    if (use_hw && !hw_is_mask) {  // every filter's hit mask in one launch
        HitMasks hms{};
        for (uint32_t i = 0; i < nf; ++i) hms.hm[i] = hitmasks[i] + hm_off;
        const dim3 hgrid(std::max<uint32_t>(1, grid_for(neg_words, 256, 4096) / nf), nf);
        k_hw_to_hitmask<<<hgrid, 256, 0, s>>>(hw, neg_words, b.n, hms);
        LAUNCHED(f, "k_hw_to_hitmask");
    }
    return PBF_OK;
}

int run_tiled_probe(pbf_filter_t* f, const Batch& b, uint8_t* hitmask) {
    pbf_filter_t* fs[1] = {f};
    uint8_t* outs[1] = {hitmask};
    return run_tiled_probe_set(f, fs, 1, b, outs, 0);
}

// The partition pass needs its tile counters plus a stage of one key per thread in LDS.
bool part_fits(uint32_t B, uint32_t k, bool probe) {
    return size_t(3 * B + 17) * 4 + size_t(kPartThreads) * k * (probe ? 6 : 4) <= 156 * 1024;
}

bool want_tiled(pbf_filter_t* f, uint64_t n) {
    if (!f->tiled_ok || f->k == 0 || f->k > 32 || !part_fits(f->tm.nbuckets, f->k, false)) return false;
    if (f->mode == PBF_BUILD_TILED) return true;
    if (f->mode == PBF_BUILD_ATOMIC) return false;
    const uint64_t npos = n * f->k;
    // the tile pass streams the whole bitmap once (twice when not pristine); a random atomic
    // costs ~16x a streamed position.  Tiles win once positions are a small fraction of it.
    const uint64_t bitmap_bytes = f->words * 4 * (f->pristine ? 1 : 2);
    return npos >= (uint64_t(1) << 16) && npos * 64 >= bitmap_bytes;
}

bool want_tiled_probe(pbf_filter_t* f, uint64_t n) {
    if (!f->tiled_ok || f->k == 0 || f->k > 32 || f->tm.tb > kSlotShift || !part_fits(f->tm.nbuckets, f->k, true))
        return false;
    if (f->probe_mode == PBF_PROBE_TILED) return true;
    if (f->probe_mode == PBF_PROBE_DIRECT) return false;
    // direct: ~1..k random 64-B requests per key, cheap while the bitmap stays in one XCD's
    // 4 MiB L2; tiled: ~16 streamed bytes per position + one pass over the bitmap.
    const uint64_t npos = n * f->k;
    return f->words * 4 > (uint64_t(8) << 20) && npos >= (uint64_t(1) << 20) && npos * 16 >= f->words * 4;
}

// Largest probe batch one tiled pipeline takes: the gather keeps a u16 run-boundary table
// (B x (nq+1), one row per 4096-key group) and a bit per key of its workgroup in LDS, and
// positions stay u32.
// Keys per tiled-probe pipeline for a batch of `total` keys: the largest batch whose gather
// workgroup fits the LDS (halving, then a search between the last two sizes in 64Ki-key steps),
// then the batch split into equal pipelines (C5's 100M keys: 3 x 33.3M instead of 4 x 22.4M +
// 10.4M — every pipeline streams the filters' bitmaps once, however few keys it holds).
uint64_t tiled_probe_batch(pbf_filter_t* f, int km, uint32_t nf, uint64_t total) {
    const uint32_t k = f->k;
    auto fits = [&](uint64_t m) {
        const PartPlan pl = plan_for(f->tm, k, km, m, true, nf, f->spare_cu);
        // the tile test addresses a region word by a u32 global index (run_tiled_probe_set)
        return pl.lds_gather <= 156 * 1024 && pl.pg.cap <= 65535 &&
               uint64_t(pl.pg.G) * f->tm.nbuckets * (pl.pg.cap / 32) < (uint64_t(1) << 32);
    };
    const uint64_t top = std::max<uint64_t>(64, (kMaxProbePositions / k) & ~uint64_t(63));
    uint64_t n = top;
    while (n > 64 * 1024 && !fits(n)) n = std::max<uint64_t>(64 * 1024, (n / 2) & ~uint64_t(63));
    if (n < top && n >= 64 * 1024) {
        uint64_t lo = n, hi = std::min<uint64_t>(2 * n, top);
        while (hi - lo > 65536) {
            const uint64_t mid = ((lo + hi) / 2) & ~uint64_t(65535);
            if (mid <= lo) break;
            (fits(mid) ? lo : hi) = mid;
        }
        n = lo;
    }
    if (total > n) {  // equal pipelines, each a multiple of 64 keys (whole hit-mask words)
        const uint64_t np = (total + n - 1) / n;
        n = std::min<uint64_t>(n, (((total + np - 1) / np) + 63) & ~uint64_t(63));
    }
    return n;
}

int add_device(pbf_filter_t* f, const Batch& b) {
    if (b.n == 0 || f->k == 0) return PBF_OK;
    if (want_tiled(f, b.n)) {
        f->spare_cu = resident_live(f->device);
        // positions are counted in u32 inside one pipeline, and a region holds < 2^24 entries
        // (the partitions' 24-bit region addressing): batch very large inputs
        const double share = busiest_tile_share(f->tm);
        const double cap_keys = double((1u << 24) - 64) * part_max_groups(false) / (double(f->k) * share * 1.25);
        const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(kMaxPositions / f->k, uint64_t(cap_keys)));
        for (uint64_t i0 = 0; i0 < b.n; i0 += per) {
            int rc = run_tiled(f, slice(b, i0, std::min<uint64_t>(per, b.n - i0)));
            if (rc) return rc;
        }
        f->last_mode = PBF_BUILD_TILED;
        return PBF_OK;
    }
    f->last_mode = PBF_BUILD_ATOMIC;
    return run_atomic(f, b);
}

int probe_device(pbf_filter_t* f, const Batch& b, uint8_t* hitmask_dev) {
    if (b.n == 0) return PBF_OK;
    int rc = materialise(f);
    if (rc) return rc;
    if (want_tiled_probe(f, b.n)) {
        f->spare_cu = resident_live(f->device);
        const uint64_t per = tiled_probe_batch(f, b.km, 1, b.n);
        for (uint64_t i0 = 0; i0 < b.n; i0 += per) {
            rc = run_tiled_probe(f, slice(b, i0, std::min<uint64_t>(per, b.n - i0)), hitmask_dev + i0 / 8);
            if (rc) return rc;
        }
        f->last_probe_detail |= uint32_t(std::min<uint64_t>((b.n + per - 1) / per, 4095)) << 16;
        f->last_probe_mode = PBF_PROBE_TILED;
        return PBF_OK;
    }
    const uint32_t grid = grid_for(b.n, 256, 1u << 20);
    dispatch(kmax_for(f->k), b.km, [&](auto KMAX, auto KM) {
        k_probe<decltype(KMAX)::value, decltype(KM)::value>
            <<<grid, 256, 0, f->stream>>>(b.ks, b.n, int(f->k), f->im, f->bitmap, hitmask_dev, kProbeStage1);
    });
    LAUNCHED(f, "k_probe");
    f->last_probe_mode = PBF_PROBE_DIRECT;
    f->last_probe_detail = 0;
    return PBF_OK;
}

// ---- multi-filter probe (LsmStorage.get over a key batch, src/lsm_storage.py:164-179) ----

hipError_t filter_event(pbf_filter_t* f) {
    if (f->ev) return hipSuccess;
    return hipEventCreateWithFlags(&f->ev, hipEventDisableTiming);
}

// One pipeline serves the whole set when every filter has fs[0]'s (nb_bytes, k) and the tiled
// probe is what fs[0] would pick for this batch (a filter pinned to the direct probe opts out).
bool shared_probe(pbf_filter_t* const* fs, uint32_t nf, uint64_t n) {
    for (uint32_t i = 1; i < nf; ++i)
        if (fs[i]->nb_bytes != fs[0]->nb_bytes || fs[i]->k != fs[0]->k || fs[i]->probe_mode == PBF_PROBE_DIRECT)
            return false;
    return want_tiled_probe(fs[0], n);
}

// Filters of a set that take the fused direct probe (k_probe_set): those whose own probe would be
// the direct one for this batch (small filters: an LSM's SSTables of a few MB), grouped by k.
bool set_direct(pbf_filter_t* f, uint64_t n) {
    return kmax_for(f->k) > 0 && (f->probe_mode == PBF_PROBE_DIRECT || !want_tiled_probe(f, n));
}

// The 8 XCD slots of one k_probe_set launch (set_kernels.hpp): with nf <= 8 filters, slot x
// takes filter x % nf and 1/(slots of that filter) of the keys; with more, the filters are dealt
// largest first onto the slot with the fewest bitmap bytes so far, each slot all the keys.
XcdPlan plan_xcd(const std::vector<pbf_filter_t*>& grp, size_t g0, uint32_t nf) {
    XcdPlan xp{};
    if (nf <= 8) {
        uint32_t at = 0;
        for (uint32_t f = 0; f < nf; ++f) {
            const uint32_t parts = 8 / nf + (f < 8 % nf ? 1u : 0u);
            for (uint32_t p = 0; p < parts; ++p) {
                const uint32_t x = f + p * nf;
                xp.first[x] = uint8_t(at);
                xp.count[x] = 1;
                xp.part[x] = uint8_t(p);
                xp.nparts[x] = uint8_t(parts);
            }
            xp.order[at++] = uint8_t(f);
        }
        return xp;
    }
    std::vector<uint32_t> idx(nf);
    for (uint32_t f = 0; f < nf; ++f) idx[f] = f;
    std::stable_sort(idx.begin(), idx.end(),
                     [&](uint32_t a, uint32_t b) { return grp[g0 + a]->nb_bytes > grp[g0 + b]->nb_bytes; });
    std::vector<std::vector<uint32_t>> slot(8);
    uint64_t load[8] = {};
    for (uint32_t f : idx) {
        const int x = int(std::min_element(load, load + 8) - load);
        slot[x].push_back(f);
        load[x] += grp[g0 + f]->nb_bytes;
    }
    uint32_t at = 0;
    for (int x = 0; x < 8; ++x) {
        xp.first[x] = uint8_t(at);
        xp.count[x] = uint8_t(slot[x].size());
        xp.part[x] = 0;
        xp.nparts[x] = 1;
        for (uint32_t f : slot[x]) xp.order[at++] = uint8_t(f);
    }
    return xp;
}

// One launch of k_probe_set per (k, up to 64 filters).
int probe_set_direct(pbf_filter_t* f0, std::vector<pbf_filter_t*>& grp, std::vector<uint8_t*>& hms, const Batch& b) {
    const uint32_t k = grp[0]->k;
    for (size_t g0 = 0; g0 < grp.size(); g0 += kMaxFilterSet) {
        FilterSet fset{};
        fset.nf = uint32_t(std::min<size_t>(kMaxFilterSet, grp.size() - g0));
        for (uint32_t i = 0; i < fset.nf; ++i) {
            fset.bm[i] = grp[g0 + i]->bitmap;
            fset.im[i] = grp[g0 + i]->im;
            fset.hm[i] = hms[g0 + i];
        }
        const XcdPlan xp = plan_xcd(grp, g0, fset.nf);
        // 8 slots x up to 512 workgroups of 256 keys
        const uint32_t grid = 8 * grid_for((b.n + 7) / 8, 256, 512);
        dispatch(kmax_for(k), b.km, [&](auto KMAX, auto KM) {
            if constexpr (decltype(KMAX)::value > 0)
                k_probe_set<decltype(KMAX)::value, decltype(KM)::value>
                    <<<grid, 256, 0, f0->stream>>>(b.ks, b.n, int(k), fset, xp);
        });
        LAUNCHED(f0, "k_probe_set");
    }
    for (pbf_filter_t* f : grp) {
        f->last_probe_mode = PBF_PROBE_DIRECT;
        f->last_probe_detail = PBF_DETAIL_SET | (uint32_t(std::min<size_t>(grp.size(), kMaxFilterSet)) << 8);
    }
    return PBF_OK;
}

// Device keys / hit masks; asynchronous on fs[0]'s stream.  Every other filter's stream first
// hands its pending work (a build, a from_bytes) to fs[0]'s stream and afterwards waits for the
// probe, so later calls on any handle are ordered after it.
//   * every filter of one (nb_bytes, k), tiled: ONE partition for the set (run_tiled_probe_set);
//   * otherwise the filters whose own probe would be direct go through k_probe_set, grouped by
//     k (mixed sizes: each key hashed once for the group), and the rest (large filters of
//     distinct sizes) each through its own pipeline on fs[0]'s stream.
int probe_multi_device(pbf_filter_t* const* fs, uint32_t nf, const Batch& b, uint8_t* const* hitmasks) {
    pbf_filter_t* f0 = fs[0];
    hipStream_t s0 = f0->stream;
    int rc = materialise(f0);
    if (rc) return rc;
    HIP_TRY(filter_event(f0));
    for (uint32_t i = 1; i < nf; ++i) {
        pbf_filter_t* fi = fs[i];
        rc = materialise(fi);
        if (rc) return rc;
        HIP_TRY(filter_event(fi));
        if (fi->stream != s0) {
            HIP_TRY(hipEventRecord(fi->ev, fi->stream));
            HIP_TRY(hipStreamWaitEvent(s0, fi->ev, 0));
        }
    }
    if (shared_probe(fs, nf, b.n)) {
        f0->spare_cu = resident_live(f0->device);
        const uint64_t per = tiled_probe_batch(f0, b.km, std::min<uint32_t>(nf, kMaxProbeSet), b.n);
        for (uint64_t i0 = 0; i0 < b.n; i0 += per) {
            const Batch c = slice(b, i0, std::min<uint64_t>(per, b.n - i0));
            for (uint32_t g0 = 0; g0 < nf; g0 += kMaxProbeSet) {
                rc = run_tiled_probe_set(f0, fs + g0, std::min<uint32_t>(kMaxProbeSet, nf - g0), c, hitmasks + g0,
                                         i0 / 8);
                if (rc) return rc;
            }
        }
        f0->last_probe_detail |= uint32_t(std::min<uint64_t>((b.n + per - 1) / per, 4095)) << 16;
        for (uint32_t i = 0; i < nf; ++i) {
            fs[i]->last_probe_mode = PBF_PROBE_TILED;
            fs[i]->last_probe_detail = f0->last_probe_detail.load();
        }
    } else {
        // direct groups by k (in first-appearance order), then the per-filter pipelines
        std::vector<uint32_t> ks;
        std::vector<uint32_t> rest;
        for (uint32_t i = 0; i < nf; ++i) {
            if (!set_direct(fs[i], b.n)) {
                rest.push_back(i);
            } else if (std::find(ks.begin(), ks.end(), fs[i]->k) == ks.end()) {
                ks.push_back(fs[i]->k);
            }
        }
        for (uint32_t k : ks) {
            std::vector<pbf_filter_t*> grp;
            std::vector<uint8_t*> hms;
            for (uint32_t i = 0; i < nf; ++i)
                if (fs[i]->k == k && set_direct(fs[i], b.n)) {
                    grp.push_back(fs[i]);
                    hms.push_back(hitmasks[i]);
                }
            rc = probe_set_direct(f0, grp, hms, b);
            if (rc) return rc;
        }
        if (!rest.empty()) {
            // the large filters of distinct sizes: each its own pipeline on its own stream and
            // scratch set (fs[0] with the caller's lease), after the keys are ready on s0, then
            // joined back into s0
            HIP_TRY(hipEventRecord(f0->ev, s0));
            for (uint32_t i : rest)
                if (fs[i]->stream != s0) HIP_TRY(hipStreamWaitEvent(fs[i]->stream, f0->ev, 0));
            for (uint32_t i : rest) {
                if (i == 0) {
                    rc = probe_device(f0, b, hitmasks[0]);
                } else {
                    Lease li(fs[i]);
                    rc = li.acquire();
                    if (!rc) rc = probe_device(fs[i], b, hitmasks[i]);
                }
                if (rc) return rc;
            }
            for (uint32_t i : rest) {
                if (fs[i]->stream == s0) continue;
                HIP_TRY(hipEventRecord(fs[i]->ev, fs[i]->stream));
                HIP_TRY(hipStreamWaitEvent(s0, fs[i]->ev, 0));
            }
        }
    }
    HIP_TRY(hipEventRecord(f0->ev, s0));
    for (uint32_t i = 1; i < nf; ++i) {
        if (fs[i]->stream != s0) HIP_TRY(hipStreamWaitEvent(fs[i]->stream, f0->ev, 0));
        fs[i]->pending = true;
    }
    return PBF_OK;
}

int hash_device(pbf_filter_t* f, const Batch& b, uint64_t* out_dev) {
    if (b.n == 0 || f->k == 0) return PBF_OK;
    const uint32_t grid = grid_for(b.n, 256);
    dispatch(kmax_for(f->k), b.km, [&](auto KMAX, auto KM) {
        k_hash_indices<decltype(KMAX)::value, decltype(KM)::value>
            <<<grid, 256, 0, f->stream>>>(b.ks, b.n, int(f->k), f->im, out_dev);
    });
    LAUNCHED(f, "k_hash_indices");
    return PBF_OK;
}

// True when p is page-locked host memory (hipHostMalloc / hipHostRegister / torch pin_memory).
bool is_pinned_host(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: clear the sticky error
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Host-resident keys: stream them through pinned double buffers in chunks of whole keys.
// `op(batch_on_device, first_key_index)` runs the device work for one chunk.
template <class Op>
int for_host_chunks(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                    uint64_t key_align, Op&& op) {
    const bool pinned = is_pinned_host(keys) && (!offsets || is_pinned_host(offsets));
    uint64_t i0 = 0;
    while (i0 < n) {
        // choose [i0, i1)
        uint64_t i1;
        if (offsets) {
            // largest i1 with bytes <= stage_bytes() (at least one key)
            uint64_t lo = i0 + 1, hi = n;
            const uint64_t start = offsets[i0];
            if (offsets[n] - start <= stage_bytes()) {
                i1 = n;
            } else {
                while (lo < hi) {
                    uint64_t mid = (lo + hi + 1) / 2;
                    if (offsets[mid] - start <= stage_bytes()) lo = mid; else hi = mid - 1;
                }
                i1 = lo;
                // every chunk but the last holds a multiple of key_align keys, so the next one
                // starts on a whole hit-mask byte (probes: 64); when fewer than key_align keys
                // fit the byte budget the chunk takes key_align keys anyway (staging buffers are
                // sized from the chunk's actual bytes)
                if (i1 - i0 >= key_align)
                    i1 = i0 + ((i1 - i0) / key_align) * key_align;
                else
                    i1 = std::min<uint64_t>(n, i0 + key_align);
            }
        } else {
            uint64_t per = std::max<uint64_t>(1, stage_bytes() / std::max<uint32_t>(1, key_len));
            per = std::max<uint64_t>(key_align, (per / key_align) * key_align);
            i1 = std::min<uint64_t>(n, i0 + per);
        }
        const uint64_t cn = i1 - i0;
        const uint64_t byte0 = offsets ? offsets[i0] : i0 * key_len;
        const uint64_t nbytes = offsets ? offsets[i1] - offsets[i0] : cn * key_len;
        const size_t off_bytes = offsets ? size_t(cn + 1) * 8 : 0;
        // device staging (single buffer: stream order serialises reuse)
        HIP_TRY(f->sc->dkeys.ensure(((nbytes + 15) & ~uint64_t(15)) + 16));
        if (offsets) HIP_TRY(f->sc->doffs.ensure(off_bytes));
        if (pinned) {
            // caller's buffers are page-locked: DMA straight from them (the call syncs before
            // returning, so they stay valid for the copy)
            if (nbytes) HIP_TRY(hipMemcpyAsync(f->sc->dkeys.p, keys + byte0, nbytes, hipMemcpyHostToDevice, f->stream));
            if (offsets)
                HIP_TRY(hipMemcpyAsync(f->sc->doffs.p, offsets + i0, off_bytes, hipMemcpyHostToDevice, f->stream));
        } else {
            PinBuf& pb = f->sc->pin[f->sc->pin_next];
            f->sc->pin_next ^= 1;
            if (pb.done) HIP_TRY(hipEventSynchronize(pb.done));
            HIP_TRY(pb.ensure(nbytes + off_bytes + 16));
            if (!pb.done) HIP_TRY(hipEventCreateWithFlags(&pb.done, hipEventDisableTiming));
            const size_t off_at = (nbytes + 15) & ~uint64_t(15);
            std::memcpy(pb.p, keys + byte0, nbytes);
            if (offsets) std::memcpy(static_cast<uint8_t*>(pb.p) + off_at, offsets + i0, off_bytes);
            HIP_TRY(hipMemcpyAsync(f->sc->dkeys.p, pb.p, nbytes, hipMemcpyHostToDevice, f->stream));
            if (offsets)
                HIP_TRY(hipMemcpyAsync(f->sc->doffs.p, static_cast<uint8_t*>(pb.p) + off_at, off_bytes,
                                       hipMemcpyHostToDevice, f->stream));
            HIP_TRY(hipEventRecord(pb.done, f->stream));
        }
        Batch b = make_batch(static_cast<const uint8_t*>(f->sc->dkeys.p),
                             offsets ? static_cast<const uint64_t*>(f->sc->doffs.p) : nullptr, key_len, cn);
        int rc = op(b, i0);
        if (rc) return rc;
        i0 = i1;
    }
    return PBF_OK;
}

int check_keys(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint32_t key_len, uint64_t n,
               bool var) {
    int rc = enter(f);
    if (rc) return rc;
    if (n == 0) return PBF_OK;
    if (!keys) return fail(PBF_ERR_INVALID, "null keys pointer");
    if (var && !offsets) return fail(PBF_ERR_INVALID, "variable-length keys need offsets[n+1]");
    if (!var && key_len == 0) {
        // zero-length fixed keys are legal (key ""), handled through the variable path below
    }
    return PBF_OK;
}

// Wait for everything queued on f's stream.  Polls first (a caller that waits is about to use
// the results), then keeps polling with sleeps that back off from 10 us to 200 us, so a long
// wait costs a host core almost nothing and does not depend on an interrupt-driven wake-up
// (PBF_SPIN_US sets the pure polling budget, default 200 us).
//
// A wait has a reporting deadline (PBF_WAIT_S seconds, default 60 — no call of this library
// runs for more than a fraction of a second of GPU time; the GPU box's own silence limit is 3
// minutes): past it the wait prints the stream and the last kernel enqueued on it to stderr, then
// blocks until the stream is idle (queued copies may still target host memory the caller owns,
// and the leased scratch must not be reused under running kernels) and the call returns
// PBF_ERR_HIP.  A stream that never finishes is therefore reported, not returned from: the
// deadline is a diagnostic, not a bound.  (Round 2 saw one GPU-suite run hang inside a wait that
// blocked on an event created with hipEventBlockingSync, an interrupt-driven wake-up; since the
// polling wait replaced it no run has hung: DESIGN.md §1.)
int wait_raw(hipStream_t stream, int device, const char* last_kernel) {
    static const long spin_us = [] {
        const char* e = std::getenv("PBF_SPIN_US");
        return e ? std::atol(e) : 200L;
    }();
    static const double limit_s = [] {
        const char* e = std::getenv("PBF_WAIT_S");
        const double x = e ? std::atof(e) : 0.0;
        return x > 0 ? x : 60.0;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    const auto spin = std::chrono::microseconds(spin_us);
    const auto limit = std::chrono::duration<double>(limit_s);
    long nap_us = 10;
    for (;;) {
        const hipError_t e = hipStreamQuery(stream);
        if (e == hipSuccess) return PBF_OK;
        (void)hipGetLastError();  // "not ready" is not an error (see event_done)
        if (e != hipErrorNotReady) return fail(PBF_ERR_HIP, std::string("hipStreamQuery: ") + hipGetErrorString(e));
        const auto waited = std::chrono::steady_clock::now() - t0;
        if (waited > limit) {
            // Report, then keep waiting: queued copies may still target host memory the caller
            // (or this call's stack) owns, and the leased scratch must not be handed back while
            // kernels still use it.  The call fails only once the stream is idle.
            char msg[256];
            std::snprintf(msg, sizeof msg,
                          "stream %p of device %d did not finish within %.1f s (PBF_WAIT_S); last kernel enqueued: %s",
                          static_cast<void*>(stream), device, limit_s, last_kernel);
            std::fprintf(stderr, "pebblebloom: %s; waiting for it to drain\n", msg);
            std::fflush(stderr);
            const hipError_t se = hipStreamSynchronize(stream);
            if (se != hipSuccess) (void)hipGetLastError();
            return fail(PBF_ERR_HIP, msg);
        }
        if (waited > spin) {
            std::this_thread::sleep_for(std::chrono::microseconds(nap_us));
            nap_us = std::min(nap_us * 2, 200L);
        }
    }
}

int wait_stream(pbf_filter_t* f) {
    const int rc = wait_raw(f->stream, f->device, f->last_kernel);
    f->pending = false;  // (also after a timeout: wait_raw returns once the stream has drained)
    return rc;
}

#define WAIT(f)                       \
    do {                              \
        int wrc_ = wait_stream(f);    \
        if (wrc_) return wrc_;        \
    } while (0)

// Every entry point that touches a handle holds its mutex: the reference probes one filter from
// many reader threads without a lock (lsm_storage.py:153-179), and a call's host-side state
// (the leased scratch, staging, pending modes) must not be shared between two of them.
#define LOCK(f)                                                         \
    if (!(f)) return fail(PBF_ERR_INVALID, "null filter handle");       \
    std::unique_lock<std::shared_mutex> lock_((f)->mu)

int add_impl(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint32_t key_len, uint64_t n,
             int on_device) {
    LOCK(f);
    int rc = check_keys(f, keys, offsets, key_len, n, offsets != nullptr);
    if (rc || n == 0) return rc;
    LEASE(f);
    if (on_device) return add_device(f, make_batch(keys, offsets, key_len, n));
    rc = for_host_chunks(f, keys, offsets, key_len, n, 1, [&](const Batch& b, uint64_t) { return add_device(f, b); });
    if (rc) return rc;
    WAIT(f);
    return PBF_OK;
}

int probe_impl(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint32_t key_len, uint64_t n,
               uint8_t* hitmask, int on_device) {
    LOCK(f);
    int rc = check_keys(f, keys, offsets, key_len, n, offsets != nullptr);
    if (rc || n == 0) return rc;
    if (!hitmask) return fail(PBF_ERR_INVALID, "null hitmask");
    LEASE(f);
    if (on_device) return probe_device(f, make_batch(keys, offsets, key_len, n), hitmask);
    rc = for_host_chunks(f, keys, offsets, key_len, n, 64, [&](const Batch& b, uint64_t i0) {
        HIP_TRY(f->sc->dout.ensure((b.n + 7) / 8 + 8));
        int r = probe_device(f, b, static_cast<uint8_t*>(f->sc->dout.p));
        if (r) return r;
        HIP_TRY(hipMemcpyAsync(hitmask + i0 / 8, f->sc->dout.p, (b.n + 7) / 8, hipMemcpyDeviceToHost, f->stream));
        WAIT(f);
        return PBF_OK;
    });
    if (rc) return rc;
    WAIT(f);
    return PBF_OK;
}

int probe_multi_impl(pbf_filter_t* const* fs, uint32_t nf, const uint8_t* keys, const uint64_t* offsets,
                     uint32_t key_len, uint64_t n, uint8_t* const* hitmasks, int on_device) {
    if (nf == 0) return PBF_OK;
    if (!fs || !hitmasks) return fail(PBF_ERR_INVALID, "null filter or hitmask array");
    for (uint32_t i = 0; i < nf; ++i) {
        if (!fs[i]) return fail(PBF_ERR_INVALID, "null filter handle in set");
        if (fs[i]->device != fs[0]->device) return fail(PBF_ERR_INVALID, "filters of one multi-probe must share a device");
        if (n && !hitmasks[i]) return fail(PBF_ERR_INVALID, "null hitmask in set");
        for (uint32_t j = 0; j < i; ++j)
            if (fs[j] == fs[i]) return fail(PBF_ERR_INVALID, "a filter appears twice in the set");
    }
    // every handle of the set, in address order (two overlapping sets cannot deadlock)
    std::vector<pbf_filter_t*> order(fs, fs + nf);
    std::sort(order.begin(), order.end());
    std::vector<std::unique_lock<std::shared_mutex>> locks;
    locks.reserve(nf);
    for (pbf_filter_t* p : order) locks.emplace_back(p->mu);
    int rc = check_keys(fs[0], keys, offsets, key_len, n, offsets != nullptr);
    if (rc || n == 0) return rc;
    pbf_filter_t* f0 = fs[0];
    LEASE(f0);
    if (on_device) return probe_multi_device(fs, nf, make_batch(keys, offsets, key_len, n), hitmasks);
    std::vector<uint8_t*> douts(nf);
    rc = for_host_chunks(f0, keys, offsets, key_len, n, 64, [&](const Batch& b, uint64_t i0) {
        const size_t stride = (((b.n + 7) / 8) + 255) & ~size_t(255);
        HIP_TRY(f0->sc->dout.ensure(stride * nf + 8));
        for (uint32_t i = 0; i < nf; ++i) douts[i] = static_cast<uint8_t*>(f0->sc->dout.p) + i * stride;
        int r = probe_multi_device(fs, nf, b, douts.data());
        if (r) return r;
        for (uint32_t i = 0; i < nf; ++i)
            HIP_TRY(hipMemcpyAsync(hitmasks[i] + i0 / 8, douts[i], (b.n + 7) / 8, hipMemcpyDeviceToHost, f0->stream));
        WAIT(f0);
        return PBF_OK;
    });
    if (rc) return rc;
    WAIT(f0);
    return PBF_OK;
}

// A filter set spread over several placement groups (LsmStorage.get's filters placed one per GPU,
// src/lsm_storage.py:164-179): each group — filters of one device — is probed by probe_multi_impl
// on its own host thread, every group staging the host key batch to its own device (a replicated
// H2D), its hit masks written to the caller's buffers at the filters' own places in the set (the
// get order).  The calling thread runs the first group.  Host keys and hit masks only.
int probe_multi_groups(pbf_filter_t* const* fs, uint32_t nf, const uint32_t* group_of, const uint8_t* keys,
                       const uint64_t* offsets, uint32_t key_len, uint64_t n, uint8_t* const* hitmasks) {
    std::vector<int32_t> dev(nf);
    for (uint32_t i = 0; i < nf; ++i) {
        if (!fs[i]) return fail(PBF_ERR_INVALID, "null filter handle in set");
        for (uint32_t j = 0; j < i; ++j)
            if (fs[j] == fs[i]) return fail(PBF_ERR_INVALID, "a filter appears twice in the set");
        dev[i] = fs[i]->device;
    }
    std::vector<uint32_t> slot(nf);
    uint32_t ng = 0;
    if (int rc = pbf_plan_groups(group_of, dev.data(), nf, slot.data(), &ng)) return rc;
    const size_t G = ng;
    std::vector<uint32_t> ids(G);  // group ids, first-appearance order
    std::vector<std::vector<pbf_filter_t*>> gfs(G);
    std::vector<std::vector<uint8_t*>> ghm(G);
    for (uint32_t i = 0; i < nf; ++i) {
        ids[slot[i]] = group_of[i];
        gfs[slot[i]].push_back(fs[i]);
        ghm[slot[i]].push_back(hitmasks[i]);
    }
    std::vector<int> rcs(G, PBF_OK);
    std::vector<std::string> errs(G);
    auto run = [&](size_t g) {
        rcs[g] = probe_multi_impl(gfs[g].data(), uint32_t(gfs[g].size()), keys, offsets, key_len, n, ghm[g].data(), 0);
        if (rcs[g]) errs[g] = g_last_error;
    };
    std::vector<std::thread> th;
    th.reserve(G);
    for (size_t g = 1; g < G; ++g) th.emplace_back(run, g);
    run(0);
    for (auto& t : th) t.join();
    for (size_t g = 0; g < G; ++g)
        if (rcs[g]) return fail(rcs[g], "placement group " + std::to_string(ids[g]) + ": " + errs[g]);
    return PBF_OK;
}

int hash_impl(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint32_t key_len, uint64_t n,
              uint64_t* out, int on_device) {
    LOCK(f);
    int rc = check_keys(f, keys, offsets, key_len, n, offsets != nullptr);
    if (rc || n == 0) return rc;
    if (!out) return fail(PBF_ERR_INVALID, "null output");
    if (on_device) return hash_device(f, make_batch(keys, offsets, key_len, n), out);
    LEASE(f);
    rc = for_host_chunks(f, keys, offsets, key_len, n, 1, [&](const Batch& b, uint64_t i0) {
        HIP_TRY(f->sc->dout.ensure(b.n * f->k * 8 + 8));
        int r = hash_device(f, b, static_cast<uint64_t*>(f->sc->dout.p));
        if (r) return r;
        HIP_TRY(hipMemcpyAsync(out + i0 * f->k, f->sc->dout.p, b.n * f->k * 8, hipMemcpyDeviceToHost, f->stream));
        WAIT(f);
        return PBF_OK;
    });
    if (rc) return rc;
    WAIT(f);
    return PBF_OK;
}

// mmh3.hash(key, seed) for one key (the signed int32 bloom_filter.py:46 takes): SURVEY.md §8b's
// pbf_murmur3_x86_32, computed on the device like every other hash of the library.
__global__ void k_murmur_one(const uint8_t* key, uint32_t len, uint32_t seed, int32_t* out) {
    if (threadIdx.x != 0) return;
    murmur_seeds_loop(key, len, 1, [&](int, uint32_t h) { *out = int32_t(h); }, int(seed));
}

__global__ void k_popcount(const uint32_t* __restrict__ w, uint64_t n, unsigned long long* out) {
    __shared__ unsigned long long part[4];
    unsigned long long s = 0;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) s += __popc(w[i]);
    for (int d = 32; d > 0; d >>= 1) s += __shfl_down(s, d, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, part[0] + part[1] + part[2] + part[3]);
}

// Scratch of pbf_encode_data_blocks, one per device (the encoder is not tied to a filter).
struct EncodeCtx {
    std::mutex mu;
    hipStream_t stream = nullptr;
    DevBuf keys, vals, offs, out, err;
};

EncodeCtx& encode_ctx(int device) {
    static std::mutex mu;
    static std::map<int, EncodeCtx*> ctx;
    std::lock_guard<std::mutex> lock(mu);
    auto& p = ctx[device];
    if (!p) p = new EncodeCtx();
    return *p;
}

// Mapped, coherent pinned memory for the one-key probe (pbf_may_contain): result byte at 0,
// offsets at kOneKeyOffs, key bytes at kOneKeyData (16-B aligned).  One per (thread, device):
// calls from different threads never share it; it lives as long as the thread.
constexpr size_t kOneKeyOffs = 64, kOneKeyData = 128, kOneKeyMax = 4096;
struct OneKeyStage {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    OneKeyStage() = default;
    OneKeyStage(const OneKeyStage&) = delete;
    OneKeyStage& operator=(const OneKeyStage&) = delete;
    ~OneKeyStage() {  // the thread ends: its pinned stage goes back (reader pools churn threads)
        if (host) (void)hipHostFree(host);
    }
};

int one_key_stage(int device, OneKeyStage** out) {
    thread_local std::map<int, OneKeyStage> stages;
    OneKeyStage& st = stages[device];
    if (!st.host) {
        void* h = nullptr;
        HIP_TRY(hipHostMalloc(&h, kOneKeyData + kOneKeyMax + 64, hipHostMallocMapped | hipHostMallocCoherent));
        void* d = nullptr;
        const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(h);
            return fail(PBF_ERR_HIP, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
        }
        st.host = static_cast<uint8_t*>(h);
        st.dev = static_cast<uint8_t*>(d);
    }
    *out = &st;
    return PBF_OK;
}

// Streams for one-key probes that hold the filter's lock shared (PBF_READER_STREAMS, default 4
// = the process's hardware queues): a reader's one-wave kernel does not queue behind another
// reader's, nor behind a later build on the filter's own stream.  Created once per device; a
// thread keeps the stream it was dealt.
hipError_t reader_stream(int device, hipStream_t* out) {
    static std::mutex mu;
    static std::map<int, std::vector<hipStream_t>> pools;
    static std::atomic<uint32_t> next{0};
    static const size_t nstreams = [] {
        const char* e = std::getenv("PBF_READER_STREAMS");
        const int x = e ? std::atoi(e) : 0;
        return x > 0 ? size_t(std::min(x, 32)) : size_t(4);
    }();
    thread_local std::map<int, hipStream_t> mine;
    auto it = mine.find(device);
    if (it != mine.end()) {
        *out = it->second;
        return hipSuccess;
    }
    std::lock_guard<std::mutex> lock(mu);
    auto& pool = pools[device];
    while (pool.size() < nstreams) {
        hipStream_t st = nullptr;
        const hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        if (e != hipSuccess) {
            if (pool.empty()) return e;
            (void)hipGetLastError();
            break;
        }
        pool.push_back(st);
        register_stream(device, st);
    }
    *out = mine[device] = pool[next++ % pool.size()];
    return hipSuccess;
}

// ---------------------------------------------------------------- resident one-key reader
// (reader_service.hpp) One board per device in mapped, coherent pinned memory, one resident
// wave serving it on a high-priority non-blocking stream (it gets a hardware queue of its own,
// so the resident wave never holds up other streams' work, and the null stream does not wait for
// it), one slot per host thread.
// PBF_RESIDENT_READER=0 sends every one-key probe through the per-key launch instead;
// PBF_RESIDENT_IDLE_US (default 2000) is how long the wave waits for a key before it leaves.
struct ResidentReader {
    std::mutex mu;
    SvcBoard* host = nullptr;
    SvcBoard* dev = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;  // recorded after each launch: the wave has left once it completes
    bool launched = false;
    uint32_t launches = 0;
    uint32_t nslots = 0;
    std::vector<uint32_t> free_slots;
    uint64_t idle_ticks = 0, life_ticks = 0;
    int device = 0;
    // the board's descriptor table (reader_service.hpp SvcBoard::desc): indexes handed to filters
    // at their first resident probe, returned when they are destroyed; every return bumps the
    // epoch, which requests carry, so the wave's descriptor cache never outlives an index's owner
    std::vector<uint32_t> free_ids;
    uint32_t next_id = 1;
    std::atomic<uint32_t> epoch{1};
    // answered requests and the wave's time on them (pbf_resident_stats)
    std::atomic<uint64_t> answered{0}, answer_ticks{0};
    uint64_t khz = 0;
};

std::atomic<int> g_resident_on{-1};  // -1: PBF_RESIDENT_READER not read yet

bool resident_enabled() {
    int on = g_resident_on.load(std::memory_order_relaxed);
    if (on < 0) {
        const char* e = std::getenv("PBF_RESIDENT_READER");
        int want = (e && e[0] == '0') ? 0 : 1;
        int expected = -1;
        g_resident_on.compare_exchange_strong(expected, want);
        on = g_resident_on.load(std::memory_order_relaxed);
    }
    return on != 0;
}

std::mutex g_resident_mu;
std::map<int, ResidentReader*> g_resident;  // never freed: a wave may still poll its board at exit
std::atomic<ResidentReader*> g_resident_fast[64];  // (the same, lock-free lookups)

// At exit: every resident wave is told to leave and given a few milliseconds to do so (it
// leaves by itself after its idle time anyway).
void resident_shutdown() {
    std::lock_guard<std::mutex> lock(g_resident_mu);
    for (auto& kv : g_resident) {
        ResidentReader* rr = kv.second;
        if (!rr || !rr->host) continue;
        __atomic_store_n(&rr->host->stop, 1u, __ATOMIC_RELEASE);
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (auto& kv : g_resident) {
        ResidentReader* rr = kv.second;
        if (!rr || !rr->host) continue;
        while (__atomic_load_n(&rr->host->state, __ATOMIC_ACQUIRE) != 0 &&
               std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(20)) {
        }
        // and the launch itself has completed (its end is recorded on rr->done), so no kernel of
        // the library is still in flight when the runtime (and a profiler's tool) tears down
        std::lock_guard<std::mutex> lock(rr->mu);
        while (rr->launched && !event_done(rr->done) &&
               std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(50)) {
        }
    }
}

// The device's reader (created on first use), or nullptr if it cannot be set up (the caller
// then launches per key).
ResidentReader* resident_reader(int device) {
    std::lock_guard<std::mutex> lock(g_resident_mu);
    auto it = g_resident.find(device);
    if (it != g_resident.end()) return it->second;
    ResidentReader* rr = nullptr;
    do {
        if (hipSetDevice(device) != hipSuccess) break;  // (the one-key callers do not set it)
        void* h = nullptr;
        if (hipHostMalloc(&h, sizeof(SvcBoard), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) break;
        std::memset(h, 0, sizeof(SvcBoard));
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
            (void)hipHostFree(h);
            break;
        }
        int ncu = 0, khz = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
            hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || ncu <= 0 || khz <= 0) {
            (void)hipHostFree(h);
            break;
        }
        // A high-priority non-blocking stream: it gets a hardware queue of its own (the pool
        // streams' kernels are not held up behind the wave) and the null stream does not wait
        // for it.  (A CU-masked stream also has its own queue, but hipExtStreamCreateWithCUMask
        // makes a BLOCKING stream: null-stream work -- torch's default stream -- waited for the
        // wave; tools/microbench/cumask_block.hip, profiles/r06/ab/summary.md.)
        int least = 0, greatest = 0;
        hipStream_t st = nullptr;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
            hipStreamCreateWithPriority(&st, hipStreamNonBlocking, greatest) != hipSuccess) {
            (void)hipHostFree(h);
            break;
        }
        hipEvent_t ev = nullptr;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            (void)hipStreamDestroy(st);
            (void)hipHostFree(h);
            break;
        }
        rr = new ResidentReader();
        rr->host = static_cast<SvcBoard*>(h);
        rr->dev = static_cast<SvcBoard*>(d);
        rr->stream = st;
        rr->done = ev;
        rr->device = device;
        rr->khz = uint64_t(khz);
        const char* e = std::getenv("PBF_RESIDENT_IDLE_US");
        const uint64_t idle_us = e && std::atoi(e) > 0 ? uint64_t(std::atoi(e)) : 2000;
        rr->idle_ticks = uint64_t(khz) * idle_us / 1000;
        rr->life_ticks = uint64_t(khz) * 200;  // 200 ms
        if (g_resident.empty()) std::atexit(resident_shutdown);
    } while (false);
    (void)hipGetLastError();
    g_resident[device] = rr;
    if (rr && device >= 0 && device < 64) g_resident_fast[device].store(rr, std::memory_order_release);
    return rr;
}

// Whether the device's resident reader wave is on the GPU now (lock-free: the board's state word).
bool resident_live(int device) {
    static const int force = [] {  // PBF_SPARE_CU=0/1 forces the planning either way (A/B)
        const char* e = std::getenv("PBF_SPARE_CU");
        return e ? std::atoi(e) : -1;
    }();
    if (force >= 0) return force != 0;
    if (device < 0 || device >= 64) return false;
    ResidentReader* rr = g_resident_fast[device].load(std::memory_order_acquire);
    return rr && rr->host && __atomic_load_n(&rr->host->state, __ATOMIC_ACQUIRE) != 0;
}

// A wave serving rr's board: launch one unless the last launch is still running (or queued).
int resident_ensure(ResidentReader* rr) {
    std::lock_guard<std::mutex> lock(rr->mu);
    if (rr->launched) {
        const hipError_t q = hipEventQuery(rr->done);
        if (q == hipErrorNotReady) {
            (void)hipGetLastError();
            return PBF_OK;
        }
        HIP_TRY(q);
    }
    HIP_TRY(hipSetDevice(rr->device));
    k_reader_service<<<1, 64, 0, rr->stream>>>(rr->dev, ++rr->launches, rr->idle_ticks, rr->life_ticks);
    CHECK_LAUNCH();
    HIP_TRY(hipEventRecord(rr->done, rr->stream));
    rr->launched = true;
    return PBF_OK;
}

// The calling thread's slot on a device's board (returned to the board when the thread ends).
struct ResidentSlot {
    ResidentReader* rr = nullptr;
    int slot = -1;
    uint32_t seq = 0;
    ResidentSlot() = default;
    ResidentSlot(const ResidentSlot&) = delete;
    ResidentSlot& operator=(const ResidentSlot&) = delete;
    ~ResidentSlot() {
        if (rr && slot >= 0) {
            std::lock_guard<std::mutex> lock(rr->mu);
            rr->free_slots.push_back(uint32_t(slot));
        }
    }
};

// f's index in rr's descriptor table, registering it (its descriptor written to the board) on
// first use; 0 when the table is full (the caller launches per key).
uint32_t svc_index(ResidentReader* rr, pbf_filter_t* f) {
    uint32_t id = f->svc_id.load(std::memory_order_acquire);
    if (id) return id;
    std::lock_guard<std::mutex> lock(rr->mu);
    id = f->svc_id.load(std::memory_order_relaxed);
    if (id) return id;
    if (!rr->free_ids.empty()) {
        id = rr->free_ids.back();
        rr->free_ids.pop_back();
    } else if (rr->next_id < kSvcDescs) {
        id = rr->next_id++;
    } else {
        return 0;
    }
    rr->host->desc[id] = SvcFilter{f->bitmap, f->im};  // before any request names id (x86: in order)
    f->svc_id.store(id, std::memory_order_release);
    return id;
}

// pbf_destroy: f's index back to its device's table.  The epoch moves on, so a request that names
// the index for its next owner cannot meet f's descriptor in the wave's cache.
void svc_release(pbf_filter_t* f) {
    const uint32_t id = f->svc_id.load(std::memory_order_acquire);
    if (!id || f->device < 0 || f->device >= 64) return;
    ResidentReader* rr = g_resident_fast[f->device].load(std::memory_order_acquire);
    if (!rr) return;
    std::lock_guard<std::mutex> lock(rr->mu);
    rr->epoch.fetch_add(1, std::memory_order_acq_rel);
    rr->free_ids.push_back(id);
    f->svc_id.store(0, std::memory_order_relaxed);
}

// One key against nf filters sharing k through the resident reader: *bits (bit f = filters f's
// answer) and *taken = true, or *taken = false when this call cannot use it (disabled, key or
// set too large, no free slot, no board, descriptor table full): the caller launches per key.
// The filters' bitmaps must have no work still queued (reader_ok).
int resident_probe(int device, pbf_filter_t* const* fs, uint32_t nf, uint32_t k, const uint8_t* key, uint64_t len,
                   uint64_t* bits, bool* taken) {
    *taken = false;
    if (!resident_enabled() || len > kSvcKeyMax || k == 0 || k > 32 || nf == 0 || nf > kSvcFilters) return PBF_OK;
    thread_local std::map<int, ResidentSlot> mine;
    ResidentSlot& ts = mine[device];
    if (ts.slot < 0) {
        ResidentReader* rr = resident_reader(device);
        if (!rr) return PBF_OK;
        std::lock_guard<std::mutex> lock(rr->mu);
        uint32_t slot;
        if (!rr->free_slots.empty()) {
            slot = rr->free_slots.back();
            rr->free_slots.pop_back();
        } else if (rr->nslots < kSvcSlots) {
            slot = rr->nslots++;
            __atomic_store_n(&rr->host->nused, rr->nslots, __ATOMIC_RELEASE);
        } else {
            return PBF_OK;  // 64 threads hold slots: launch per key
        }
        ts.rr = rr;
        ts.slot = int(slot);
        ts.seq = __atomic_load_n(&rr->host->head[slot].req, __ATOMIC_ACQUIRE);  // a recycled slot's last
    }
    ResidentReader* rr = ts.rr;
    uint16_t ids[kSvcFilters];
    for (uint32_t i = 0; i < nf; ++i) {
        const uint32_t id = svc_index(rr, fs[i]);
        if (!id) return PBF_OK;
        ids[i] = uint16_t(id);
    }
    const uint32_t epoch = rr->epoch.load(std::memory_order_acquire);  // (after the registrations)
    SvcHead& hd = rr->host->head[ts.slot];
    SvcSlot& sl = rr->host->slot[ts.slot];
    // the body first (indexes past the 16th, a key too long for the head), then head line 1 (its
    // tag req2 last), then line 0 (req last): the wave takes the request once both lines carry the
    // new sequence (reader_service.hpp SvcHead)
    if (nf > kSvcInlineIds) std::memcpy(sl.ids + kSvcInlineIds, ids + kSvcInlineIds, (nf - kSvcInlineIds) * sizeof(uint16_t));
    const bool inl = len <= kSvcInlineKey;
    if (!inl) std::memcpy(sl.key, key, len);
    uint32_t seq = ts.seq + 1;
    if (seq == 0) seq = 1;
    ts.seq = seq;
    if (inl && len > 16) std::memcpy(hd.key1, key + 16, len - 16);
    __atomic_store_n(&hd.req2, seq, __ATOMIC_RELEASE);
    hd.shape = nf | (k << 8) | (uint32_t(len) << 16);
    hd.epoch = epoch;
    std::memcpy(hd.ids, ids, std::min(nf, kSvcInlineIds) * sizeof(uint16_t));
    if (inl && len) std::memcpy(hd.key0, key, std::min<uint64_t>(len, 16));
    __atomic_store_n(&hd.req, seq, __ATOMIC_RELEASE);
    int rc = PBF_OK;
    if (__atomic_load_n(&rr->host->state, __ATOMIC_ACQUIRE) == 0) {
        rc = resident_ensure(rr);
        if (rc) return rc;
    }
    // the answer: poll the slot's ack; a wave that left after its last look at the heads (the
    // request stranded) is relaunched
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 1; __atomic_load_n(&sl.ack, __ATOMIC_ACQUIRE) != seq; ++spin) {
        if ((spin & 63) == 0) {
            const auto el = std::chrono::steady_clock::now() - t0;
            if (el > std::chrono::microseconds(50) && __atomic_load_n(&rr->host->state, __ATOMIC_ACQUIRE) == 0) {
                rc = resident_ensure(rr);
                if (rc) return rc;
            }
            if (el > std::chrono::seconds(2)) {
                // Retract the request before the caller may free or rebuild the bitmap: a wave
                // that has not taken it yet acknowledges a head with no filters without reading
                // any memory; one that has taken it answers within microseconds of doing so.
                __atomic_store_n(&hd.shape, 0u, __ATOMIC_RELEASE);
                const auto t1 = std::chrono::steady_clock::now();
                while (__atomic_load_n(&sl.ack, __ATOMIC_ACQUIRE) != seq &&
                       __atomic_load_n(&rr->host->state, __ATOMIC_ACQUIRE) != 0 &&
                       std::chrono::steady_clock::now() - t1 < std::chrono::milliseconds(100)) {
                }
                return fail(PBF_ERR_HIP, "resident reader: no answer within 2 s (request retracted)");
            }
        }
    }
    *bits = __atomic_load_n(&sl.bits, __ATOMIC_ACQUIRE);
    rr->answered.fetch_add(1, std::memory_order_relaxed);
    rr->answer_ticks.fetch_add(__atomic_load_n(&sl.ticks, __ATOMIC_RELAXED), std::memory_order_relaxed);
    *taken = true;
    return PBF_OK;
}

// Whether a one-key probe of f may run under f's lock held SHARED: the filter is materialised,
// nothing of it is still queued on its stream (its last build / from_bytes has completed, so a
// reader stream sees the finished bitmap), and the key takes the mapped one-key kernel.
// (PBF_SHARED_READERS=0 sends every one-key probe through the exclusive path: A/B measurements.)
bool reader_ok(pbf_filter_t* f, uint64_t len) {
    static const bool enabled = [] {
        const char* e = std::getenv("PBF_SHARED_READERS");
        return !(e && e[0] == '0');
    }();
    if (!enabled) return false;
    if (f->k == 0) return true;
    if (kmax_for(f->k) == 0 || len > kOneKeyMax || f->pristine) return false;
    if (!f->pending.load(std::memory_order_relaxed)) return true;
    const hipError_t q = hipStreamQuery(f->stream);
    if (q != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    // drained: later readers skip the query (a get probes the same published filters again and
    // again; 16 stream queries cost a get several microseconds).  No writer can have queued work
    // since: writers hold the lock exclusively and this reader holds it shared.
    f->pending.store(false, std::memory_order_relaxed);
    return true;
}

// One key of a built filter (reader_ok, lock held shared) through the resident reader:
// PBF_OK with *out, an error, or kNotTaken when the reader does not take it (the caller launches).
constexpr int kNotTaken = 1;
int one_key_resident(pbf_filter_t* f, const uint8_t* key, uint64_t len, int* out) {
    uint64_t bits = 0;
    bool taken = false;
    const int rc = resident_probe(f->device, &f, 1, f->k, key, len, &bits, &taken);
    if (rc) return rc;
    if (!taken) return kNotTaken;
    *out = int(bits & 1u);
    f->last_probe_mode.store(PBF_PROBE_DIRECT, std::memory_order_relaxed);
    f->last_probe_detail.store(PBF_DETAIL_ONE_KEY | PBF_DETAIL_SHARED | PBF_DETAIL_RESIDENT, std::memory_order_relaxed);
    return PBF_OK;
}

// The mapped one-key probe of f on stream s (a launch).  shared: the caller holds f's lock shared
// (reader_ok held), so nothing of the handle is written but the probe diagnostics (atomics).
int one_key_probe(pbf_filter_t* f, const uint8_t* key, uint64_t len, int* out, hipStream_t s, bool shared) {
    int rc = PBF_OK;
    OneKeyStage* st = nullptr;
    rc = one_key_stage(f->device, &st);
    if (rc) return rc;
    // the key and its two offsets go into mapped pinned memory the kernel reads over the bus;
    // the kernel's hit byte comes back the same way: one launch, no copies
    uint64_t* offs = reinterpret_cast<uint64_t*>(st->host + kOneKeyOffs);
    offs[0] = 0;
    offs[1] = len;
    if (len) std::memcpy(st->host + kOneKeyData, key, len);
    st->host[0] = 0xEE;
    KeySet ks{};
    ks.data = st->dev + kOneKeyData;
    ks.offsets = reinterpret_cast<const uint64_t*>(st->dev + kOneKeyOffs);
    ks.off0 = ks.offsets;
    dispatch(kmax_for(f->k), kVar, [&](auto KMAX, auto KM) {
        k_probe<decltype(KMAX)::value, decltype(KM)::value>
            <<<1, 64, 0, s>>>(ks, 1, int(f->k), f->im, f->bitmap, st->dev, int(f->k));
    });
    if (shared) {
        CHECK_LAUNCH();
    } else {
        LAUNCHED(f, "k_probe<one key>");
    }
    // The kernel's hit byte lands in mapped host memory as soon as it is stored (the key bytes
    // were read before it), which is earlier than the stream's completion signal: poll the byte,
    // and fall back to the stream wait (which also reports a failed kernel) after 2 ms.
    volatile uint8_t* res = reinterpret_cast<volatile uint8_t*>(st->host);
    const auto t0 = std::chrono::steady_clock::now();
    uint8_t hit = 0xEE;
    for (uint32_t spin = 0;; ++spin) {
        hit = *res;
        if (hit != 0xEE) break;
        if ((spin & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
            if (shared) {
                rc = wait_raw(s, f->device, "k_probe<one key>");
                if (rc) return rc;
            } else {
                WAIT(f);
            }
            hit = *res;
            break;
        }
    }
    if (hit > 1) return fail(PBF_ERR_HIP, "one-key probe: result byte not written");
    *out = hit;
    f->last_probe_mode = PBF_PROBE_DIRECT;
    f->last_probe_detail = PBF_DETAIL_ONE_KEY | (shared ? PBF_DETAIL_SHARED : 0u);
    return PBF_OK;
}

// BloomFilter.may_contain (bloom_filter.py:67-74) for one key; the caller holds f's lock.
int may_contain_locked(pbf_filter_t* f, const uint8_t* key, uint64_t len, int* out) {
    int rc = enter(f);
    if (rc) return rc;
    if (!out || (len && !key)) return fail(PBF_ERR_INVALID, "null key or out");
    if (f->k == 0) {  // the AND over no bits (bloom_filter.py:71-74 runs no iteration)
        *out = 1;
        return PBF_OK;
    }
    rc = materialise(f);
    if (rc) return rc;
    if (len > kOneKeyMax) {  // long keys: the staged batch path
        uint64_t offs[2] = {0, len};
        uint8_t hm = 0;
        LEASE(f);
        rc = for_host_chunks(f, key, offs, 0, 1, 64, [&](const Batch& b, uint64_t) {
            HIP_TRY(f->sc->dout.ensure(8));
            int r = probe_device(f, b, static_cast<uint8_t*>(f->sc->dout.p));
            if (r) return r;
            HIP_TRY(hipMemcpyAsync(&hm, f->sc->dout.p, 1, hipMemcpyDeviceToHost, f->stream));
            return PBF_OK;
        });
        if (rc) return rc;
        WAIT(f);
        *out = hm & 1;
        return PBF_OK;
    }
    return one_key_probe(f, key, len, out, f->stream, false);
}

// The filters' pending work (builds, from_bytes) ordered before work on stream s: a filter
// whose stream may still run queued work and has not finished it hands it over by an event.
int join_into(pbf_filter_t* f, hipStream_t s) {
    if (!f->pending || f->stream == s) return PBF_OK;
    const hipError_t q = hipStreamQuery(f->stream);
    if (q == hipSuccess) {
        f->pending = false;
        return PBF_OK;
    }
    (void)hipGetLastError();  // "not ready"
    HIP_TRY(filter_event(f));
    HIP_TRY(hipEventRecord(f->ev, f->stream));
    HIP_TRY(hipStreamWaitEvent(s, f->ev, 0));
    return PBF_OK;
}

// LsmStorage.get's bloom checks for ONE key over a set of SSTable filters (src/lsm_storage.py:
// 164-179: every L0 table, and each level table whose key range holds the key): one
// k_may_contain_set launch per k and 64 filters, the key in and the answer out through mapped
// pinned memory.  Bit i of out_bits (LSB-first) = filters[i]->may_contain(key).  The caller
// holds every filter's lock.
int may_contain_set_locked(pbf_filter_t* const* fs, uint32_t nf, const uint8_t* key, uint64_t len, uint8_t* out_bits,
                           hipStream_t rs = nullptr) {
    const bool shared = rs != nullptr;  // every handle held shared, reader_ok for each (no writes)
    pbf_filter_t* f0 = fs[0];
    int rc = enter(f0);
    if (rc) return rc;
    std::memset(out_bits, 0, (nf + 7) / 8);
    auto put = [&](uint32_t i, bool hit) {
        if (hit) out_bits[i >> 3] |= uint8_t(1u << (i & 7));
    };
    // filters the fused kernel does not take (k > 32, keys longer than the mapped stage): one
    // may_contain each
    std::vector<uint32_t> ks;
    for (uint32_t i = 0; i < nf; ++i) {
        pbf_filter_t* f = fs[i];
        if (f->k == 0) {
            put(i, true);  // the AND over no bits
        } else if (kmax_for(f->k) == 0 || len > kOneKeyMax) {
            int hit = 0;
            rc = may_contain_locked(f, key, len, &hit);
            if (rc) return rc;
            put(i, hit != 0);
        } else if (std::find(ks.begin(), ks.end(), f->k) == ks.end()) {
            ks.push_back(f->k);
        }
    }
    if (ks.empty()) return PBF_OK;
    OneKeyStage* st = nullptr;
    rc = one_key_stage(f0->device, &st);
    if (rc) return rc;
    if (len) std::memcpy(st->host + kOneKeyData, key, len);
    hipStream_t s = shared ? rs : f0->stream;
    std::vector<uint8_t> resident_set(nf, 0);  // filters the resident reader answered
    for (uint32_t k : ks) {
        std::vector<uint32_t> idx;
        for (uint32_t i = 0; i < nf; ++i)
            if (fs[i]->k == k) idx.push_back(i);
        for (size_t c0 = 0; c0 < idx.size(); c0 += kMaxFilterSet) {
            const uint32_t nsub = uint32_t(std::min<size_t>(kMaxFilterSet, idx.size() - c0));
            if (shared) {  // every handle reader_ok: the resident reader may answer
                pbf_filter_t* sub[kMaxFilterSet];
                for (uint32_t j = 0; j < nsub; ++j) sub[j] = fs[idx[c0 + j]];
                uint64_t bits = 0;
                bool taken = false;
                rc = resident_probe(f0->device, sub, nsub, k, key, len, &bits, &taken);
                if (rc) return rc;
                if (taken) {
                    for (uint32_t j = 0; j < nsub; ++j) {
                        put(idx[c0 + j], (bits >> j) & 1u);
                        resident_set[idx[c0 + j]] = 1;
                    }
                    continue;
                }
            }
            FilterSet fset{};
            fset.nf = nsub;
            for (uint32_t j = 0; j < fset.nf; ++j) {
                pbf_filter_t* f = fs[idx[c0 + j]];
                if (!shared) {
                    rc = materialise(f);
                    if (rc) return rc;
                    rc = join_into(f, s);
                    if (rc) return rc;
                }
                fset.bm[j] = f->bitmap;
                fset.im[j] = f->im;
            }
            volatile uint8_t* flag = st->host + 8;
            *flag = 0;
            dispatch(kmax_for(k), kVar, [&](auto KMAX, auto) {
                if constexpr (decltype(KMAX)::value > 0)
                    k_may_contain_set<decltype(KMAX)::value>
                        <<<1, 64, 0, s>>>(st->dev + kOneKeyData, uint32_t(len), int(k), fset, st->dev);
            });
            if (shared) {
                CHECK_LAUNCH();
            } else {
                LAUNCHED(f0, "k_may_contain_set");
            }
            // poll the flag the kernel sets after its answer (earlier than the stream's
            // completion signal); the stream wait (which also reports a failed kernel) after 2 ms
            const auto t0 = std::chrono::steady_clock::now();
            for (uint32_t spin = 0; !*flag; ++spin) {
                if ((spin & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
                    if (shared) {
                        rc = wait_raw(s, f0->device, "k_may_contain_set");
                        if (rc) return rc;
                    } else {
                        WAIT(f0);
                    }
                    if (!*flag) return fail(PBF_ERR_HIP, "one-key set probe: answer not written");
                    break;
                }
            }
            const uint64_t bits = *reinterpret_cast<volatile uint64_t*>(st->host);
            for (uint32_t j = 0; j < fset.nf; ++j) put(idx[c0 + j], (bits >> j) & 1u);
        }
    }
    // only the filters k_may_contain_set covered (k == 0 filters were not probed; the others
    // recorded their own path in may_contain_locked)
    for (uint32_t i = 0; i < nf; ++i) {
        if (std::find(ks.begin(), ks.end(), fs[i]->k) == ks.end()) continue;
        fs[i]->last_probe_mode = PBF_PROBE_DIRECT;
        fs[i]->last_probe_detail = PBF_DETAIL_ONE_KEY | PBF_DETAIL_SET | (resident_set[i] ? PBF_DETAIL_RESIDENT : 0u);
    }
    return PBF_OK;
}

}  // namespace

namespace {

// Peer access from device a to device b's memory, enabled once per pair where the platform allows
// (xGMI between MI355X GPUs of a node); hipMemcpyPeerAsync stages through the host otherwise.
void enable_peer(int a, int b) {
    if (a == b) return;
    static std::mutex mu;
    static std::map<std::pair<int, int>, bool> done;
    std::lock_guard<std::mutex> lock(mu);
    if (done.count({a, b})) return;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can && hipSetDevice(a) == hipSuccess) {
        const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        (void)e;  // hipErrorPeerAccessAlreadyEnabled is fine too
    }
    (void)hipGetLastError();
    done[{a, b}] = true;
}

// dst (just created with src's nb_bytes and k) receives src's bitmap: device to device, or through
// pinned host memory (bounce).  Synchronous.  src's lock is held by the caller.
int copy_filter_into(pbf_filter_t* src, pbf_filter_t* dst, bool bounce) {
    dst->mode = src->mode;
    dst->probe_mode = src->probe_mode;
    if (src->pristine) {
        // logically all zero: the replica as created is that already (its unreachable middle,
        // m > 2^32, zeroed by pbf_create; a pristine src has a clean middle, pbf_clear)
        HIP_TRY(hipSetDevice(dst->device));
        return wait_stream(dst);
    }
    HIP_TRY(hipSetDevice(src->device));
    int rc = wait_stream(src);  // src's last build / load is in its bitmap
    if (rc) return rc;
    HIP_TRY(hipSetDevice(dst->device));
    rc = wait_stream(dst);  // the replica's allocation and zeroing are done
    if (rc) return rc;
    const size_t bytes = size_t(src->alloc_words) * 4;  // (the tail past nb_bytes is zero in src)
    if (!bounce) {
        if (src->device == dst->device) {
            HIP_TRY(hipMemcpyAsync(dst->bitmap, src->bitmap, bytes, hipMemcpyDeviceToDevice, dst->stream));
        } else {
            enable_peer(dst->device, src->device);
            HIP_TRY(hipSetDevice(dst->device));
            HIP_TRY(hipMemcpyPeerAsync(dst->bitmap, dst->device, src->bitmap, src->device, bytes, dst->stream));
        }
    } else {
        // pinned host bounce in 64 MiB pieces, each D2H on src's stream then H2D on dst's
        const size_t piece = std::min<size_t>(bytes, size_t(64) << 20);
        void* host = nullptr;
        HIP_TRY(hipHostMalloc(&host, piece, hipHostMallocDefault));
        hipError_t e = hipSuccess;
        for (size_t o = 0; o < bytes && e == hipSuccess; o += piece) {
            const size_t c = std::min(piece, bytes - o);
            e = hipSetDevice(src->device);
            if (e == hipSuccess)
                e = hipMemcpyAsync(host, reinterpret_cast<uint8_t*>(src->bitmap) + o, c, hipMemcpyDeviceToHost, src->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(src->stream);
            if (e == hipSuccess) e = hipSetDevice(dst->device);
            if (e == hipSuccess)
                e = hipMemcpyAsync(reinterpret_cast<uint8_t*>(dst->bitmap) + o, host, c, hipMemcpyHostToDevice, dst->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(dst->stream);
        }
        (void)hipHostFree(host);
        HIP_TRY(e);
    }
    dst->pristine = false;
    dst->middle_dirty = src->middle_dirty;
    dst->pending = true;
    return wait_stream(dst);
}

}  // namespace

extern "C" {

int pbf_version(void) { return 100; }

int pbf_device_count(int* count) {
    if (!count) return fail(PBF_ERR_INVALID, "null count");
    HIP_TRY(hipGetDeviceCount(count));
    return PBF_OK;
}

const char* pbf_last_error(void) { return g_last_error.c_str(); }

#ifndef PBF_SOURCE_DIGEST
#define PBF_SOURCE_DIGEST "none"
#endif
// the digest behind a marker, so build.py reads it from the file without loading the library
__attribute__((used)) const char pbf_source_digest_tag[] = "pbf-source-digest:" PBF_SOURCE_DIGEST;
const char* pbf_source_digest(void) { return pbf_source_digest_tag + 18; }

int pbf_create(int device, uint64_t nb_bytes, uint32_t nb_hash_functions, pbf_filter_t** out) {
    if (!out) return fail(PBF_ERR_INVALID, "null out");
    *out = nullptr;
    if (nb_bytes == 0) return fail(PBF_ERR_ZERO_SIZE, "nb_bytes == 0 (integer modulo by zero)");
    HIP_TRY(hipSetDevice(device));
    auto* f = new pbf_filter();
    f->device = device;
    f->nb_bytes = nb_bytes;
    f->k = nb_hash_functions;
    f->words = (nb_bytes + 3) / 4;
    f->alloc_words = (f->words + 3) & ~uint64_t(3);
    const uint64_t m = nb_bytes * 8;
    f->im = make_index_map(m);
    // tile geometry
    const bool cspace = m > (uint64_t(1) << 32);
    const uint64_t P = cspace ? (uint64_t(1) << 32) : m;
    TileMap tm{};
    tm.im = f->im;
    tm.tb = std::min<uint32_t>(20, std::max<uint32_t>(10, ceil_log2(P)));
    tm.nbuckets = uint32_t((P + (uint64_t(1) << tm.tb) - 1) >> tm.tb);
    tm.cspace = cspace ? 1 : 0;
    tm.total_words = f->words;
    f->tiled_ok = true;
    if (cspace) {
        const uint64_t delta = m - (uint64_t(1) << 32);
        if (delta % 32) f->tiled_ok = false;
        tm.delta_words = delta / 32;
    }
    if (tm.nbuckets > 8192) f->tiled_ok = false;  // LDS budget of k_part
    f->tm = tm;
    hipError_t e = pooled_stream(device, &f->stream);
    if (e == hipSuccess) {
        void* p = nullptr;
        e = bitmap_alloc(device, bitmap_alloc_bytes(f->alloc_words), &p, f->stream);
        f->bitmap = static_cast<uint32_t*>(p);
        if (e == hipSuccess) f->dpop = reinterpret_cast<uint64_t*>(f->bitmap + f->alloc_words);
    }
    // The tiled build writes every reachable word itself; the unreachable middle of a
    // m > 2^32 filter is zeroed once here.  Otherwise start from an explicit zero bitmap.
    if (e == hipSuccess) {
        if (f->tiled_ok && cspace) {
            const uint64_t lo_w = (uint64_t(1) << 31) / 32;
            const uint64_t hi_w = tm.delta_words + lo_w;  // first word of [m - 2^31, m)
            if (hi_w > lo_w) e = hipMemsetAsync(f->bitmap + lo_w, 0, (hi_w - lo_w) * 4, f->stream);
            f->pristine = true;
        } else {
            e = hipMemsetAsync(f->bitmap, 0, f->alloc_words * 4, f->stream);
            f->pristine = false;
        }
    }
    if (e == hipSuccess && !f->tiled_ok) f->pristine = false;
    // the allocation and the zeroing are queued on f's stream: a multi-filter call on another
    // filter's stream must order after them (join_into)
    f->pending = true;
    if (e != hipSuccess) {
        std::string msg = std::string("pbf_create: ") + hipGetErrorString(e);
        pbf_destroy(f);
        return fail(PBF_ERR_HIP, msg);
    }
    *out = f;
    return PBF_OK;
}

int pbf_destroy(pbf_filter_t* f) {
    if (!f) return PBF_OK;
    (void)hipSetDevice(f->device);
    // Everything that reads this filter's bitmap is ordered before the end of its stream: its
    // own calls run there, and a multi-filter probe that read it on another filter's stream made
    // this stream wait for that probe (probe_multi_device's closing joins).  So after this sync
    // the bitmap can go back to the recycle cache.  (Scratch sets keep their last_stream: pooled
    // streams are never destroyed, so a later lease from another stream still waits on the
    // set's event.)
    if (f->stream) (void)hipStreamSynchronize(f->stream);
    svc_release(f);  // (no request names f any more: its callers have returned)
    if (f->bitmap) bitmap_release(f->device, bitmap_alloc_bytes(f->alloc_words), f->bitmap);
    if (f->ev) (void)hipEventDestroy(f->ev);
    if (f->wait_ev) (void)hipEventDestroy(f->wait_ev);
    if (f->sig_ev) (void)hipEventDestroy(f->sig_ev);
    delete f;  // the stream belongs to the device's pool
    return PBF_OK;
}

int pbf_trim(int device) {
    HIP_TRY(hipSetDevice(device));
    bitmap_cache_trim(device);
    {
        // the cached bitmaps went back to the device's stream-ordered pool (release threshold
        // raised, bitmap_alloc): hand its free blocks back to the device
        hipMemPool_t pool = nullptr;
        if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) HIP_TRY(hipMemPoolTrimTo(pool, 0));
        else (void)hipGetLastError();
    }
    DevicePool& pool = device_pool(device);
    std::lock_guard<std::mutex> lock(pool.mu);
    for (Scratch* sc : pool.sets) {
        if (sc->leased) continue;
        if (sc->last) HIP_TRY(hipEventSynchronize(sc->last));
        sc->release_all();
    }
    return PBF_OK;
}

int pbf_scratch_bytes(int device, uint64_t* out) {
    if (!out) return fail(PBF_ERR_INVALID, "null out");
    DevicePool& pool = device_pool(device);
    std::lock_guard<std::mutex> lock(pool.mu);
    uint64_t t = 0;
    for (Scratch* sc : pool.sets)
        for (const DevBuf* d : {&sc->regions, &sc->fill, &sc->ovf, &sc->ovf_count, &sc->pref, &sc->rbits, &sc->neg, &sc->hw, &sc->dkeys, &sc->doffs, &sc->dout, &sc->svals, &sc->splan,
                                &sc->ssec, &sc->serr})
            t += d->bytes;
    *out = t;
    return PBF_OK;
}

int pbf_clear(pbf_filter_t* f) {
    LOCK(f);
    int rc = enter(f);
    if (rc) return rc;
    f->pending = true;
    if (f->tiled_ok) {
        // The next tiled build rewrites every reachable word; a read or an atomic build
        // materialises the zero bitmap first.  Only a from_bytes() can have dirtied the
        // unreachable middle of an m > 2^32 filter.
        if (f->tm.cspace && f->middle_dirty) {
            const uint64_t lo_w = (uint64_t(1) << 31) / 32;
            const uint64_t hi_w = f->tm.delta_words + lo_w;
            HIP_TRY(hipMemsetAsync(f->bitmap + lo_w, 0, (hi_w - lo_w) * 4, f->stream));
            f->middle_dirty = false;
        }
        f->pristine = true;
        return PBF_OK;
    }
    HIP_TRY(hipMemsetAsync(f->bitmap, 0, f->alloc_words * 4, f->stream));
    f->pristine = false;
    return PBF_OK;
}

int pbf_add_fixed(pbf_filter_t* f, const uint8_t* keys, uint32_t key_len, uint64_t n, int on_device) {
    if (key_len == 0 && n > 0) {
        // n empty keys: the variable-length path with all-equal offsets
        LOCK(f);
        int rc = enter(f);
        if (rc) return rc;
        if (f->k == 0) return PBF_OK;
        LEASE(f);
        HIP_TRY(f->sc->doffs.ensure((n + 1) * 8));
        HIP_TRY(hipMemsetAsync(f->sc->doffs.p, 0, (n + 1) * 8, f->stream));
        HIP_TRY(f->sc->dkeys.ensure(16));
        rc = add_device(f, make_batch(static_cast<const uint8_t*>(f->sc->dkeys.p),
                                      static_cast<const uint64_t*>(f->sc->doffs.p), 0, n));
        if (rc) return rc;
        if (!on_device) WAIT(f);
        return PBF_OK;
    }
    return add_impl(f, keys, nullptr, key_len, n, on_device);
}

// SURVEY.md §8b's name for the batch add (BloomFilter.add over n keys, bloom_filter.py:60-65).
int pbf_build(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint64_t n, int keys_on_device) {
    return pbf_add(f, keys, offsets, n, keys_on_device);
}

int pbf_add(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint64_t n, int on_device) {
    if (!offsets && n > 0) return fail(PBF_ERR_INVALID, "null offsets");
    return add_impl(f, keys ? keys : reinterpret_cast<const uint8_t*>(offsets), offsets, 0, n, on_device);
}

int pbf_probe_fixed(pbf_filter_t* f, const uint8_t* keys, uint32_t key_len, uint64_t n, uint8_t* hitmask,
                    int on_device) {
    if (key_len == 0 && n > 0) return fail(PBF_ERR_INVALID, "key_len 0: use pbf_probe with offsets");
    return probe_impl(f, keys, nullptr, key_len, n, hitmask, on_device);
}

int pbf_probe(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint8_t* hitmask,
              int on_device) {
    if (!offsets && n > 0) return fail(PBF_ERR_INVALID, "null offsets");
    return probe_impl(f, keys ? keys : reinterpret_cast<const uint8_t*>(offsets), offsets, 0, n, hitmask, on_device);
}

// Host batches over filters on several devices fan out to one host thread per device.
static bool multi_device(pbf_filter_t* const* fs, uint32_t nf) {
    for (uint32_t i = 1; i < nf; ++i)
        if (fs[i] && fs[0] && fs[i]->device != fs[0]->device) return true;
    return false;
}

static int by_device(pbf_filter_t* const* fs, uint32_t nf, std::vector<uint32_t>& group_of) {
    group_of.resize(nf);
    for (uint32_t i = 0; i < nf; ++i) {
        if (!fs[i]) return fail(PBF_ERR_INVALID, "null filter handle in set");
        group_of[i] = uint32_t(fs[i]->device);
    }
    return PBF_OK;
}

int pbf_probe_multi_fixed(pbf_filter_t* const* filters, uint32_t nfilters, const uint8_t* keys, uint32_t key_len,
                          uint64_t n, uint8_t* const* hitmasks, int on_device) {
    if (key_len == 0 && n > 0) return fail(PBF_ERR_INVALID, "key_len 0: use pbf_probe_multi with offsets");
    if (!on_device && filters && hitmasks && multi_device(filters, nfilters)) {
        std::vector<uint32_t> grp;
        int rc = by_device(filters, nfilters, grp);
        if (rc) return rc;
        return probe_multi_groups(filters, nfilters, grp.data(), keys, nullptr, key_len, n, hitmasks);
    }
    return probe_multi_impl(filters, nfilters, keys, nullptr, key_len, n, hitmasks, on_device);
}

int pbf_probe_multi(pbf_filter_t* const* filters, uint32_t nfilters, const uint8_t* keys, const uint64_t* offsets,
                    uint64_t n, uint8_t* const* hitmasks, int on_device) {
    if (!offsets && n > 0) return fail(PBF_ERR_INVALID, "null offsets");
    const uint8_t* kp = keys ? keys : reinterpret_cast<const uint8_t*>(offsets);
    if (!on_device && filters && hitmasks && multi_device(filters, nfilters)) {
        std::vector<uint32_t> grp;
        int rc = by_device(filters, nfilters, grp);
        if (rc) return rc;
        return probe_multi_groups(filters, nfilters, grp.data(), kp, offsets, 0, n, hitmasks);
    }
    return probe_multi_impl(filters, nfilters, kp, offsets, 0, n, hitmasks, on_device);
}

int pbf_plan_groups(const uint32_t* group_of, const int32_t* device_of, uint32_t n, uint32_t* slot_of,
                    uint32_t* ngroups) {
    if (n && (!group_of || !device_of || !slot_of)) return fail(PBF_ERR_INVALID, "null group, device or slot array");
    std::vector<uint32_t> ids;   // distinct groups in first-appearance order
    std::vector<int32_t> gdev;  // each group's device
    for (uint32_t i = 0; i < n; ++i) {
        const size_t g = size_t(std::find(ids.begin(), ids.end(), group_of[i]) - ids.begin());
        if (g == ids.size()) {
            ids.push_back(group_of[i]);
            gdev.push_back(device_of[i]);
        } else if (gdev[g] != device_of[i]) {
            return fail(PBF_ERR_INVALID, "the filters of one placement group must share a device");
        }
        slot_of[i] = uint32_t(g);
    }
    if (ngroups) *ngroups = uint32_t(ids.size());
    return PBF_OK;
}

int pbf_probe_multi_placed(pbf_filter_t* const* filters, uint32_t nfilters, const uint32_t* group_of,
                           const uint8_t* keys, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                           uint8_t* const* hitmasks) {
    if (nfilters == 0) return PBF_OK;
    if (!filters || !hitmasks || !group_of) return fail(PBF_ERR_INVALID, "null filter, group or hitmask array");
    if (!offsets && key_len == 0 && n > 0) return fail(PBF_ERR_INVALID, "fixed keys need key_len > 0");
    for (uint32_t i = 0; i < nfilters; ++i)
        if (n && !hitmasks[i]) return fail(PBF_ERR_INVALID, "null hitmask in set");
    const uint8_t* kp = keys ? keys : reinterpret_cast<const uint8_t*>(offsets);
    return probe_multi_groups(filters, nfilters, group_of, kp, offsets, offsets ? 0 : key_len, n, hitmasks);
}

int pbf_hash_indices_fixed(pbf_filter_t* f, const uint8_t* keys, uint32_t key_len, uint64_t n, uint64_t* out,
                           int on_device) {
    if (key_len == 0 && n > 0) return fail(PBF_ERR_INVALID, "key_len 0: use pbf_hash_indices with offsets");
    return hash_impl(f, keys, nullptr, key_len, n, out, on_device);
}

int pbf_hash_indices(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint64_t* out,
                     int on_device) {
    if (!offsets && n > 0) return fail(PBF_ERR_INVALID, "null offsets");
    return hash_impl(f, keys ? keys : reinterpret_cast<const uint8_t*>(offsets), offsets, 0, n, out, on_device);
}

int pbf_get_bitmap(pbf_filter_t* f, uint8_t* out, uint64_t nb_bytes) {
    LOCK(f);
    int rc = enter(f);
    if (rc) return rc;
    if (nb_bytes != f->nb_bytes) return fail(PBF_ERR_INVALID, "nb_bytes mismatch");
    if (!out) return fail(PBF_ERR_INVALID, "null out");
    rc = materialise(f);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, f->bitmap, nb_bytes, hipMemcpyDeviceToHost, f->stream));
    WAIT(f);
    return PBF_OK;
}

int pbf_set_bitmap(pbf_filter_t* f, const uint8_t* in, uint64_t nb_bytes) {
    LOCK(f);
    int rc = enter(f);
    if (rc) return rc;
    if (nb_bytes != f->nb_bytes) return fail(PBF_ERR_INVALID, "nb_bytes mismatch");
    if (!in) return fail(PBF_ERR_INVALID, "null input");
    if (f->alloc_words * 4 > nb_bytes)
        HIP_TRY(hipMemsetAsync(reinterpret_cast<uint8_t*>(f->bitmap) + nb_bytes, 0, f->alloc_words * 4 - nb_bytes,
                               f->stream));
    HIP_TRY(hipMemcpyAsync(f->bitmap, in, nb_bytes, hipMemcpyHostToDevice, f->stream));
    WAIT(f);
    f->pristine = false;
    f->middle_dirty = f->tm.cspace != 0;
    return PBF_OK;
}

int pbf_set_bitmap_device(pbf_filter_t* f, const void* in_dev, uint64_t nb_bytes) {
    LOCK(f);
    int rc = enter(f);
    if (rc) return rc;
    if (nb_bytes != f->nb_bytes) return fail(PBF_ERR_INVALID, "nb_bytes mismatch");
    if (!in_dev) return fail(PBF_ERR_INVALID, "null input");
    f->pending = true;
    if (f->alloc_words * 4 > nb_bytes)
        HIP_TRY(hipMemsetAsync(reinterpret_cast<uint8_t*>(f->bitmap) + nb_bytes, 0, f->alloc_words * 4 - nb_bytes,
                               f->stream));
    HIP_TRY(hipMemcpyAsync(f->bitmap, in_dev, nb_bytes, hipMemcpyDeviceToDevice, f->stream));
    f->pristine = false;
    f->middle_dirty = f->tm.cspace != 0;
    return PBF_OK;
}

int pbf_get_bitmap_device(pbf_filter_t* f, void* out_dev, uint64_t nb_bytes) {
    LOCK(f);
    int rc = enter(f);
    if (rc) return rc;
    if (nb_bytes != f->nb_bytes) return fail(PBF_ERR_INVALID, "nb_bytes mismatch");
    if (!out_dev) return fail(PBF_ERR_INVALID, "null out");
    rc = materialise(f);
    if (rc) return rc;
    f->pending = true;
    HIP_TRY(hipMemcpyAsync(out_dev, f->bitmap, nb_bytes, hipMemcpyDeviceToDevice, f->stream));
    return PBF_OK;
}

int pbf_copy_filter(pbf_filter_t* src, int dst_device, int flags, pbf_filter_t** out) {
    if (!out) return fail(PBF_ERR_INVALID, "null out");
    *out = nullptr;
    if (flags & ~PBF_COPY_BOUNCE) return fail(PBF_ERR_INVALID, "bad copy flags");
    LOCK(src);  // exclusive: no build or load of src while its bitmap is read
    int rc = enter(src);
    if (rc) return rc;
    pbf_filter_t* dst = nullptr;
    rc = pbf_create(dst_device, src->nb_bytes, src->k, &dst);
    if (rc) return rc;
    rc = copy_filter_into(src, dst, (flags & PBF_COPY_BOUNCE) != 0);
    if (rc) {
        const std::string msg = g_last_error;
        pbf_destroy(dst);
        return fail(rc, msg);
    }
    *out = dst;
    return PBF_OK;
}

int pbf_popcount(pbf_filter_t* f, uint64_t* out) {
    LOCK(f);
    int rc = enter(f);
    if (rc) return rc;
    if (!out) return fail(PBF_ERR_INVALID, "null out");
    rc = materialise(f);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(f->dpop, 0, 8, f->stream));
    k_popcount<<<grid_for(f->alloc_words, 256, 4096), 256, 0, f->stream>>>(
        f->bitmap, f->alloc_words, reinterpret_cast<unsigned long long*>(f->dpop));
    LAUNCHED(f, "k_popcount");
    HIP_TRY(hipMemcpyAsync(out, f->dpop, 8, hipMemcpyDeviceToHost, f->stream));
    WAIT(f);
    return PBF_OK;
}

int pbf_sync(pbf_filter_t* f) {
    LOCK(f);
    int rc = enter(f);
    if (rc) return rc;
    return wait_stream(f);
}

int pbf_index_params(uint64_t nb_bytes, uint32_t* mode, uint64_t* magic, uint32_t* shift) {
    if (!mode || !magic || !shift) return fail(PBF_ERR_INVALID, "null out");
    if (nb_bytes == 0) return fail(PBF_ERR_ZERO_SIZE, "nb_bytes == 0 (integer modulo by zero)");
    const IndexMap im = make_index_map(nb_bytes * 8);
    *mode = im.mode;
    *magic = im.magic;
    *shift = im.mask;
    return PBF_OK;
}

int pbf_wait_stream(pbf_filter_t* f, void* stream) {
    LOCK(f);
    int rc = enter(f);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (s == f->stream) return PBF_OK;
    if (!f->wait_ev) HIP_TRY(hipEventCreateWithFlags(&f->wait_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(f->wait_ev, s));
    HIP_TRY(hipStreamWaitEvent(f->stream, f->wait_ev, 0));
    f->pending = true;  // the filter's stream now has (a wait) queued
    return PBF_OK;
}

int pbf_signal_stream(pbf_filter_t* f, void* stream) {
    LOCK(f);
    int rc = enter(f);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (s == f->stream) return PBF_OK;
    if (!f->sig_ev) HIP_TRY(hipEventCreateWithFlags(&f->sig_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(f->sig_ev, f->stream));
    HIP_TRY(hipStreamWaitEvent(s, f->sig_ev, 0));
    return PBF_OK;
}

int pbf_resident_enable(int on) {
    g_resident_on.store(on ? 1 : 0);
    return PBF_OK;
}

int pbf_resident_stats(int device, uint64_t* requests, uint64_t* device_ns) {
    if (!requests || !device_ns) return fail(PBF_ERR_INVALID, "null out");
    *requests = *device_ns = 0;
    ResidentReader* rr = device >= 0 && device < 64 ? g_resident_fast[device].load(std::memory_order_acquire) : nullptr;
    if (rr && rr->khz) {
        *requests = rr->answered.load(std::memory_order_relaxed);
        *device_ns = rr->answer_ticks.load(std::memory_order_relaxed) * 1000000ull / rr->khz;
    }
    return PBF_OK;
}

int pbf_resident_launches(int device, uint32_t* launches) {
    if (!launches) return fail(PBF_ERR_INVALID, "null out");
    *launches = 0;
    ResidentReader* rr = nullptr;
    {
        std::lock_guard<std::mutex> lock(g_resident_mu);
        auto it = g_resident.find(device);
        if (it != g_resident.end()) rr = it->second;
    }
    if (rr) {
        std::lock_guard<std::mutex> lock(rr->mu);
        *launches = rr->launches;
    }
    return PBF_OK;
}

int pbf_murmur3_x86_32(int device, const uint8_t* key, uint64_t len, uint32_t seed, int32_t* out) {
    if (!out || (len && !key)) return fail(PBF_ERR_INVALID, "null key or out");
    if (len > kOneKeyMax) return fail(PBF_ERR_INVALID, "key longer than 4096 bytes");
    HIP_TRY(hipSetDevice(device));
    OneKeyStage* st = nullptr;
    int rc = one_key_stage(device, &st);
    if (rc) return rc;
    if (len) std::memcpy(st->host + kOneKeyData, key, len);
    int32_t* res = reinterpret_cast<int32_t*>(st->host + 8);
    *reinterpret_cast<volatile int32_t*>(res) = 0;
    k_murmur_one<<<1, 64, 0, nullptr>>>(st->dev + kOneKeyData, uint32_t(len), seed,
                                          reinterpret_cast<int32_t*>(st->dev + 8));
    CHECK_LAUNCH();
    HIP_TRY(hipStreamSynchronize(nullptr));
    *out = *reinterpret_cast<volatile int32_t*>(res);
    return PBF_OK;
}

int pbf_may_contain(pbf_filter_t* f, const uint8_t* key, uint64_t len, int* out) {
    if (!f) return fail(PBF_ERR_INVALID, "null filter handle");
    if (!out || (len && !key)) return fail(PBF_ERR_INVALID, "null key or out");
    {
        // a built filter: readers share the handle and each runs on its reader stream
        std::shared_lock<std::shared_mutex> rl(f->mu);
        if (reader_ok(f, len)) {
            if (f->k == 0) {  // the AND over no bits (bloom_filter.py:71-74 runs no iteration)
                *out = 1;
                return PBF_OK;
            }
            // the resident reader first: no HIP call on its path (no hipSetDevice either)
            int rc = one_key_resident(f, key, len, out);
            if (rc != kNotTaken) return rc;
            rc = enter(f);
            if (rc) return rc;
            hipStream_t rs = nullptr;
            HIP_TRY(reader_stream(f->device, &rs));
            return one_key_probe(f, key, len, out, rs, true);
        }
    }
    LOCK(f);
    return may_contain_locked(f, key, len, out);
}

int pbf_may_contain_set(pbf_filter_t* const* filters, uint32_t nfilters, const uint8_t* key, uint64_t len,
                        uint8_t* out_bits) {
    if (nfilters == 0) return PBF_OK;
    if (!filters || !out_bits || (len && !key)) return fail(PBF_ERR_INVALID, "null pointer");
    for (uint32_t i = 0; i < nfilters; ++i) {
        if (!filters[i]) return fail(PBF_ERR_INVALID, "null filter handle in set");
        if (filters[i]->device != filters[0]->device) return fail(PBF_ERR_INVALID, "filters of one set must share a device");
    }
    if (nfilters <= kSvcFilters) {
        // LsmStorage.get's usual set (product-sized filters of one k, at most 64): straight to the
        // resident reader with no allocation -- the distinct handles in address order on the stack,
        // held shared while the reader answers
        pbf_filter_t* ord[kSvcFilters];
        std::copy(filters, filters + nfilters, ord);
        std::sort(ord, ord + nfilters);
        const uint32_t nu = uint32_t(std::unique(ord, ord + nfilters) - ord);
        struct Held {
            pbf_filter_t** p;
            uint32_t n = 0;
            ~Held() {
                for (uint32_t i = 0; i < n; ++i) p[i]->mu.unlock_shared();
            }
        } held{ord};
        const uint32_t k0 = filters[0]->k;
        bool ok = k0 > 0 && kmax_for(k0) > 0;
        for (uint32_t i = 0; i < nu && ok; ++i) {
            ord[i]->mu.lock_shared();
            held.n = i + 1;
            ok = ord[i]->k == k0 && reader_ok(ord[i], len);
        }
        if (ok) {
            uint64_t bits = 0;
            bool taken = false;
            const int rc = resident_probe(filters[0]->device, filters, nfilters, k0, key, len, &bits, &taken);
            if (rc) return rc;
            if (taken) {
                std::memset(out_bits, 0, (nfilters + 7) / 8);
                for (uint32_t i = 0; i < nfilters; ++i)
                    if ((bits >> i) & 1u) out_bits[i >> 3] |= uint8_t(1u << (i & 7));
                for (uint32_t i = 0; i < nu; ++i) {
                    ord[i]->last_probe_mode.store(PBF_PROBE_DIRECT, std::memory_order_relaxed);
                    ord[i]->last_probe_detail.store(PBF_DETAIL_ONE_KEY | PBF_DETAIL_SET | PBF_DETAIL_RESIDENT,
                                                    std::memory_order_relaxed);
                }
                return PBF_OK;
            }
        }
        // otherwise (locks released here): the general path below
    }
    // every distinct handle of the set, in address order (a table may appear twice)
    std::vector<pbf_filter_t*> order(filters, filters + nfilters);
    std::sort(order.begin(), order.end());
    order.erase(std::unique(order.begin(), order.end()), order.end());
    {
        // built filters: held shared, the launch on the thread's reader stream
        std::vector<std::shared_lock<std::shared_mutex>> rlocks;
        rlocks.reserve(order.size());
        bool ok = true;
        for (pbf_filter_t* p : order) {
            rlocks.emplace_back(p->mu);
            if (!reader_ok(p, len)) {
                ok = false;
                break;
            }
        }
        if (ok) {
            // every filter of one k (LsmStorage.get's usual set: product-sized SSTable filters,
            // fp 0.001 -> k = 10), at most 64 of them: straight to the resident reader, no HIP call
            const uint32_t k0 = filters[0]->k;
            bool one_k = nfilters <= kSvcFilters && k0 > 0 && kmax_for(k0) > 0;
            for (uint32_t i = 1; i < nfilters && one_k; ++i) one_k = filters[i]->k == k0;
            if (one_k) {
                uint64_t bits = 0;
                bool taken = false;
                const int rc = resident_probe(filters[0]->device, filters, nfilters, k0, key, len, &bits, &taken);
                if (rc) return rc;
                if (taken) {
                    std::memset(out_bits, 0, (nfilters + 7) / 8);
                    for (uint32_t i = 0; i < nfilters; ++i) {
                        if ((bits >> i) & 1u) out_bits[i >> 3] |= uint8_t(1u << (i & 7));
                        filters[i]->last_probe_mode = PBF_PROBE_DIRECT;
                        filters[i]->last_probe_detail = PBF_DETAIL_ONE_KEY | PBF_DETAIL_SET | PBF_DETAIL_RESIDENT;
                    }
                    return PBF_OK;
                }
            }
            HIP_TRY(hipSetDevice(filters[0]->device));
            hipStream_t rs = nullptr;
            HIP_TRY(reader_stream(filters[0]->device, &rs));
            return may_contain_set_locked(filters, nfilters, key, len, out_bits, rs);
        }
    }
    std::vector<std::unique_lock<std::shared_mutex>> locks;
    locks.reserve(order.size());
    for (pbf_filter_t* p : order) locks.emplace_back(p->mu);
    return may_contain_set_locked(filters, nfilters, key, len, out_bits);
}

void* pbf_stream(pbf_filter_t* f) { return f ? static_cast<void*>(f->stream) : nullptr; }
void* pbf_device_bitmap(pbf_filter_t* f) {
    if (!f) return nullptr;
    if (materialise(f)) return nullptr;
    return f->bitmap;
}

int pbf_set_build_mode(pbf_filter_t* f, int mode) {
    LOCK(f);
    if (mode < PBF_BUILD_AUTO || mode > PBF_BUILD_TILED) return fail(PBF_ERR_INVALID, "bad build mode");
    if (mode == PBF_BUILD_TILED && (!f->tiled_ok || f->k > 32 || !part_fits(f->tm.nbuckets, f->k, false)))
        return fail(PBF_ERR_INVALID, "tiled build unsupported for this m / k");
    f->mode = mode;
    return PBF_OK;
}

int pbf_last_build_mode(pbf_filter_t* f) { return f ? f->last_mode : 0; }

int pbf_set_probe_mode(pbf_filter_t* f, int mode) {
    LOCK(f);
    if (mode < PBF_PROBE_AUTO || mode > PBF_PROBE_TILED) return fail(PBF_ERR_INVALID, "bad probe mode");
    if (mode == PBF_PROBE_TILED &&
        (!f->tiled_ok || f->k > 32 || f->tm.tb > kSlotShift || !part_fits(f->tm.nbuckets, f->k, true)))
        return fail(PBF_ERR_INVALID, "tiled probe unsupported for this m / k");
    f->probe_mode = mode;
    return PBF_OK;
}

int pbf_last_probe_mode(pbf_filter_t* f) { return f ? f->last_probe_mode.load() : 0; }
uint32_t pbf_last_probe_detail(pbf_filter_t* f) { return f ? f->last_probe_detail.load() : 0u; }
uint32_t pbf_last_build_detail(pbf_filter_t* f) { return f ? f->last_build_detail : 0; }

int pbf_encode_data_blocks(int device, const uint8_t* keys, const uint64_t* key_offsets, const uint8_t* values,
                           const uint64_t* value_offsets, uint64_t n, const uint64_t* block_first,
                           const uint64_t* block_out, uint64_t nblocks, uint8_t* out, int on_device) {
    if (nblocks == 0) return PBF_OK;
    if (!key_offsets || !value_offsets || !block_first || !block_out || !out)
        return fail(PBF_ERR_INVALID, "null pointer");
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(allow_lds(k_encode_blocks, kEncodeLds));
    EncodeCtx& c = encode_ctx(device);
    std::lock_guard<std::mutex> lock(c.mu);
    if (!c.stream) {
        HIP_TRY(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
        register_stream(device, c.stream);
    }
    HIP_TRY(c.err.ensure(4));
    HIP_TRY(hipMemsetAsync(c.err.p, 0, 4, c.stream));
    const uint8_t *dk = keys, *dv = values;
    const uint64_t *dko = key_offsets, *dvo = value_offsets, *dbf = block_first, *dbo = block_out;
    uint8_t* dout = out;
    uint64_t out_bytes = 0;
    if (!on_device) {
        // the host plan is checked here: blocks cover records 0..n in order, each fits a block
        if (block_first[0] != 0 || block_first[nblocks] != n || block_out[0] != 0)
            return fail(PBF_ERR_INVALID, "block plan must cover records [0, n) from byte 0");
        for (uint64_t b = 0; b < nblocks; ++b) {
            const uint64_t r0 = block_first[b], r1 = block_first[b + 1];
            if (r1 < r0) return fail(PBF_ERR_INVALID, "block plan not monotonic");
            const uint64_t dl = (key_offsets[r1] - key_offsets[r0]) + (value_offsets[r1] - value_offsets[r0]) + 8 * (r1 - r0);
            if (dl > kMaxBlockData) return fail(PBF_ERR_INVALID, "a block's records exceed 65536 bytes");
            if (block_out[b + 1] - block_out[b] != dl + 2 * (r1 - r0) + 2)
                return fail(PBF_ERR_INVALID, "block_out does not match the blocks' encoded sizes");
        }
        out_bytes = block_out[nblocks];
        const uint64_t kb = key_offsets[n], vb = value_offsets[n];
        HIP_TRY(c.keys.ensure(kb + 16));
        HIP_TRY(c.vals.ensure(vb + 16));
        HIP_TRY(c.offs.ensure((2 * (n + 1) + 2 * (nblocks + 1)) * 8));
        HIP_TRY(c.out.ensure(out_bytes + 16));
        auto* o = static_cast<uint64_t*>(c.offs.p);
        if (kb) HIP_TRY(hipMemcpyAsync(c.keys.p, keys, kb, hipMemcpyHostToDevice, c.stream));
        if (vb) HIP_TRY(hipMemcpyAsync(c.vals.p, values, vb, hipMemcpyHostToDevice, c.stream));
        HIP_TRY(hipMemcpyAsync(o, key_offsets, (n + 1) * 8, hipMemcpyHostToDevice, c.stream));
        HIP_TRY(hipMemcpyAsync(o + n + 1, value_offsets, (n + 1) * 8, hipMemcpyHostToDevice, c.stream));
        HIP_TRY(hipMemcpyAsync(o + 2 * (n + 1), block_first, (nblocks + 1) * 8, hipMemcpyHostToDevice, c.stream));
        HIP_TRY(hipMemcpyAsync(o + 2 * (n + 1) + nblocks + 1, block_out, (nblocks + 1) * 8, hipMemcpyHostToDevice,
                               c.stream));
        dk = static_cast<const uint8_t*>(c.keys.p);
        dv = static_cast<const uint8_t*>(c.vals.p);
        dko = o;
        dvo = o + n + 1;
        dbf = o + 2 * (n + 1);
        dbo = o + 2 * (n + 1) + nblocks + 1;
        dout = static_cast<uint8_t*>(c.out.p);
    }
    hipStream_t s = on_device ? nullptr : c.stream;
    if (on_device) HIP_TRY(hipMemsetAsync(c.err.p, 0, 4, s));
    k_encode_blocks<<<uint32_t(nblocks), 512, kEncodeLds, s>>>(dk, dko, dv, dvo, dbf, dbo, dout,
                                                               static_cast<unsigned int*>(c.err.p));
    CHECK_LAUNCH();
    unsigned int err = 0;
    HIP_TRY(hipMemcpyAsync(&err, c.err.p, 4, hipMemcpyDeviceToHost, s));
    if (!on_device) HIP_TRY(hipMemcpyAsync(out, dout, out_bytes, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (err) return fail(PBF_ERR_INVALID, std::to_string(err) + " block(s) exceed 65536 data bytes; not written");
    return PBF_OK;
}

int pbf_build_sstable(pbf_filter_t* f, const uint8_t* keys, const uint64_t* key_offsets, const uint8_t* values,
                      const uint64_t* value_offsets, uint64_t n, const uint64_t* block_first, const uint64_t* block_out,
                      uint64_t nblocks, uint8_t* data_out, uint8_t* bitmap_out) {
    LOCK(f);
    int rc = enter(f);
    if (rc) return rc;
    if (n == 0 || nblocks == 0) return fail(PBF_ERR_INVALID, "an SSTable needs at least one record");
    if (!keys || !key_offsets || !values || !value_offsets || !block_first || !block_out || !data_out)
        return fail(PBF_ERR_INVALID, "null pointer");
    if (key_offsets[0] != 0 || value_offsets[0] != 0) return fail(PBF_ERR_INVALID, "offsets must start at 0");
    // the host plan is checked as in pbf_encode_data_blocks
    if (block_first[0] != 0 || block_first[nblocks] != n || block_out[0] != 0)
        return fail(PBF_ERR_INVALID, "block plan must cover records [0, n) from byte 0");
    for (uint64_t b = 0; b < nblocks; ++b) {
        const uint64_t r0 = block_first[b], r1 = block_first[b + 1];
        if (r1 < r0) return fail(PBF_ERR_INVALID, "block plan not monotonic");
        const uint64_t dl = (key_offsets[r1] - key_offsets[r0]) + (value_offsets[r1] - value_offsets[r0]) + 8 * (r1 - r0);
        if (dl > kMaxBlockData) return fail(PBF_ERR_INVALID, "a block's records exceed 65536 bytes");
        if (block_out[b + 1] - block_out[b] != dl + 2 * (r1 - r0) + 2)
            return fail(PBF_ERR_INVALID, "block_out does not match the blocks' encoded sizes");
    }
    HIP_TRY(allow_lds(k_encode_blocks, kEncodeLds));
    LEASE(f);
    Scratch* sc = f->sc;
    hipStream_t s = f->stream;
    const uint64_t kb = key_offsets[n], vb = value_offsets[n], out_bytes = block_out[nblocks];
    HIP_TRY(sc->dkeys.ensure(((kb + 15) & ~uint64_t(15)) + 32));
    HIP_TRY(sc->doffs.ensure((n + 1) * 8));
    HIP_TRY(sc->svals.ensure(((vb + 15) & ~uint64_t(15)) + 32 + (n + 1) * 8));
    HIP_TRY(sc->splan.ensure(2 * (nblocks + 1) * 8));
    HIP_TRY(sc->ssec.ensure(out_bytes + 32));
    HIP_TRY(sc->serr.ensure(4));
    auto* dk = static_cast<uint8_t*>(sc->dkeys.p);
    auto* dko = static_cast<uint64_t*>(sc->doffs.p);
    auto* dv = static_cast<uint8_t*>(sc->svals.p);
    auto* dvo = reinterpret_cast<uint64_t*>(dv + ((vb + 15) & ~uint64_t(15)) + 32);
    auto* dbf = static_cast<uint64_t*>(sc->splan.p);
    auto* dbo = dbf + nblocks + 1;
    // Page-lock the large host spans for the duration of the call so the copies are direct DMA
    // (pageable copies go through the runtime's staging at a fraction of the rate); spans that
    // are already pinned, or cannot be registered, are copied as they are.
    std::vector<void*> registered;
    auto lock_span = [&](const void* p, uint64_t bytes) {
        if (bytes < (uint64_t(4) << 20) || is_pinned_host(p)) return;
        if (hipHostRegister(const_cast<void*>(p), bytes, hipHostRegisterDefault) == hipSuccess)
            registered.push_back(const_cast<void*>(p));
        else
            (void)hipGetLastError();
    };
    struct Unregister {
        std::vector<void*>& v;
        ~Unregister() {
            for (void* p : v) (void)hipHostUnregister(p);
        }
    } unreg{registered};
    lock_span(keys, kb);
    lock_span(values, vb);
    lock_span(key_offsets, (n + 1) * 8);
    lock_span(value_offsets, (n + 1) * 8);
    lock_span(data_out, out_bytes);
    // one H2D of the packed records; the data blocks and the filter are both built from it
    if (kb) HIP_TRY(hipMemcpyAsync(dk, keys, kb, hipMemcpyHostToDevice, s));
    if (vb) HIP_TRY(hipMemcpyAsync(dv, values, vb, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dko, key_offsets, (n + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dvo, value_offsets, (n + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dbf, block_first, (nblocks + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dbo, block_out, (nblocks + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(sc->serr.p, 0, 4, s));
    k_encode_blocks<<<uint32_t(nblocks), 512, kEncodeLds, s>>>(dk, dko, dv, dvo, dbf, dbo, static_cast<uint8_t*>(sc->ssec.p),
                                                               static_cast<unsigned int*>(sc->serr.p));
    LAUNCHED(f, "k_encode_blocks");
    if (f->k > 0) {  // SSTableBuilder.build's filter over every key (sstable.py:274)
        rc = add_device(f, make_batch(dk, dko, 0, n));
        if (rc) return rc;
    }
    unsigned int err = 0;
    HIP_TRY(hipMemcpyAsync(&err, sc->serr.p, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(data_out, sc->ssec.p, out_bytes, hipMemcpyDeviceToHost, s));
    if (bitmap_out) {
        rc = materialise(f);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(bitmap_out, f->bitmap, f->nb_bytes, hipMemcpyDeviceToHost, s));
    }
    WAIT(f);
    if (err) return fail(PBF_ERR_INVALID, std::to_string(err) + " block(s) exceed 65536 data bytes");
    return PBF_OK;
}

// Compaction's N output SSTables (src/lsm_storage.py:233-251) from ONE upload of the record
// run: the host plan (pebbledb_amd/sstable_data.plan_compaction: every output's blocks, laid end
// to end) is encoded by one k_encode_blocks launch for all outputs; output t's filter is built
// from its slice of the same device keys on its own stream (the filters' streams are dealt
// round-robin from the device's pool, so up to 8 builds run side by side); the data sections
// leave on filters[0]'s stream while the filters build.  Synchronous.
int pbf_build_sstables(pbf_filter_t* const* filters, uint32_t ntables, const uint8_t* keys, const uint64_t* key_offsets,
                       const uint8_t* values, const uint64_t* value_offsets, uint64_t n, const uint64_t* block_first,
                       const uint64_t* block_out, uint64_t nblocks, const uint64_t* table_blocks,
                       uint8_t* const* data_outs, uint8_t* const* bitmap_outs) {
    if (ntables == 0) return PBF_OK;
    if (!filters || !keys || !key_offsets || !values || !value_offsets || !block_first || !block_out || !table_blocks ||
        !data_outs)
        return fail(PBF_ERR_INVALID, "null pointer");
    for (uint32_t t = 0; t < ntables; ++t) {
        if (!filters[t] || !data_outs[t]) return fail(PBF_ERR_INVALID, "null filter or output in the set");
        if (filters[t]->device != filters[0]->device) return fail(PBF_ERR_INVALID, "the outputs' filters must share a device");
        for (uint32_t j = 0; j < t; ++j)
            if (filters[j] == filters[t]) return fail(PBF_ERR_INVALID, "a filter appears twice");
    }
    if (key_offsets[0] != 0 || value_offsets[0] != 0) return fail(PBF_ERR_INVALID, "offsets must start at 0");
    if (nblocks == 0 || block_first[0] != 0 || block_out[0] != 0 || block_first[nblocks] > n)
        return fail(PBF_ERR_INVALID, "block plan must cover records [0, written) from byte 0");
    if (table_blocks[0] != 0 || table_blocks[ntables] != nblocks) return fail(PBF_ERR_INVALID, "tables must cover the blocks");
    for (uint32_t t = 0; t < ntables; ++t)
        if (table_blocks[t + 1] <= table_blocks[t]) return fail(PBF_ERR_INVALID, "a table without blocks");
    for (uint64_t b = 0; b < nblocks; ++b) {
        const uint64_t r0 = block_first[b], r1 = block_first[b + 1];
        if (r1 <= r0) return fail(PBF_ERR_INVALID, "block plan not increasing");
        const uint64_t dl = (key_offsets[r1] - key_offsets[r0]) + (value_offsets[r1] - value_offsets[r0]) + 8 * (r1 - r0);
        if (dl > kMaxBlockData) return fail(PBF_ERR_INVALID, "a block's records exceed 65536 bytes");
        if (block_out[b + 1] - block_out[b] != dl + 2 * (r1 - r0) + 2)
            return fail(PBF_ERR_INVALID, "block_out does not match the blocks' encoded sizes");
    }
    const uint64_t w = block_first[nblocks];  // records written (the run's tail may be left out)
    // every handle of the set, in address order
    std::vector<pbf_filter_t*> order(filters, filters + ntables);
    std::sort(order.begin(), order.end());
    std::vector<std::unique_lock<std::shared_mutex>> locks;
    locks.reserve(ntables);
    for (pbf_filter_t* p : order) locks.emplace_back(p->mu);
    pbf_filter_t* f0 = filters[0];
    int rc = enter(f0);
    if (rc) return rc;
    HIP_TRY(allow_lds(k_encode_blocks, kEncodeLds));
    LEASE(f0);
    Scratch* sc = f0->sc;
    hipStream_t s0 = f0->stream;
    const uint64_t kb = key_offsets[w], vb = value_offsets[w], out_bytes = block_out[nblocks];
    HIP_TRY(sc->dkeys.ensure(((kb + 15) & ~uint64_t(15)) + 32));
    HIP_TRY(sc->doffs.ensure((w + 1) * 8));
    HIP_TRY(sc->svals.ensure(((vb + 15) & ~uint64_t(15)) + 32 + (w + 1) * 8));
    HIP_TRY(sc->splan.ensure(2 * (nblocks + 1) * 8));
    HIP_TRY(sc->ssec.ensure(out_bytes + 32));
    HIP_TRY(sc->serr.ensure(4));
    auto* dk = static_cast<uint8_t*>(sc->dkeys.p);
    auto* dko = static_cast<uint64_t*>(sc->doffs.p);
    auto* dv = static_cast<uint8_t*>(sc->svals.p);
    auto* dvo = reinterpret_cast<uint64_t*>(dv + ((vb + 15) & ~uint64_t(15)) + 32);
    auto* dbf = static_cast<uint64_t*>(sc->splan.p);
    auto* dbo = dbf + nblocks + 1;
    auto* dsec = static_cast<uint8_t*>(sc->ssec.p);
    std::vector<void*> registered;
    auto lock_span = [&](const void* p, uint64_t bytes) {
        if (bytes < (uint64_t(4) << 20) || is_pinned_host(p)) return;
        if (hipHostRegister(const_cast<void*>(p), bytes, hipHostRegisterDefault) == hipSuccess)
            registered.push_back(const_cast<void*>(p));
        else
            (void)hipGetLastError();
    };
    struct Unregister {
        std::vector<void*>& v;
        ~Unregister() {
            for (void* p : v) (void)hipHostUnregister(p);
        }
    } unreg{registered};
    lock_span(keys, kb);
    lock_span(values, vb);
    lock_span(key_offsets, (w + 1) * 8);
    lock_span(value_offsets, (w + 1) * 8);
    for (uint32_t t = 0; t < ntables; ++t) {
        lock_span(data_outs[t], block_out[table_blocks[t + 1]] - block_out[table_blocks[t]]);
        if (bitmap_outs && bitmap_outs[t]) lock_span(bitmap_outs[t], filters[t]->nb_bytes);
    }
    // one H2D of the run; the data blocks of every output and every filter are built from it
    if (kb) HIP_TRY(hipMemcpyAsync(dk, keys, kb, hipMemcpyHostToDevice, s0));
    if (vb) HIP_TRY(hipMemcpyAsync(dv, values, vb, hipMemcpyHostToDevice, s0));
    HIP_TRY(hipMemcpyAsync(dko, key_offsets, (w + 1) * 8, hipMemcpyHostToDevice, s0));
    HIP_TRY(hipMemcpyAsync(dvo, value_offsets, (w + 1) * 8, hipMemcpyHostToDevice, s0));
    HIP_TRY(hipMemcpyAsync(dbf, block_first, (nblocks + 1) * 8, hipMemcpyHostToDevice, s0));
    HIP_TRY(hipMemcpyAsync(dbo, block_out, (nblocks + 1) * 8, hipMemcpyHostToDevice, s0));
    HIP_TRY(hipMemsetAsync(sc->serr.p, 0, 4, s0));
    k_encode_blocks<<<uint32_t(nblocks), 512, kEncodeLds, s0>>>(dk, dko, dv, dvo, dbf, dbo, dsec,
                                                                static_cast<unsigned int*>(sc->serr.p));
    LAUNCHED(f0, "k_encode_blocks");
    HIP_TRY(filter_event(f0));
    HIP_TRY(hipEventRecord(f0->ev, s0));  // the run is on the device
    // the data sections go back on s0 while the filters build on their own streams
    for (uint32_t t = 0; t < ntables; ++t) {
        const uint64_t o0 = block_out[table_blocks[t]], o1 = block_out[table_blocks[t + 1]];
        HIP_TRY(hipMemcpyAsync(data_outs[t], dsec + o0, o1 - o0, hipMemcpyDeviceToHost, s0));
    }
    const Batch all = make_batch(dk, dko, 0, w);
    for (uint32_t t = 0; t < ntables; ++t) {
        pbf_filter_t* ft = filters[t];
        const uint64_t r0 = block_first[table_blocks[t]], r1 = block_first[table_blocks[t + 1]];
        if (ft != f0 && ft->stream != s0) HIP_TRY(hipStreamWaitEvent(ft->stream, f0->ev, 0));
        if (ft->k > 0) {  // SSTableBuilder.build's filter over the output's keys (sstable.py:274)
            if (ft == f0) {
                rc = add_device(ft, slice(all, r0, r1 - r0));
            } else {
                Lease lt(ft);
                rc = lt.acquire();
                if (!rc) rc = add_device(ft, slice(all, r0, r1 - r0));
            }
            if (rc) return rc;
        }
        if (bitmap_outs && bitmap_outs[t]) {
            rc = materialise(ft);
            if (rc) return rc;
            HIP_TRY(hipMemcpyAsync(bitmap_outs[t], ft->bitmap, ft->nb_bytes, hipMemcpyDeviceToHost, ft->stream));
        }
        ft->pending = true;
    }
    // s0 (whose lease covers the device copy of the run) waits for every build that read it
    for (uint32_t t = 1; t < ntables; ++t) {
        pbf_filter_t* ft = filters[t];
        if (ft->stream == s0) continue;
        HIP_TRY(filter_event(ft));
        HIP_TRY(hipEventRecord(ft->ev, ft->stream));
        HIP_TRY(hipStreamWaitEvent(s0, ft->ev, 0));
    }
    unsigned int err = 0;
    HIP_TRY(hipMemcpyAsync(&err, sc->serr.p, 4, hipMemcpyDeviceToHost, s0));
    WAIT(f0);
    for (uint32_t t = 1; t < ntables; ++t)
        if (filters[t]->pending) WAIT(filters[t]);
    if (err) return fail(PBF_ERR_INVALID, std::to_string(err) + " block(s) exceed 65536 data bytes");
    return PBF_OK;
}

int pbf_plan_blocks(const uint64_t* key_offsets, const uint64_t* value_offsets, uint64_t n, uint64_t block_size,
                    uint64_t* block_first, uint64_t* block_out, uint64_t* nblocks) {
    if (!key_offsets || !value_offsets || !block_first || !block_out || !nblocks) return fail(PBF_ERR_INVALID, "null pointer");
    if (n == 0) return fail(PBF_ERR_INVALID, "an SSTable needs at least one record");
    if (block_size == 0 || block_size > kMaxBlockData) return fail(PBF_ERR_INVALID, "block_size must be in (0, 65536]");
    // DataBlockBuilder.add (blocks.py:78-95): a record joins the open block iff the block's
    // record bytes stay <= block_size; a record larger than a block cannot be placed (the
    // reference would drop it, blocks.py:84-85)
    uint64_t nb = 0, used = 0, out = 0, cnt = 0;
    block_first[0] = 0;
    block_out[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t sz = (key_offsets[i + 1] - key_offsets[i]) + (value_offsets[i + 1] - value_offsets[i]) + 8;
        if (sz > block_size) return fail(PBF_ERR_INVALID, "a record is larger than block_size");
        if (cnt && used + sz > block_size) {
            out += used + 2 * cnt + 2;
            ++nb;
            block_first[nb] = i;
            block_out[nb] = out;
            used = 0;
            cnt = 0;
        }
        used += sz;
        ++cnt;
    }
    out += used + 2 * cnt + 2;
    ++nb;
    block_first[nb] = n;
    block_out[nb] = out;
    *nblocks = nb;
    return PBF_OK;
}

int pbf_plan_compaction(const uint64_t* key_offsets, const uint64_t* value_offsets, uint64_t n, uint64_t block_size,
                        uint64_t max_sstable_size, uint64_t* block_first, uint64_t* block_out, uint64_t* table_blocks,
                        uint64_t* nblocks, uint64_t* ntables, uint64_t* written) {
    if (!key_offsets || !value_offsets || !block_first || !block_out || !table_blocks || !nblocks || !ntables || !written)
        return fail(PBF_ERR_INVALID, "null pointer");
    if (block_size == 0 || block_size > kMaxBlockData) return fail(PBF_ERR_INVALID, "block_size must be in (0, 65536]");
    // (the reference tests the position after every add, lsm_storage.py:241, so a size of 0 would
    // make one table per record there; splitting where blocks finish agrees for any size > 0)
    if (max_sstable_size == 0) return fail(PBF_ERR_INVALID, "max_sstable_size must be positive");
    // LsmStorage._compact (lsm_storage.py:233-251) over the greedy blocks of DataBlockBuilder.add
    // (blocks.py:78-95): a builder's position advances when a record does not fit the open block
    // (sstable.py:246-266); at position >= max_sstable_size the builder is built, its last block
    // holding only that record; at the end the last builder is built only if its position is > 0
    uint64_t nb = 0, nt = 0, out = 0;  // blocks, tables, byte offset (outputs' data end to end)
    block_first[0] = 0;
    block_out[0] = 0;
    table_blocks[0] = 0;
    uint64_t i = 0;
    while (i < n) {
        uint64_t pos = 0, used = 0, cnt = 0;  // builder position; the open block's bytes / records
        bool split = false;
        const uint64_t nb_table0 = nb;
        for (; i < n; ++i) {
            const uint64_t sz = (key_offsets[i + 1] - key_offsets[i]) + (value_offsets[i + 1] - value_offsets[i]) + 8;
            if (sz > block_size) return fail(PBF_ERR_INVALID, "a record is larger than block_size");
            if (cnt && used + sz > block_size) {  // record i finishes the open block
                const uint64_t bsz = used + 2 * cnt + 2;
                pos += bsz;
                out += bsz;
                block_first[++nb] = i;
                block_out[nb] = out;
                used = 0;
                cnt = 0;
                if (pos >= max_sstable_size) {  // build(): [i] alone is the table's last block
                    out += sz + 4;
                    block_first[++nb] = i + 1;
                    block_out[nb] = out;
                    table_blocks[++nt] = nb;
                    ++i;
                    split = true;
                    break;
                }
            }
            used += sz;
            ++cnt;
        }
        if (!split) {
            if (pos > 0) {  // the open block ends the last table
                out += used + 2 * cnt + 2;
                block_first[++nb] = n;
                block_out[nb] = out;
                table_blocks[++nt] = nb;
            } else {  // records of the last builder's first open block are not written
                nb = nb_table0;
            }
            break;
        }
    }
    *nblocks = nb;
    *ntables = nt;
    *written = block_first[nb];
    return PBF_OK;
}

int pbf_key_range_mask(int device, void* stream, const uint8_t* keys, const uint64_t* offsets, uint32_t key_len,
                       uint64_t n, const uint8_t* bounds, const uint64_t* bound_offsets, uint32_t ntables, uint8_t* out,
                       int on_device) {
    if (n == 0 || ntables == 0) return PBF_OK;
    if (!bound_offsets || !out || (!keys && !offsets)) return fail(PBF_ERR_INVALID, "null pointer");
    HIP_TRY(hipSetDevice(device));
    const uint64_t stride = (n + 7) / 8;
    // table groups whose bounds fit the LDS stage (host-side sizes: the offsets are read on the
    // host for the host path, copied back first for the device path)
    std::vector<uint64_t> bo(2 * size_t(ntables) + 1);
    if (on_device) {
        // ordered after whatever the caller queued on its stream (the offsets may come from it)
        HIP_TRY(hipMemcpyAsync(bo.data(), bound_offsets, bo.size() * 8, hipMemcpyDeviceToHost,
                               static_cast<hipStream_t>(stream)));
        HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    } else
        std::memcpy(bo.data(), bound_offsets, bo.size() * 8);
    std::vector<std::pair<uint32_t, uint32_t>> groups;  // (t0, nt, words)
    std::vector<uint32_t> gwords;
    {
        uint32_t t0 = 0, w = 0;
        for (uint32_t t = 0; t < ntables; ++t) {
            uint32_t tw = 0;
            for (int e = 0; e < 2; ++e) {
                const uint64_t bl = bo[2 * t + e + 1] - bo[2 * t + e];
                if (bl > 64 * 1024) return fail(PBF_ERR_INVALID, "an SSTable bound key is longer than 65536 bytes");
                tw += uint32_t((bl + 3) / 4);
            }
            const uint32_t nt = t - t0 + 1;
            if (t > t0 && (size_t(w + tw) * 4 + size_t(4 * nt + 1) * 4 > kRangeLdsBytes || nt > 4096)) {
                groups.emplace_back(t0, t - t0);
                gwords.push_back(w);
                t0 = t;
                w = 0;
            }
            w += tw;
        }
        groups.emplace_back(t0, ntables - t0);
        gwords.push_back(w);
    }
    EncodeCtx& c = encode_ctx(device);
    std::lock_guard<std::mutex> lock(c.mu);
    if (!c.stream) {
        HIP_TRY(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
        register_stream(device, c.stream);
    }
    hipStream_t s = on_device ? static_cast<hipStream_t>(stream) : c.stream;
    const uint8_t *dk = keys, *db = bounds;
    const uint64_t *dko = offsets, *dbo = bound_offsets;
    uint8_t* dout = out;
    if (!on_device) {
        const uint64_t kb = offsets ? offsets[n] - offsets[0] : n * uint64_t(key_len);
        const uint64_t bb = bo[2 * size_t(ntables)] - bo[0];
        HIP_TRY(c.keys.ensure(kb + 16));
        HIP_TRY(c.vals.ensure(bb + 16));
        HIP_TRY(c.offs.ensure(((offsets ? n + 1 : 0) + bo.size()) * 8));
        HIP_TRY(c.out.ensure(stride * ntables + 16));
        auto* o = static_cast<uint64_t*>(c.offs.p);
        if (kb) HIP_TRY(hipMemcpyAsync(c.keys.p, keys + (offsets ? offsets[0] : 0), kb, hipMemcpyHostToDevice, s));
        if (bb) HIP_TRY(hipMemcpyAsync(c.vals.p, bounds + bo[0], bb, hipMemcpyHostToDevice, s));
        if (offsets) HIP_TRY(hipMemcpyAsync(o, offsets, (n + 1) * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(o + (offsets ? n + 1 : 0), bo.data(), bo.size() * 8, hipMemcpyHostToDevice, s));
        dk = static_cast<const uint8_t*>(c.keys.p);
        db = static_cast<const uint8_t*>(c.vals.p);
        dko = offsets ? o : nullptr;
        dbo = o + (offsets ? n + 1 : 0);
        dout = static_cast<uint8_t*>(c.out.p);
    }
    const Batch b = make_batch(dk, dko, key_len, n);
    const uint32_t grid = grid_for(n, 256, 1024);
    for (size_t gi = 0; gi < groups.size(); ++gi) {
        RangeSet rs{};
        rs.bytes = db;
        rs.offsets = dbo;
        rs.t0 = groups[gi].first;
        rs.nt = groups[gi].second;
        rs.lds_words = gwords[gi];
        const size_t lds = (size_t(4 * rs.nt + 1) + rs.lds_words) * 4;
        if (b.km == kVar) {
            HIP_TRY(allow_lds(k_range_mask<kVar>, lds));
            k_range_mask<kVar><<<grid, 256, lds, s>>>(b.ks, n, rs, dout, stride);
        } else {
            HIP_TRY(allow_lds(k_range_mask<kFixedN>, lds));
            k_range_mask<kFixedN><<<grid, 256, lds, s>>>(b.ks, n, rs, dout, stride);
        }
        CHECK_LAUNCH();
    }
    if (!on_device) {
        HIP_TRY(hipMemcpyAsync(out, dout, stride * ntables, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    return PBF_OK;
}

int pbf_gen_splitmix_hex(int device, void* stream, uint8_t* out_dev, uint64_t seed, uint64_t start, uint64_t n) {
    HIP_TRY(hipSetDevice(device));
    if (n == 0) return PBF_OK;
    if (!out_dev || (reinterpret_cast<uintptr_t>(out_dev) & 15)) return fail(PBF_ERR_INVALID, "out must be 16-B aligned");
    k_gen_splitmix_hex<<<grid_for(n, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(out_dev, seed, start, n);
    CHECK_LAUNCH();
    // the null stream does not order the filters' non-blocking streams: with no stream given the
    // keys are complete on return (a build enqueued next must not read them half-written)
    if (!stream) HIP_TRY(hipStreamSynchronize(nullptr));
    return PBF_OK;
}

int pbf_gen_varlen(int device, void* stream, uint8_t* out_dev, const uint64_t* offsets_dev, uint64_t seed,
                   uint64_t start, uint64_t n) {
    HIP_TRY(hipSetDevice(device));
    if (n == 0) return PBF_OK;
    if (!out_dev || !offsets_dev) return fail(PBF_ERR_INVALID, "null pointer");
    k_gen_varlen<<<grid_for(n, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(out_dev, offsets_dev, seed, start, n);
    CHECK_LAUNCH();
    if (!stream) HIP_TRY(hipStreamSynchronize(nullptr));  // as pbf_gen_splitmix_hex
    return PBF_OK;
}

}  // extern "C"
