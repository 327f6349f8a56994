/*
 * pebblebloom — C-ABI of the MI355X bloom-filter engine (libpebblebloom.so).
 *
 * Drop-in boundary for MaudGautier/pebbledb's per-SSTable filter, src/bloom_filter.py.  The
 * reference has no FFI layer: its boundary is the Python class BloomFilter, whose callers are
 * src/sstable.py:274 (build), :82 (to_bytes), :100 (from_bytes), :146 (__eq__) and
 * src/lsm_storage.py:165,175 (may_contain).  pebbledb_amd/bloom_filter.py keeps that class's
 * surface and binds every entry point below through ctypes.
 *
 * Conventions
 *   - All functions return 0 (PBF_OK) or a negative PBF_ERR_*; pbf_last_error() gives the
 *     message of the last failure on the calling thread.
 *   - Keys are UTF-8 bytes (bloom_filter.py:43).  A batch is either fixed-width (key i =
 *     keys[i*key_len, (i+1)*key_len)) or variable-length (key i = keys[offsets[i] - offsets[0],
 *     offsets[i+1] - offsets[0]); offsets has n+1 entries).
 *   - keys_on_device = 0: keys/offsets/hitmask are host pointers; the call copies what it needs
 *     (pinned staging + hipMemcpyAsync) and returns when the host buffers may be reused.
 *     keys_on_device = 1: they are device pointers on the filter's device; the call is
 *     asynchronous on the filter's stream (pbf_stream) and the caller keeps them alive until
 *     pbf_sync (or an event recorded on that stream) completes.
 *   - A handle is one filter on one device with one HIP stream.  Calls that build, load or
 *     batch-probe take the handle's lock exclusively; one-key probes (pbf_may_contain,
 *     pbf_may_contain_set) of a built filter take it SHARED and run on a per-thread reader
 *     stream, so reader threads probe one filter concurrently (the reference builds a filter
 *     under the flush mutex, lsm_storage.py:220, and then probes it from any reader thread
 *     without a lock, lsm_storage.py:153-179); distinct handles run concurrently.
 *   - Working memory of the tiled pipelines and the host staging path is a per-device pool
 *     shared by all handles (pbf_trim releases it), not per-filter: a long-lived filter holds
 *     only its bitmap.
 */
#ifndef PEBBLEBLOOM_H
#define PEBBLEBLOOM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBF_OK 0
#define PBF_ERR_INVALID (-1)   /* bad argument (null handle or pointer, size mismatch) */
#define PBF_ERR_HIP (-2)       /* a HIP runtime call failed */
#define PBF_ERR_ZERO_SIZE (-3) /* nb_bytes == 0: the reference raises ZeroDivisionError at
                                  `hashed_key % self.bits_size` (bloom_filter.py:47) */

/* Build strategies (pbf_set_build_mode).  All give bit-identical bitmaps. */
#define PBF_BUILD_AUTO 0
#define PBF_BUILD_ATOMIC 1 /* one lane per key, k global atomicOr */
#define PBF_BUILD_TILED 2  /* partition positions by LDS tile, OR in LDS, write tiles once */

/* Probe strategies (pbf_set_probe_mode).  All give identical hit masks. */
#define PBF_PROBE_AUTO 0
#define PBF_PROBE_DIRECT 1 /* one lane per key, k random word loads, wave ballot */
#define PBF_PROBE_TILED 2  /* partition (key, position) entries by LDS tile, test in LDS, gather */

/* What the last probe ran (pbf_last_probe_detail): bit flags | (filters per fused gather << 8)
 * | (tiled pipelines the key batch was split into << 16). */
#define PBF_DETAIL_RING 1    /* tiled: ring partition (k_part_ring) */
#define PBF_DETAIL_SORT 2    /* tiled: counting-sort partition (k_part) */
#define PBF_DETAIL_ONE_KEY 4 /* pbf_may_contain's one-key launch */
#define PBF_DETAIL_SET 8     /* multi-filter direct probe (k_probe_set: each key hashed once for the set) */
#define PBF_DETAIL_PACKED 16 /* tiled build: region entries packed three positions per 8 bytes */
#define PBF_DETAIL_SHARED 32 /* one-key probe under the handle's lock held shared (a reader stream) */
#define PBF_DETAIL_RESIDENT 64 /* one-key probe answered by the resident reader wave (no launch per key) */

typedef struct pbf_filter pbf_filter_t;

/* Library version (major*10000 + minor*100 + patch). */
int pbf_version(void);

/* Number of visible HIP devices. */
int pbf_device_count(int* count);

/* BloomFilter(nb_bytes, nb_hash_functions) — bloom_filter.py:26-31.  The bitmap is
 * 8*nb_bytes bits, all zero.  nb_bytes == 0 → PBF_ERR_ZERO_SIZE (the Python layer keeps such a
 * filter host-side and raises ZeroDivisionError on add/may_contain, like the reference).
 * Any nb_hash_functions is accepted, as in the reference; serialising one above 255 fails in
 * the Python layer exactly where the reference's struct.pack("B", k) does (bloom_filter.py:80). */
int pbf_create(int device, uint64_t nb_bytes, uint32_t nb_hash_functions, pbf_filter_t** out);
int pbf_destroy(pbf_filter_t* f);

/* Reset to the all-zero filter (bits = 0, bloom_filter.py:31). */
int pbf_clear(pbf_filter_t* f);

/* BloomFilter.add for a batch of keys (bloom_filter.py:60-65): ORs k bits per key. */
int pbf_add_fixed(pbf_filter_t* f, const uint8_t* keys, uint32_t key_len, uint64_t n, int keys_on_device);
int pbf_add(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint64_t n, int keys_on_device);
/* The same call under SURVEY.md §8b's name. */
int pbf_build(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint64_t n, int keys_on_device);

/* BloomFilter.may_contain for a batch (bloom_filter.py:67-74).  hitmask receives ceil(n/8)
 * bytes, LSB-first: bit (i & 7) of hitmask[i >> 3] = may_contain(key i).  The hitmask pointer
 * is host or device memory as keys_on_device says. */
int pbf_probe_fixed(pbf_filter_t* f, const uint8_t* keys, uint32_t key_len, uint64_t n, uint8_t* hitmask,
                    int keys_on_device);
int pbf_probe(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint8_t* hitmask,
              int keys_on_device);

/* LsmStorage.get's filter checks for a batch of keys against several SSTable filters
 * (src/lsm_storage.py:164-169 L0 newest-first, :173-175 per level): hitmasks[i] receives
 * may_contain over the batch for filters[i], ceil(n/8) bytes LSB-first, host or device memory as
 * keys_on_device says (hitmasks itself is a host array of nfilters pointers).  Filters must be
 * distinct; with keys_on_device = 1 they must share one device, while a HOST batch over filters
 * on several devices fans out to one host thread per device (pbf_probe_multi_placed, grouped by
 * device).  When they share (nb_bytes, k) and are large (the tiled
 * probe) the keys are hashed and partitioned once for up to 8 filters and only the tile test
 * and gather run per filter.  Otherwise -- SSTable filters of mixed sizes, the usual LSM case
 * (each sized from its own key count, sstable.py:274) -- the filters whose own probe is direct
 * are probed by one kernel per k and 64 filters that hashes every key ONCE and tests every
 * filter from those hashes (MurmurHash3 does not depend on m); large filters of distinct sizes
 * each run their own pipeline on their own stream.  With keys_on_device = 1 the call is
 * asynchronous on filters[0]'s stream (pbf_sync(filters[0])); every other filter's stream is
 * ordered before and after it. */
int pbf_probe_multi_fixed(pbf_filter_t* const* filters, uint32_t nfilters, const uint8_t* keys, uint32_t key_len,
                          uint64_t n, uint8_t* const* hitmasks, int keys_on_device);
int pbf_probe_multi(pbf_filter_t* const* filters, uint32_t nfilters, const uint8_t* keys, const uint64_t* offsets,
                    uint64_t n, uint8_t* const* hitmasks, int keys_on_device);

/* The host-batch multi-probe over a filter set placed on several devices from one process (an
 * LSM's SSTable filters spread one per GPU; LsmStorage.get, src/lsm_storage.py:164-179):
 * group_of[i] names filter i's placement group (filters of one group must share a device; a
 * device may hold several groups).  Each group runs pbf_probe_multi on its own host thread,
 * staging the batch to its device itself (a replicated H2D); hitmasks[i] receives filter i's
 * mask, so the masks come back in the caller's (get) order.  offsets == NULL: fixed key_len.
 * Synchronous. */
int pbf_probe_multi_placed(pbf_filter_t* const* filters, uint32_t nfilters, const uint32_t* group_of,
                           const uint8_t* keys, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                           uint8_t* const* hitmasks);

/* The placement step of pbf_probe_multi_placed (and of a host-batch pbf_probe_multi over
 * filters on several devices, grouped by device), as a pure function that runs without a GPU:
 * slot_of[i] = filter i's group in first-appearance order of group_of (the order the groups'
 * host threads start), *ngroups = the number of groups.  PBF_ERR_INVALID when two filters of
 * one group name different devices (device_of[i] = filter i's device). */
int pbf_plan_groups(const uint32_t* group_of, const int32_t* device_of, uint32_t n, uint32_t* slot_of,
                    uint32_t* ngroups);

/* BloomFilter.may_contain(key) for ONE key (bloom_filter.py:67-74), the per-key call of
 * LsmStorage.get (lsm_storage.py:165,175): key is host memory (UTF-8 bytes, len may be 0),
 * *out = 1 or 0.  Synchronous; the key goes to the kernel through mapped pinned memory and the
 * hit byte comes back the same way (one launch, no copies, no allocation after the first call
 * on a thread). */
int pbf_may_contain(pbf_filter_t* f, const uint8_t* key, uint64_t len, int* out);

/* LsmStorage.get's bloom checks for ONE key over a set of SSTable filters of any sizes
 * (lsm_storage.py:164-179: every L0 filter, then each level filter whose key range holds the
 * key — the range check stays with the caller): out_bits[i >> 3] bit (i & 7) =
 * filters[i].may_contain(key), ceil(nfilters/8) bytes LSB-first.  One launch per k and 64
 * filters (the key hashed once, one lane per filter), the key in and the answer out through
 * mapped pinned memory; synchronous.  All filters on one device (a filter may repeat). */
int pbf_may_contain_set(pbf_filter_t* const* filters, uint32_t nfilters, const uint8_t* key, uint64_t len,
                        uint8_t* out_bits);

/* pbf_may_contain / pbf_may_contain_set on built, idle filters (nothing queued on their streams)
 * are answered by a resident reader: ONE wave per device stays on a stream of its own while keys
 * arrive, polling per-thread request slots in mapped pinned memory (no launch per key); it leaves
 * after PBF_RESIDENT_IDLE_US (default 2000) without a key and is relaunched by the next one.
 * PBF_RESIDENT_READER=0 (read once) launches per key instead.  Keys over 1024 bytes, k > 32 and
 * threads beyond 64 per device take the per-key launch.  *launches = the waves started so far on
 * `device` (0 before the first resident answer). */
int pbf_resident_launches(int device, uint32_t* launches);
/* Requests the device's resident reader has answered so far, and the wave's time on them: from
 * seeing a request in its poll to writing the answer (device wall clock), summed.  The rest of a
 * call's time is the host's and the bus's (posting, the poll's round trip, the answer's write). */
int pbf_resident_stats(int device, uint64_t* requests, uint64_t* device_ns);
/* Turns the resident reader on (1) or off (0) for later calls of the process (overrides
 * PBF_RESIDENT_READER; a wave already resident leaves after its idle time). */
int pbf_resident_enable(int on);

/* mmh3.hash(key, seed) (bloom_filter.py:46: MurmurHash3_x86_32, signed int32) of one host key
 * of at most 4096 bytes, computed on `device` (one launch). */
int pbf_murmur3_x86_32(int device, const uint8_t* key, uint64_t len, uint32_t seed, int32_t* out);

/* The k bit indices of each key, BloomFilter._hash (bloom_filter.py:38-49): out[i*k + s] =
 * mmh3.hash(key_i, s) % bits_size (Python floor-mod).  out is host or device memory as
 * keys_on_device says (n*k uint64).  Used for index-math parity at any m. */
int pbf_hash_indices_fixed(pbf_filter_t* f, const uint8_t* keys, uint32_t key_len, uint64_t n, uint64_t* out,
                           int keys_on_device);
int pbf_hash_indices(pbf_filter_t* f, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint64_t* out,
                     int keys_on_device);

/* to_bytes() minus the trailing k byte (bloom_filter.py:76-81): copies the nb_bytes-byte
 * little-endian bitmap into host memory `out` (nb_bytes must equal the filter's). */
int pbf_get_bitmap(pbf_filter_t* f, uint8_t* out, uint64_t nb_bytes);

/* from_bytes() (bloom_filter.py:83-90): loads an nb_bytes-byte bitmap from host memory. */
int pbf_set_bitmap(pbf_filter_t* f, const uint8_t* in, uint64_t nb_bytes);

/* from_bytes() / to_bytes() against DEVICE memory on the filter's device (nb_bytes bytes, the
 * little-endian bitmap without the k byte), e.g. a tensor an RCCL all-gather filled with other
 * ranks' filters.  Asynchronous on the filter's stream (order a producer on another stream with
 * pbf_wait_stream, a consumer with pbf_signal_stream or pbf_sync). */
int pbf_set_bitmap_device(pbf_filter_t* f, const void* in_dev, uint64_t nb_bytes);
int pbf_get_bitmap_device(pbf_filter_t* f, void* out_dev, uint64_t nb_bytes);

/* A replica of a built filter on dst_device (the same device or another): *out = a new handle
 * with src's nb_bytes, k and bitmap -- what from_bytes(src.to_bytes()) onto that device gives
 * (src/sstable.py:99-100), without the host round trip.  The bitmap goes device to device
 * (hipMemcpyPeerAsync over xGMI, peer access enabled once per device pair where the platform
 * allows it; the runtime stages the copy otherwise), or with flags = PBF_COPY_BOUNCE through
 * pinned host memory.  Synchronous: the replica is complete on return and src may change after.
 * An LSM builds each SSTable's filter once (src/sstable.py:274) and every get probes all of them
 * (src/lsm_storage.py:164-179): the key-partitioned multi-GPU layout holds every filter on every
 * GPU by replication, not by rebuilding. */
#define PBF_COPY_BOUNCE 1
int pbf_copy_filter(pbf_filter_t* src, int dst_device, int flags, pbf_filter_t** out);

/* Population count of the bitmap (device reduction; host-visible result). */
int pbf_popcount(pbf_filter_t* f, uint64_t* out);

/* Wait for all work queued on the filter's stream. */
int pbf_sync(pbf_filter_t* f);

/* The device index map of a filter of nb_bytes (host-side, no GPU): how `hash % bits_size`
 * (Python floor-mod of the signed hash, bloom_filter.py:47) is computed for m = 8*nb_bytes.
 * mode 0: m a power of two <= 2^32, u32(h) & (m-1); 1: m < 2^30, a mod m = a - (mulhi(a, magic)
 * >> shift) * m for a = h >= 0 ? h : ~h; 2: m >= 2^31, h or h + m; 3: 2^30 < m < 2^31, one
 * conditional subtract.  Exposed so the reciprocal can be checked exhaustively on the host. */
int pbf_index_params(uint64_t nb_bytes, uint32_t* mode, uint64_t* magic, uint32_t* shift);

/* Stream ordering for device-pointer calls (keys_on_device = 1) without a device-wide sync:
 * pbf_wait_stream makes the filter's stream wait for everything queued on `stream` so far
 * (e.g. the torch stream that produced a key batch; NULL = the null stream) -- the next
 * add / probe of f runs after that producer; pbf_signal_stream makes `stream` wait for
 * everything queued on the filter's stream so far (a consumer of a device hit mask or bitmap).
 * Both only enqueue an event record + wait; neither blocks the host. */
int pbf_wait_stream(pbf_filter_t* f, void* stream);
int pbf_signal_stream(pbf_filter_t* f, void* stream);

/* The filter's hipStream_t (for events / interop) and its device bitmap (uint32 words). */
void* pbf_stream(pbf_filter_t* f);
void* pbf_device_bitmap(pbf_filter_t* f);

/* Select the build strategy (PBF_BUILD_*); the strategy actually used by the last add is
 * returned by pbf_last_build_mode. */
int pbf_set_build_mode(pbf_filter_t* f, int mode);
int pbf_last_build_mode(pbf_filter_t* f);

/* Select the probe strategy (PBF_PROBE_*); the one used by the last probe is returned by
 * pbf_last_probe_mode, and how it ran by pbf_last_probe_detail (PBF_DETAIL_*). */
int pbf_set_probe_mode(pbf_filter_t* f, int mode);
int pbf_last_probe_mode(pbf_filter_t* f);
uint32_t pbf_last_probe_detail(pbf_filter_t* f);
/* How the last tiled build ran: PBF_DETAIL_RING or _SORT [| _PACKED] | (keys per sub-chunk / 256) << 12. */
uint32_t pbf_last_build_detail(pbf_filter_t* f);

/* Release the device's pooled working memory (waits for its last users); the next call
 * re-allocates what it needs.  pbf_scratch_bytes reports what the pool holds now. */
int pbf_trim(int device);
int pbf_scratch_bytes(int device, uint64_t* out);

/* SSTableBuilder's data section (src/sstable.py:224-268; DataBlock.to_bytes blocks.py:33-37;
 * Record.to_bytes record.py:66-72, key_size = the key's UTF-8 CHARACTER count as the reference's
 * len(str), record.py:24).  Record i = (keys[key_offsets[i], key_offsets[i+1]),
 * values[value_offsets[i], value_offsets[i+1])).  The caller plans the blocks with the
 * DataBlockBuilder rule (blocks.py:78-95; pebbledb_amd/sstable_data.py plan_blocks): block b
 * holds records [block_first[b], block_first[b+1]) (block_first has nblocks+1 entries, 0 .. n)
 * and is written at byte block_out[b] of out (block_out[nblocks] = section size); a block's
 * records may total at most 65536 bytes.  One workgroup per block assembles it in LDS.
 * on_device = 0: all pointers are host memory (checked, staged, section copied back);
 * on_device = 1: device pointers, the offsets start at the data pointers. Synchronous. */
int pbf_encode_data_blocks(int device, const uint8_t* keys, const uint64_t* key_offsets, const uint8_t* values,
                           const uint64_t* value_offsets, uint64_t n, const uint64_t* block_first,
                           const uint64_t* block_out, uint64_t nblocks, uint8_t* out, int on_device);

/* SSTableBuilder.add x n + build (src/sstable.py:224-288) in one call, for the flush of a
 * packed run of records (host memory; offsets start at 0): one H2D of the keys, values and
 * block plan (as for pbf_encode_data_blocks), the data blocks encoded on the device, the filter
 * f (sized by the caller with the reference's build_from_keys_and_fp_rate expression, fp 0.001)
 * built from the SAME device copy of the keys, and D2H of the data section into data_out
 * (block_out[nblocks] bytes) and of the bitmap into bitmap_out (f's nb_bytes, may be NULL) —
 * the caller points both at their slices of the SSTable file buffer.  Synchronous. */
int pbf_build_sstable(pbf_filter_t* f, const uint8_t* keys, const uint64_t* key_offsets, const uint8_t* values,
                      const uint64_t* value_offsets, uint64_t n, const uint64_t* block_first, const uint64_t* block_out,
                      uint64_t nblocks, uint8_t* data_out, uint8_t* bitmap_out);

/* Compaction's output SSTables (LsmStorage._compact, src/lsm_storage.py:233-251: a new
 * SSTableBuilder once current_buffer_position >= max_sstable_size) from ONE upload of the
 * compacted record run (host memory, offsets start at 0; n records).  The caller plans the split
 * on the host (pebbledb_amd/sstable_data.plan_compaction): blocks as for pbf_build_sstable but over
 * the whole run, block_out laid end to end over the outputs' data sections, output t = blocks
 * [table_blocks[t], table_blocks[t+1]) (table_blocks has ntables+1 entries, 0 .. nblocks; the
 * plan may end before record n: the reference does not write records left in its last builder's
 * first open block).  filters[t] is output t's filter (sized by the caller from its key count
 * with build_from_keys_and_fp_rate's expression, fp 0.001, sstable.py:274), built from its slice
 * of the SAME device copy of the keys on its own stream; data_outs[t] / bitmap_outs[t]
 * (bitmap_outs or an entry may be NULL) receive the output's data section and bitmap, the
 * caller's slices of each SSTable file buffer.  Synchronous. */
int pbf_build_sstables(pbf_filter_t* const* filters, uint32_t ntables, const uint8_t* keys, const uint64_t* key_offsets,
                       const uint8_t* values, const uint64_t* value_offsets, uint64_t n, const uint64_t* block_first,
                       const uint64_t* block_out, uint64_t nblocks, const uint64_t* table_blocks,
                       uint8_t* const* data_outs, uint8_t* const* bitmap_outs);

/* DataBlockBuilder's greedy blocks (src/blocks.py:78-95, sstable.py:224-244) over n records
 * whose key / value bytes are given by their offsets: block_first[0..nblocks] record indices,
 * block_out[0..nblocks] byte offsets of the encoded blocks (both sized n+1 by the caller);
 * *nblocks receives the count.  Host-side planning for pbf_build_sstable. */
int pbf_plan_blocks(const uint64_t* key_offsets, const uint64_t* value_offsets, uint64_t n, uint64_t block_size,
                    uint64_t* block_first, uint64_t* block_out, uint64_t* nblocks);

/* Compaction's output split (LsmStorage._compact, src/lsm_storage.py:233-251) over n records,
 * host-side: the greedy blocks of pbf_plan_blocks over the whole run, a new table whenever the
 * builder's position (advanced per finished block, src/sstable.py:246-266) reaches
 * max_sstable_size (the table's last block then holds only the record that finished the previous
 * one), the last builder kept only if its position is past 0.  Outputs for pbf_build_sstables:
 * block_first / block_out (n+1 entries each; block_out laid end to end over the tables' data
 * sections), table_blocks (n+1 entries; table t = blocks [table_blocks[t], table_blocks[t+1])),
 * the counts, and the records covered (*written <= n).  max_sstable_size 0 is refused
 * (PBF_ERR_INVALID). */
int pbf_plan_compaction(const uint64_t* key_offsets, const uint64_t* value_offsets, uint64_t n, uint64_t block_size,
                        uint64_t max_sstable_size, uint64_t* block_first, uint64_t* block_out, uint64_t* table_blocks,
                        uint64_t* nblocks, uint64_t* ntables, uint64_t* written);

/* The level key-range pre-check of LsmStorage.get (src/lsm_storage.py:171-175) for a batch:
 * out[t * ceil(n/8) + i/8] bit (i & 7) = (first_t <= key_i <= last_t), Python str order =
 * bytewise lexicographic order of the UTF-8 keys.  Bounds are 2*ntables byte strings
 * (first_0, last_0, first_1, last_1, ...): bound j = bounds[bound_offsets[j] - bound_offsets[0],
 * bound_offsets[j+1] - bound_offsets[0]).  Keys as in pbf_probe (offsets != NULL) or fixed
 * key_len (offsets == NULL).  The mask layout is the hit-mask layout, so it ANDs directly with
 * the table's filter hit mask.  on_device = 0: host pointers, synchronous; on_device = 1:
 * device pointers (bound_offsets is read back first), asynchronous on `stream`. */
int pbf_key_range_mask(int device, void* stream, const uint8_t* keys, const uint64_t* offsets, uint32_t key_len,
                       uint64_t n, const uint8_t* bounds, const uint64_t* bound_offsets, uint32_t ntables, uint8_t* out,
                       int on_device);

/* Synthetic keys straight into device memory (bench / tests; definitions in
 * pebbledb_amd/keys.py): 16 hex chars of splitmix64(seed + start + i), and the variable-length
 * 8..64-byte family (offsets must already hold the n+1 offsets, relative to offsets[0]).
 * stream = NULL: the keys are complete on return (filters run on non-blocking streams, which the
 * null stream does not order); otherwise asynchronous on `stream`. */
int pbf_gen_splitmix_hex(int device, void* stream, uint8_t* out_dev, uint64_t seed, uint64_t start, uint64_t n);
int pbf_gen_varlen(int device, void* stream, uint8_t* out_dev, const uint64_t* offsets_dev, uint64_t seed,
                   uint64_t start, uint64_t n);

/* Message of the last failure on this thread ("" if none). */
const char* pbf_last_error(void);

/* sha256 (hex) of the kernel sources the library was compiled from (pebbledb_amd/build.py
 * source_digest()); the Python binding refuses a library whose digest is not the tree's. */
const char* pbf_source_digest(void);

#ifdef __cplusplus
}
#endif
#endif /* PEBBLEBLOOM_H */
