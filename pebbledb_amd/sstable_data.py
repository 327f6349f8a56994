"""SSTable build on the device: data blocks (``pbf_encode_data_blocks``), meta blocks and the
bloom filter — the byte-identical counterpart of the reference's ``SSTableBuilder``
(src/sstable.py:209-288) for a flushed / compacted run of records.

Host side (this module): pack the records into the boundary layout (key bytes + u64 offsets,
value bytes + u64 offsets), plan the data blocks with the reference's greedy rule
(``DataBlockBuilder.add``, blocks.py:78-95: a record joins the block iff the block's record
bytes stay <= block_size; offsets and count are not counted), and encode the meta blocks
(blocks.py:126-133, a few bytes per 64 KiB block).  Device side: every data block is
assembled in LDS by one workgroup and written once (csrc/sstable_kernels.hpp); the bloom
filter of all keys (fp_rate 0.001, sstable.py:274) is built by the bloom kernels and its
bitmap copied from HBM straight into the file buffer (sstable_bloom.encode_sstable).

Reference quirks kept: Record.key_size and MetaBlock key sizes are ``len(str)`` — characters,
not UTF-8 bytes (record.py:24, blocks.py:127,129).  Divergences (inputs the reference
mishandles): a record larger than block_size raises ValueError (the reference drops it from
the data silently, blocks.py:84-85, while keeping its key in the bloom filter); an empty
record list raises ValueError (the reference fails in MetaBlock.to_bytes); block_size must be
<= 65536 (the reference's u16 offsets, blocks.py:34, overflow beyond).
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np

from . import _native
from .keys import PackedKeys, PackedRecords

BLOCK_SIZE = 65_536  # SSTableBuilder default (sstable.py:215)
RECORD_HEADER = 8    # two i32 sizes (record.py:66-72)


def pack_values(values) -> tuple[np.ndarray, np.ndarray]:
    """(bytes, u64 offsets[n+1]) of a list of bytes values."""
    vals = values if isinstance(values, list) else list(values)
    lens = np.fromiter(map(len, vals), dtype=np.int64, count=len(vals))
    offs = np.zeros(len(vals) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    return np.frombuffer(b"".join(vals), dtype=np.uint8), offs


def key_offsets(pk: PackedKeys) -> np.ndarray:
    if pk.offsets is not None:
        return pk.offsets
    if pk._ko is not None:
        return pk._ko
    return np.arange(0, (pk.n + 1) * pk.key_len, max(pk.key_len, 1), dtype=np.uint64)[:pk.n + 1] \
        if pk.key_len else np.zeros(pk.n + 1, dtype=np.uint64)


def plan_blocks(ko: np.ndarray, vo: np.ndarray, block_size: int = BLOCK_SIZE) -> tuple[np.ndarray, np.ndarray]:
    """DataBlockBuilder's greedy blocks (blocks.py:78-95, sstable.py:224-244): (block_first
    [nblocks+1] record indices, block_out [nblocks+1] byte offsets of the encoded blocks)."""
    n = len(ko) - 1
    if n <= 0:
        raise ValueError("an SSTable needs at least one record (the reference fails in MetaBlock.to_bytes)")
    if not 0 < block_size <= 65_536:
        raise ValueError("block_size must be in (0, 65536]: DataBlock offsets are u16 (blocks.py:34)")
    sizes = (np.diff(ko.astype(np.int64)) + np.diff(vo.astype(np.int64)) + RECORD_HEADER)
    if int(sizes.max()) > block_size:
        raise ValueError("a record is larger than block_size (the reference would drop it, blocks.py:84-85)")
    P = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(sizes, out=P[1:])
    first = [0]
    s = 0
    while s < n:
        # the largest e with P[e] - P[s] <= block_size: records s..e-1 fill the block
        e = int(np.searchsorted(P, P[s] + block_size, side="right")) - 1
        first.append(e)
        s = e
    bf = np.asarray(first, dtype=np.uint64)
    cnt = np.diff(bf.astype(np.int64))
    data_len = P[bf[1:].astype(np.int64)] - P[bf[:-1].astype(np.int64)]
    bo = np.zeros(len(bf), dtype=np.uint64)
    np.cumsum(data_len + 2 * cnt + 2, out=bo[1:])
    return bf, bo


def plan_blocks_native(ko: np.ndarray, vo: np.ndarray, block_size: int = BLOCK_SIZE) -> tuple[np.ndarray, np.ndarray]:
    """plan_blocks by the C planner (pbf_plan_blocks: one pass over the record sizes)."""
    n = len(ko) - 1
    if n <= 0:
        raise ValueError("an SSTable needs at least one record (the reference fails in MetaBlock.to_bytes)")
    if not 0 < block_size <= 65_536:
        raise ValueError("block_size must be in (0, 65536]: DataBlock offsets are u16 (blocks.py:34)")
    ko = np.ascontiguousarray(ko, dtype=np.uint64)
    vo = np.ascontiguousarray(vo, dtype=np.uint64)
    bf = np.empty(n + 1, dtype=np.uint64)
    bo = np.empty(n + 1, dtype=np.uint64)
    nb = ctypes.c_uint64(0)
    vp = ctypes.c_void_p
    rc = _native.lib().pbf_plan_blocks(vp(ko.ctypes.data), vp(vo.ctypes.data), n, block_size, vp(bf.ctypes.data),
                                       vp(bo.ctypes.data), ctypes.byref(nb))
    if rc == _native.PBF_ERR_INVALID and "larger than block_size" in _native.lib().pbf_last_error().decode():
        raise ValueError("a record is larger than block_size (the reference would drop it, blocks.py:84-85)")
    _native.check(rc, "pbf_plan_blocks")
    return bf[:nb.value + 1].copy(), bo[:nb.value + 1].copy()


def _check_max_sstable_size(max_sstable_size: int) -> None:
    """A split size of 0 or less is refused.  (The reference checks the position after every
    add, lsm_storage.py:241, so there it would build one SSTable per record; the planners here
    split where a block finishes, which agrees with it for every positive size.)"""
    if max_sstable_size <= 0:
        raise ValueError("max_sstable_size must be positive")


def plan_compaction(ko: np.ndarray, vo: np.ndarray, block_size: int = BLOCK_SIZE,
                    max_sstable_size: int = 262_144_000):
    """Compaction's output split (``LsmStorage._compact``, src/lsm_storage.py:233-251) over a
    record run, on the host block plan.  A builder's position advances only when a data block
    finishes — when a record does not fit the open block (src/sstable.py:224-268) — and the
    builder is built as soon as that position reaches max_sstable_size: its last block then holds
    only the record that finished the previous one.  At the end of the run the last builder is
    built only if its position is past 0, so records still in its first open block are not
    written (the reference's behaviour).

    Returns (block_first, block_out, table_blocks, written): blocks as plan_blocks gives them but
    over the whole run (block_out = offsets in the outputs' data sections laid end to end),
    table t = blocks [table_blocks[t], table_blocks[t+1]), records [block_first[table_blocks[t]],
    block_first[table_blocks[t+1]]); `written` = records covered by the outputs."""
    n = len(ko) - 1
    if not 0 < block_size <= 65_536:
        raise ValueError("block_size must be in (0, 65536]: DataBlock offsets are u16 (blocks.py:34)")
    _check_max_sstable_size(max_sstable_size)
    if n <= 0:
        return (np.zeros(1, np.uint64), np.zeros(1, np.uint64), np.zeros(1, np.uint64), 0)
    sizes = (np.diff(ko.astype(np.int64)) + np.diff(vo.astype(np.int64)) + RECORD_HEADER)
    if int(sizes.max()) > block_size:
        raise ValueError("a record is larger than block_size (the reference would drop it, blocks.py:84-85)")
    P = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(sizes, out=P[1:])
    first, tables = [0], [0]  # block starts (record index); table starts (block index)
    s = 0
    while s < n:
        pos = 0  # the builder's current_buffer_position
        split = False
        while True:
            e = int(np.searchsorted(P, P[s] + block_size, side="right")) - 1  # block [s, e)
            if e >= n:
                break  # the open block: no record arrives to finish it
            pos += int(P[e] - P[s]) + 2 * (e - s) + 2
            first.append(e)
            if pos >= max_sstable_size:  # build(): finish_block() of [e] alone
                first.append(e + 1)
                tables.append(len(first) - 1)
                s = e + 1
                split = True
                break
            s = e
        if not split:
            if pos > 0:  # build() at the end: the open block [s, n) is the last one
                first.append(n)
                tables.append(len(first) - 1)
            else:  # _compact's `if current_buffer_position > 0`: [t0, n) is not written
                first = first[:tables[-1] + 1]
            break
    bf = np.asarray(first, dtype=np.uint64)
    b64 = bf.astype(np.int64)
    cnt = np.diff(b64)
    bo = np.zeros(len(bf), dtype=np.uint64)
    np.cumsum((P[b64[1:]] - P[b64[:-1]]) + 2 * cnt + 2, out=bo[1:])
    tb = np.asarray(tables, dtype=np.uint64)
    return bf, bo, tb, int(bf[-1])


def plan_compaction_native(ko: np.ndarray, vo: np.ndarray, block_size: int = BLOCK_SIZE,
                           max_sstable_size: int = 262_144_000):
    """plan_compaction by the C planner (pbf_plan_compaction: one pass over the record sizes)."""
    n = len(ko) - 1
    if not 0 < block_size <= 65_536:
        raise ValueError("block_size must be in (0, 65536]: DataBlock offsets are u16 (blocks.py:34)")
    _check_max_sstable_size(max_sstable_size)
    if n <= 0:
        return (np.zeros(1, np.uint64), np.zeros(1, np.uint64), np.zeros(1, np.uint64), 0)
    ko = np.ascontiguousarray(ko, dtype=np.uint64)
    vo = np.ascontiguousarray(vo, dtype=np.uint64)
    bf = np.empty(n + 1, dtype=np.uint64)
    bo = np.empty(n + 1, dtype=np.uint64)
    tb = np.empty(n + 1, dtype=np.uint64)
    nb, nt, w = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    vp = ctypes.c_void_p
    rc = _native.lib().pbf_plan_compaction(vp(ko.ctypes.data), vp(vo.ctypes.data), n, block_size, max_sstable_size,
                                           vp(bf.ctypes.data), vp(bo.ctypes.data), vp(tb.ctypes.data), ctypes.byref(nb),
                                           ctypes.byref(nt), ctypes.byref(w))
    if rc == _native.PBF_ERR_INVALID and "larger than block_size" in _native.lib().pbf_last_error().decode():
        raise ValueError("a record is larger than block_size (the reference would drop it, blocks.py:84-85)")
    _native.check(rc, "pbf_plan_compaction")
    return bf[:nb.value + 1].copy(), bo[:nb.value + 1].copy(), tb[:nt.value + 1].copy(), int(w.value)


def encode_data_blocks(pk: PackedKeys, vals: np.ndarray, vo: np.ndarray, block_first: np.ndarray,
                       block_out: np.ndarray, device: int = 0) -> np.ndarray:
    """The data section (every encoded DataBlock back to back), written by the device."""
    ko = np.ascontiguousarray(key_offsets(pk), dtype=np.uint64)
    vo = np.ascontiguousarray(vo, dtype=np.uint64)
    bf = np.ascontiguousarray(block_first, dtype=np.uint64)
    bo = np.ascontiguousarray(block_out, dtype=np.uint64)
    out = np.empty(int(bo[-1]), dtype=np.uint8)
    keys = pk.data if pk.data.size else np.zeros(1, np.uint8)
    vals = vals if vals.size else np.zeros(1, np.uint8)
    vp = ctypes.c_void_p
    rc = _native.lib().pbf_encode_data_blocks(device, vp(keys.ctypes.data), vp(ko.ctypes.data), vp(vals.ctypes.data),
                                              vp(vo.ctypes.data), pk.n, vp(bf.ctypes.data), vp(bo.ctypes.data),
                                              len(bf) - 1, vp(out.ctypes.data), 0)
    _native.check(rc, "pbf_encode_data_blocks")
    return out


def meta_blocks(keys, block_first: np.ndarray, block_out: np.ndarray) -> tuple[bytes, list]:
    """MetaBlock.to_bytes of every block (blocks.py:126-133) and the (first, last, offset) list.
    `keys`: list[str] or PackedKeys (only the blocks' first / last keys are decoded)."""
    key = (lambda i: keys.key(i).decode("utf-8")) if isinstance(keys, PackedKeys) else keys.__getitem__
    parts, metas = [], []
    for b in range(len(block_first) - 1):
        first, last = key(int(block_first[b])), key(int(block_first[b + 1]) - 1)
        off = int(block_out[b])
        metas.append((first, last, off))
        parts.append(struct.pack("H", len(first)) + first.encode("utf-8") + struct.pack("H", len(last)) +
                     last.encode("utf-8") + struct.pack("i", off))
    return b"".join(parts), metas


def build_sstable(keys, values=None, block_size: int = BLOCK_SIZE, fp_rate: float = 0.001, device=None):
    """The bytes SSTableBuilder(block_size=block_size) writes after add(k, v) for every record
    and build() (sstable.py:270-288), plus the meta blocks and the device BloomFilter.

    `keys` is either a PackedRecords (values None) — e.g. ``PackedRecords.from_encoded(
    iter(memtable.map))``, the flush path with no per-record Python — or list[str] with
    `values` list[bytes].  Returns (file bytes as a uint8 numpy array, meta blocks, filter).
    The device work is ONE call (``pbf_build_sstable``): the records go
    to the GPU once, the data blocks and the filter (build_from_keys_and_fp_rate's sizing,
    bloom_filter.py:109-114, fp 0.001 as sstable.py:274) are both built from that copy, and the
    data section and the bitmap are copied straight into their slices of the file buffer."""
    from math import ceil, log

    from .bloom_filter import BloomFilter, _default_device
    from .sstable_bloom import TRAILER, sstable_size

    dev = _default_device if device is None else int(device)
    if isinstance(keys, PackedRecords):
        if values is not None:
            raise ValueError("PackedRecords carries its values")
        pk, vals, vo = keys.keys, keys.values, keys.value_offsets
    else:
        keys = keys if isinstance(keys, list) else list(keys)
        pk = PackedKeys.from_strs(keys)
        vals, vo = pack_values(values)
    if len(vo) - 1 != pk.n:
        raise ValueError("keys and values differ in length")
    ko = np.ascontiguousarray(key_offsets(pk), dtype=np.uint64)
    vo = np.ascontiguousarray(vo, dtype=np.uint64)
    bf_first, bo = plan_blocks_native(ko, vo, block_size)
    meta, metas = meta_blocks(keys if isinstance(keys, list) else pk, bf_first, bo)
    n = pk.n
    m = (-n * log(fp_rate)) / (log(2) ** 2)  # bloom_filter.py:109-114, same expression order
    nb_bytes, k = ceil(m / 8), round((m / n) * log(2))
    if not 0 <= k <= 255:
        raise struct.error("ubyte format requires 0 <= number <= 255")  # SSTableEncoding -> to_bytes
    bloom = BloomFilter(nb_bytes, k, device=dev)
    data_len = int(bo[-1])
    if data_len + len(meta) > 0x7FFFFFFF:
        raise struct.error("'i' format requires -2147483648 <= number <= 2147483647")
    # the file buffer: every byte is written below (data and bitmap by the device, the rest
    # here), so it is not zero-filled first (a 76 MB bytearray's fill alone cost 14 ms)
    out = np.empty(sstable_size(data_len, len(meta), nb_bytes), dtype=np.uint8)
    buf = out
    bloom_off = data_len + len(meta)
    kbytes = pk.data if pk.data.size else np.zeros(1, np.uint8)
    vbytes = vals if vals.size else np.zeros(1, np.uint8)
    vp = ctypes.c_void_p
    rc = _native.lib().pbf_build_sstable(bloom.handle, vp(kbytes.ctypes.data), vp(ko.ctypes.data),
                                         vp(vbytes.ctypes.data), vp(vo.ctypes.data), n, vp(bf_first.ctypes.data),
                                         vp(bo.ctypes.data), len(bf_first) - 1, vp(buf.ctypes.data),
                                         vp(buf.ctypes.data + bloom_off))
    _native.check(rc, "pbf_build_sstable")
    out[data_len:bloom_off] = np.frombuffer(meta, dtype=np.uint8)
    out[bloom_off + nb_bytes] = k
    out[len(out) - TRAILER:] = np.frombuffer(struct.pack("ii", data_len, bloom_off), dtype=np.uint8)
    return out, metas, bloom


def build_sstables(keys, values=None, max_sstable_size: int = 262_144_000, block_size: int = BLOCK_SIZE,
                   fp_rate: float = 0.001, device=None):
    """Compaction's output SSTables (``LsmStorage._compact``, src/lsm_storage.py:233-251) for a
    merged record run: the split of plan_compaction, then every output's data blocks and bloom
    filter from ONE upload of the run (``pbf_build_sstables``).  `keys` / `values` as for
    build_sstable (a PackedRecords, or list[str] + list[bytes]).  Returns (outputs, written):
    outputs = [(file bytes as a uint8 numpy array, meta blocks, filter), ...] in the order
    _compact returns them, written = records covered (the reference leaves out records still in
    its last builder's first open block)."""
    from math import ceil, log

    from .bloom_filter import BloomFilter, _default_device
    from .sstable_bloom import TRAILER, sstable_size

    dev = _default_device if device is None else int(device)
    if isinstance(keys, PackedRecords):
        if values is not None:
            raise ValueError("PackedRecords carries its values")
        pk, vals, vo = keys.keys, keys.values, keys.value_offsets
    else:
        keys = keys if isinstance(keys, list) else list(keys)
        pk = PackedKeys.from_strs(keys)
        vals, vo = pack_values(values)
    if len(vo) - 1 != pk.n:
        raise ValueError("keys and values differ in length")
    ko = np.ascontiguousarray(key_offsets(pk), dtype=np.uint64)
    vo = np.ascontiguousarray(vo, dtype=np.uint64)
    bf, bo, tb, written = plan_compaction_native(ko, vo, block_size, max_sstable_size)
    nt = len(tb) - 1
    if nt == 0:
        return [], written
    key_src = keys if isinstance(keys, list) else pk
    files, metas_all, filters, datas, bitmaps, tails = [], [], [], [], [], []
    for t in range(nt):
        b0, b1 = int(tb[t]), int(tb[t + 1])
        n = int(bf[b1] - bf[b0])
        m = (-n * log(fp_rate)) / (log(2) ** 2)  # bloom_filter.py:109-114, same expression order
        nb_bytes, k = ceil(m / 8), round((m / n) * log(2))
        if not 0 <= k <= 255:
            raise struct.error("ubyte format requires 0 <= number <= 255")
        base = int(bo[b0])
        meta, metas = meta_blocks(key_src, bf[b0:b1 + 1], bo[b0:b1 + 1] - np.uint64(base))
        data_len = int(bo[b1]) - base
        if data_len + len(meta) > 0x7FFFFFFF:
            raise struct.error("'i' format requires -2147483648 <= number <= 2147483647")
        out = np.empty(sstable_size(data_len, len(meta), nb_bytes), dtype=np.uint8)
        bloom_off = data_len + len(meta)
        filters.append(BloomFilter(nb_bytes, k, device=dev))
        files.append(out)
        metas_all.append(metas)
        datas.append(out.ctypes.data)
        bitmaps.append(out.ctypes.data + bloom_off)
        tails.append((data_len, meta, bloom_off, nb_bytes, k))
    vp = ctypes.c_void_p
    hs = (vp * nt)(*[f.handle.value for f in filters])
    douts = (vp * nt)(*datas)
    bouts = (vp * nt)(*bitmaps)
    kbytes = pk.data if pk.data.size else np.zeros(1, np.uint8)
    vbytes = vals if vals.size else np.zeros(1, np.uint8)
    bf_c = np.ascontiguousarray(bf, dtype=np.uint64)
    bo_c = np.ascontiguousarray(bo, dtype=np.uint64)
    tb_c = np.ascontiguousarray(tb, dtype=np.uint64)
    rc = _native.lib().pbf_build_sstables(hs, nt, vp(kbytes.ctypes.data), vp(ko.ctypes.data), vp(vbytes.ctypes.data),
                                          vp(vo.ctypes.data), pk.n, vp(bf_c.ctypes.data), vp(bo_c.ctypes.data),
                                          len(bf_c) - 1, vp(tb_c.ctypes.data), douts, bouts)
    _native.check(rc, "pbf_build_sstables")
    for out, (data_len, meta, bloom_off, nb_bytes, k) in zip(files, tails):
        out[data_len:bloom_off] = np.frombuffer(meta, dtype=np.uint8)
        out[bloom_off + nb_bytes] = k
        out[len(out) - TRAILER:] = np.frombuffer(struct.pack("ii", data_len, bloom_off), dtype=np.uint8)
    return list(zip(files, metas_all, filters)), written
