"""The filter stage of ``LsmStorage.get`` over a batch of keys (reference
src/lsm_storage.py:153-179).

For one key the reference walks the SSTables in a fixed order and reads (``SSTable.get``) the
first ones its checks let through:

* L0, newest first (``sstables_level0``): ``bloom_filter.may_contain(key)`` (:164-169);
* every level L>=1, each SSTable in list order: ``first_key <= key <= last_key`` (:173),
  then ``may_contain(key)`` (:175).

``candidate_masks`` computes both checks for a whole batch on the device: the L0 filters and
the range-qualified level filters are probed with ``may_contain_multi`` (one shared pipeline
per SSTable size class), and the level key-range check is ``pbf_key_range_mask`` (bytewise
compare of the UTF-8 keys = Python ``str`` order).  The result is one LSB-first mask per
SSTable, numbered L0 first then level by level (``shard.candidate_order``'s numbering), whose
set bits are exactly the (key, SSTable) pairs the reference would go on to read, in the
reference's order (``candidate_lists``).  A level SSTable whose range holds no key of the batch
is never probed, as the reference never probes it.

``candidates_one`` is the per-key form (one ``get``): the range checks are Python's own ``str``
comparison on the host, and every L0 filter plus every in-range level filter is tested in ONE
launch (``pbf_may_contain_set``), whatever the filters' sizes — instead of one ``may_contain``
launch per SSTable.
"""
from __future__ import annotations

import ctypes
from typing import NamedTuple, Sequence

import numpy as np

from . import _native
from . import bloom_filter as _bfm
from .bloom_filter import BloomFilter, _default_device, may_contain_multi, may_contain_set_bits
from .keys import PackedKeys


class LevelTable(NamedTuple):
    """An L>=1 SSTable as LsmStorage.get sees it (sstable.first_key / last_key / bloom_filter)."""
    first_key: str
    last_key: str
    bloom_filter: BloomFilter


def _pack(keys) -> PackedKeys:
    return keys if isinstance(keys, PackedKeys) else PackedKeys.from_strs(list(keys))


def key_range_masks(keys, bounds: Sequence[tuple[str, str]], device: int | None = None) -> np.ndarray:
    """uint8 [len(bounds), ceil(n/8)]: bit i of row t = ``first_t <= key_i <= last_t``
    (lsm_storage.py:173), computed by ``pbf_key_range_mask`` on the device."""
    pk = _pack(keys)
    nb = (pk.n + 7) // 8
    out = np.zeros((len(bounds), nb), dtype=np.uint8)
    if pk.n == 0 or not bounds:
        return out
    enc = [s.encode("utf-8") for pair in bounds for s in pair]
    lens = np.fromiter(map(len, enc), dtype=np.int64, count=len(enc))
    boffs = np.zeros(len(enc) + 1, dtype=np.uint64)
    np.cumsum(lens, out=boffs[1:])
    bbytes = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
    keys_arr = pk.data if pk.data.size else np.zeros(1, np.uint8)
    vp = ctypes.c_void_p
    dev = _default_device if device is None else int(device)
    rc = _native.lib().pbf_key_range_mask(dev, None, vp(keys_arr.ctypes.data),
                                          None if pk.offsets is None else vp(pk.offsets.ctypes.data), pk.key_len,
                                          pk.n, vp(bbytes.ctypes.data), vp(boffs.ctypes.data), len(bounds),
                                          vp(out.ctypes.data), 0)
    _native.check(rc, "pbf_key_range_mask")
    return out


def candidate_masks(keys, level0: Sequence[BloomFilter], levels: Sequence[Sequence[LevelTable]]) -> np.ndarray:
    """uint8 [T, ceil(n/8)], T = len(level0) + sum(len(level)): row t's bit i is set iff
    LsmStorage.get(key_i) would read SSTable t if no earlier SSTable held the key
    (lsm_storage.py:164-179).  Rows: L0 in the given (newest-first) order, then each level's
    SSTables in list order."""
    pk = _pack(keys)
    nb = (pk.n + 7) // 8
    flat = [t for lvl in levels for t in lvl]
    out = np.zeros((len(level0) + len(flat), nb), dtype=np.uint8)
    if pk.n == 0:
        return out
    if level0:
        out[:len(level0)] = may_contain_multi(level0, pk)
    if flat:
        rng = key_range_masks(pk, [(t.first_key, t.last_key) for t in flat],
                              device=flat[0].bloom_filter.device)
        live = [j for j in range(len(flat)) if rng[j].any()]  # tables no key of the batch reaches
        if live:
            hits = may_contain_multi([flat[j].bloom_filter for j in live], pk)
            for r, j in enumerate(live):
                out[len(level0) + j] = rng[j] & hits[r]
    return out


def candidate_lists(masks: np.ndarray, n: int) -> list[list[int]]:
    """Per key, the SSTable rows of ``candidate_masks`` in the reference's read order."""
    bits = np.unpackbits(masks, axis=1, bitorder="little")[:, :n].astype(bool)
    return [[int(t) for t in np.flatnonzero(bits[:, i])] for i in range(n)]


def candidates_one(key: str, level0: Sequence[BloomFilter], levels: Sequence[Sequence[LevelTable]]) -> list[int]:
    """The SSTables ``LsmStorage.get(key)`` would read if none held the key, in its order
    (lsm_storage.py:164-179), numbered as ``candidate_masks`` rows: L0 filters (newest first)
    and the level filters whose ``first_key <= key <= last_key`` (:173) are tested together in
    one ``pbf_may_contain_set`` launch.  The whole stage runs in C (``_pebblefast.candidates_one``:
    the range checks, the handles and the call, ~3 us less per get than this loop); it hands back
    None when this path must take the call (buffered adds, a non-str key, filters on several
    devices, more than 64 filters), which then raises what the reference raises."""
    r = (_bfm._FAST or _bfm._fast()).candidates_one(key, level0, levels)
    if r is not None:
        return r
    n0 = len(level0)
    in_range, tested = [], list(level0)
    j = n0
    for lvl in levels:
        for t in lvl:
            if t.first_key <= key <= t.last_key:
                in_range.append(j)
                tested.append(t.bloom_filter)
            j += 1
    if not tested:
        return []
    bits = may_contain_set_bits(tested, key)
    out = list(_set_bits(bits & ((1 << n0) - 1)))
    if in_range:
        out += [in_range[r] for r in _set_bits(bits >> n0)]
    return out


_SET_BITS: dict = {}


def _set_bits(b: int) -> tuple:
    """The indices of b's set bits, ascending (memoised: a get's hit pattern over its L0 and
    in-range tables repeats)."""
    r = _SET_BITS.get(b)
    if r is None:
        r = tuple(i for i in range(b.bit_length()) if b >> i & 1)
        if len(_SET_BITS) < 1 << 16:
            _SET_BITS[b] = r
    return r
