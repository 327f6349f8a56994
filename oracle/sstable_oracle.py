"""ORACLE — test infrastructure only (never imported by the product package ``pebbledb_amd``).

A plain-Python restatement of the reference's SSTable build (src/sstable.py:209-288), the
checker for the device data-block encoder (pebbledb_amd/sstable_data.py,
``pbf_encode_data_blocks``).  Pinned to the real reference by tests/golden/sstable_build.json
(tools/gen_golden_sstable.py) in tests/test_sstable_data_cpu.py.

Semantics kept exactly, including the reference's quirks:
* Record (record.py:51-72): i32 key_size ‖ key UTF-8 ‖ i32 value_size ‖ value, where key_size
  is ``len(key)`` — the CHARACTER count (record.py:24), not the byte count, for non-ASCII keys.
* DataBlockBuilder.add (blocks.py:78-95): a record joins the block iff data_length + its size
  <= block_size (the u16 offsets and the count are not counted).
* DataBlock.to_bytes (blocks.py:33-37): records ‖ u16 offset per record ‖ u16 count.
* MetaBlock.to_bytes (blocks.py:126-133): u16 len(first_key) (characters) ‖ first key ‖ u16
  len(last_key) ‖ last key ‖ i32 block offset.
* SSTableBuilder.build (sstable.py:270-288): the bloom filter of every added key with
  fp_rate 0.001 (bloom_filter.py:92-119), SSTableEncoding.to_bytes (sstable.py:80-86).
"""
from __future__ import annotations

import struct

import numpy as np


def record_bytes(key: str, value: bytes) -> bytes:
    """record.py:66-72 (key_size = len(key), record.py:24)."""
    return struct.pack("i", len(key)) + key.encode("utf-8") + struct.pack("i", len(value)) + value


def data_blocks(keys, values, block_size: int):
    """SSTableBuilder.add / finish_block (sstable.py:224-268): [(first_key, last_key, block bytes)]."""
    blocks = []
    cur, offs, first, last = bytearray(), [], None, None
    for k, v in zip(keys, values):
        rec = record_bytes(k, v)
        if len(cur) + len(rec) > block_size:  # blocks.py:84-85
            blocks.append((first, last, bytes(cur) + struct.pack("H" * len(offs), *offs) + struct.pack("H", len(offs))))
            cur, offs, first, last = bytearray(), [], None, None
            if len(rec) > block_size:  # the reference drops such a record silently (blocks.py:84-85)
                raise ValueError("record larger than block_size")
        offs.append(len(cur))
        cur += rec
        if first is None:
            first = k
        last = k
    blocks.append((first, last, bytes(cur) + struct.pack("H" * len(offs), *offs) + struct.pack("H", len(offs))))
    return blocks


def meta_block_bytes(first_key: str, last_key: str, offset: int) -> bytes:
    """MetaBlock.to_bytes (blocks.py:126-133)."""
    return (struct.pack("H", len(first_key)) + first_key.encode("utf-8") + struct.pack("H", len(last_key)) +
            last_key.encode("utf-8") + struct.pack("i", offset))


def data_and_meta(keys, values, block_size: int) -> tuple[bytes, bytes, list[tuple[str, str, int]]]:
    data, meta, metas = bytearray(), bytearray(), []
    for first, last, blk in data_blocks(keys, values, block_size):
        metas.append((first, last, len(data)))
        meta += meta_block_bytes(first, last, len(data))
        data += blk
    return bytes(data), bytes(meta), metas


def sstable_file(keys, values, block_size: int, bloom_bitmap: np.ndarray, k: int) -> bytes:
    """SSTableEncoding(data, meta_blocks, bloom).to_bytes() (sstable.py:80-86) given the bloom
    bitmap (nb_bytes, little-endian) and its k (bloom_filter.py:76-81)."""
    data, meta, _ = data_and_meta(keys, values, block_size)
    bloom = bloom_bitmap.tobytes() + struct.pack("B", k)
    return data + meta + bloom + struct.pack("i", len(data)) + struct.pack("i", len(data) + len(meta))
