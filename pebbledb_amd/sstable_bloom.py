"""The bloom section of an SSTable file, written from / read into the device bitmap.

Reference layout (src/sstable.py:57-62, 80-86, 89-100):

    data blocks ‖ meta blocks ‖ bloom bitmap (nb_bytes) ‖ k (1 B) ‖ meta_offset (i32) ‖ bloom_offset (i32)

``meta_offset = len(data)``, ``bloom_offset = len(data) + len(meta)``; both are native-endian
``struct "i"`` (little-endian here), which caps files at 2 GiB.  ``SSTableEncoding.from_bytes``
reads the two offsets from the last 8 bytes and hands ``data[bloom_offset:len-8]`` to
``BloomFilter.from_bytes``.

``encode_sstable`` sizes the output once and copies the bitmap from HBM straight into its slice of
the file buffer (one D2H copy, no intermediate ``bytes``); ``decode_bloom_section`` uploads the
bloom slice of a file buffer (one H2D copy) — the recovery path of SSTable.build_from_path
(src/sstable.py:193-206).
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np

INT_SIZE = 4  # struct "i" (src/sstable.py:10)
TRAILER = 2 * INT_SIZE


def bloom_section_bounds(file_bytes) -> tuple[int, int, int]:
    """(meta_offset, bloom_offset, bloom_end) from an SSTable's trailer (sstable.py:91-96)."""
    n = len(file_bytes)
    if n < TRAILER:
        raise ValueError("SSTable shorter than its 8-byte trailer")
    meta_offset, bloom_offset = struct.unpack("ii", bytes(file_bytes[n - TRAILER:n]))
    if not (0 <= meta_offset <= bloom_offset <= n - TRAILER - 1):
        raise ValueError(f"bad SSTable trailer: meta_offset={meta_offset} bloom_offset={bloom_offset}")
    return meta_offset, bloom_offset, n - TRAILER


def sstable_size(data_len: int, meta_len: int, nb_bytes: int) -> int:
    return data_len + meta_len + nb_bytes + 1 + TRAILER


def assemble(data: bytes, meta: bytes, nb_bytes: int, k: int, write_bitmap) -> bytearray:
    """Lay out an SSTable; ``write_bitmap(view)`` fills the nb_bytes-long bitmap slice in place."""
    if not 0 <= k <= 255:
        raise struct.error("ubyte format requires 0 <= number <= 255")  # as struct.pack("B", k)
    total = sstable_size(len(data), len(meta), nb_bytes)
    if data and len(data) + len(meta) > 0x7FFFFFFF:
        raise struct.error("'i' format requires -2147483648 <= number <= 2147483647")
    out = bytearray(total)
    o = 0
    out[o:o + len(data)] = data
    o += len(data)
    out[o:o + len(meta)] = meta
    o += len(meta)
    if nb_bytes:
        write_bitmap(memoryview(out)[o:o + nb_bytes])
    o += nb_bytes
    out[o] = k
    o += 1
    struct.pack_into("ii", out, o, len(data), len(data) + len(meta))
    return out


def encode_sstable(data: bytes, meta: bytes, bloom) -> bytearray:
    """SSTableEncoding(data, meta_blocks, bloom).to_bytes() (sstable.py:80-86) with the bitmap
    copied device → file buffer directly.  ``meta`` is the concatenated meta-block bytes."""
    from . import _native

    def write_bitmap(view):
        bloom._flush()
        arr = np.frombuffer(view, dtype=np.uint8)
        _native.check(_native.lib().pbf_get_bitmap(bloom.handle, ctypes.c_void_p(arr.ctypes.data), bloom.nb_bytes),
                      "pbf_get_bitmap")

    return assemble(data, meta, bloom.nb_bytes, bloom.nb_hash_functions, write_bitmap)


def decode_bloom_section(file_bytes, device=None):
    """The BloomFilter of an SSTable file buffer (sstable.py:89-100), uploaded with one H2D copy."""
    from .bloom_filter import BloomFilter

    _, bloom_offset, end = bloom_section_bounds(file_bytes)
    return BloomFilter.from_bytes(memoryview(file_bytes)[bloom_offset:end], device=device)
