"""Key streams and the packed key layout handed across the C-ABI.

The reference hashes ``key.encode("utf-8")`` (src/bloom_filter.py:43).  Across the boundary a
batch of keys is either

* fixed-width: ``n`` keys of ``key_len`` bytes, back to back (``uint8[n * key_len]``), or
* variable-length: concatenated UTF-8 bytes plus ``uint64 offsets[n + 1]`` (key ``i`` is
  ``bytes[offsets[i]:offsets[i+1]]``).

Synthetic workloads — the same definitions are implemented by the device
generators ``k_gen_splitmix_hex`` / ``k_gen_varlen`` (csrc/bloom_kernels.hpp) and checked
against these in tests:

* ``splitmix_hex``: key ``i`` = 16 lowercase hex chars of ``splitmix64(seed + i)``.
* ``varlen``: ``h = splitmix64((seed << 32) + i)``; length ``8 + h % 57`` (8..64 bytes);
  char ``p`` = ``ALPHABET[byte(p % 8) of splitmix64(h + 1 + p // 8) % 36]``, alphabet [0-9a-z].
"""
from __future__ import annotations

import numpy as np

MASK64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
ALPHABET = b"0123456789abcdefghijklmnopqrstuvwxyz"
HEX = b"0123456789abcdef"


def splitmix64(x: int) -> int:
    z = (x + GOLDEN) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def _splitmix64_np(x: np.ndarray) -> np.ndarray:
    z = x.astype(np.uint64) + np.uint64(GOLDEN)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def splitmix_hex_keys_str(seed: int, start: int, n: int) -> list[str]:
    return [format(splitmix64(seed + i), "016x") for i in range(start, start + n)]


def splitmix_hex_keys(seed: int, start: int, n: int) -> np.ndarray:
    """uint8[n, 16]: the fixed-width packed form of ``splitmix_hex_keys_str``."""
    with np.errstate(over="ignore"):
        idx = np.arange(start, start + n, dtype=np.uint64) + np.uint64(seed)
        z = _splitmix64_np(idx)
    shifts = np.arange(60, -4, -4, dtype=np.uint64)  # most significant nibble first
    nib = ((z[:, None] >> shifts[None, :]) & np.uint64(0xF)).astype(np.uint8)
    return np.frombuffer(HEX, dtype=np.uint8)[nib]


def _varlen_one(seed: int, i: int) -> str:
    h = splitmix64(((seed << 32) + i) & MASK64)
    L = 8 + h % 57
    out = bytearray(L)
    for p in range(L):
        w = splitmix64((h + 1 + p // 8) & MASK64)
        out[p] = ALPHABET[((w >> (8 * (p % 8))) & 0xFF) % 36]
    return out.decode("ascii")


def varlen_keys_str(seed: int, start: int, n: int) -> list[str]:
    return [_varlen_one(seed, i) for i in range(start, start + n)]


def varlen_keys(seed: int, start: int, n: int) -> tuple[np.ndarray, np.ndarray]:
    """(uint8 bytes, uint64 offsets[n+1]) packed form of ``varlen_keys_str``."""
    with np.errstate(over="ignore"):
        i = np.arange(start, start + n, dtype=np.uint64)
        h = _splitmix64_np((np.uint64(seed) << np.uint64(32)) + i)
        lens = (np.uint64(8) + h % np.uint64(57)).astype(np.int64)
        words = np.empty((n, 8), dtype=np.uint64)
        for j in range(8):
            words[:, j] = _splitmix64_np(h + np.uint64(1 + j))
    raw = words.view(np.uint8).reshape(n, 64)  # little-endian: byte p%8 of word p//8
    chars = np.frombuffer(ALPHABET, dtype=np.uint8)[raw % 36]
    mask = np.arange(64)[None, :] < lens[:, None]
    data = chars[mask]
    offsets = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    return np.ascontiguousarray(data), offsets


class PackedKeys:
    """A batch of keys in the boundary layout. ``key_len`` > 0 ⇒ fixed-width, offsets None."""

    __slots__ = ("data", "offsets", "n", "key_len", "_ko")

    def __init__(self, data: np.ndarray, n: int, key_len: int = 0, offsets: np.ndarray | None = None):
        self._ko = None  # the packer's offsets of a fixed-width batch (sstable_data.key_offsets)
        self.data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        self.n = int(n)
        self.key_len = int(key_len)
        self.offsets = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        if self.key_len <= 0 and self.offsets is None:
            raise ValueError("variable-length keys need offsets[n+1]")
        if self.offsets is not None and len(self.offsets) != self.n + 1:
            raise ValueError("offsets must have n+1 entries")

    @classmethod
    def from_strs(cls, keys) -> "PackedKeys":
        """UTF-8 encode (bloom_filter.py:43) and pack.  The common all-ASCII batch is encoded as
        ONE joined string (byte length == character length exactly when every key is ASCII),
        about 3x faster than encoding key by key; otherwise each key is encoded on its own."""
        keys = keys if isinstance(keys, list) else list(keys)
        n = len(keys)
        if n == 0:
            return cls(np.zeros(0, np.uint8), 0, key_len=0, offsets=np.zeros(1, np.uint64))
        joined = "".join(keys).encode("utf-8")
        lens = np.fromiter(map(len, keys), dtype=np.int64, count=n)
        if int(lens.sum()) != len(joined):  # some key is not ASCII: byte lengths differ
            enc = [k.encode("utf-8") for k in keys]
            lens = np.fromiter(map(len, enc), dtype=np.int64, count=n)
            joined = b"".join(enc)
        data = np.frombuffer(joined, dtype=np.uint8)
        L0 = int(lens[0])
        if L0 > 0 and bool((lens == L0).all()):
            return cls(data, n, key_len=L0)
        offsets = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens, out=offsets[1:])
        return cls(data, n, key_len=0, offsets=offsets)

    @classmethod
    def fixed(cls, arr2d: np.ndarray) -> "PackedKeys":
        a = np.ascontiguousarray(arr2d, dtype=np.uint8)
        return cls(a.reshape(-1), a.shape[0], key_len=a.shape[1])

    @classmethod
    def from_iter(cls, keys) -> "PackedKeys":
        """Pack an iterable of str / bytes keys (or records: (key, value) pairs or objects with
        .key) as it is drained, in one C loop (csrc/ingest.c) — no list[str] materialised."""
        kb, ko, _, _, n, _, lo, hi = _ingest().pack_keys(keys)
        return cls._from_packed(kb, ko, n, lo, hi)

    @classmethod
    def _from_packed(cls, kb, ko, n, lo, hi) -> "PackedKeys":
        data = np.frombuffer(kb, dtype=np.uint8) if len(kb) else np.zeros(0, np.uint8)
        if n and lo == hi and lo > 0:
            pk = cls(data, n, key_len=int(lo))
            pk._ko = np.frombuffer(ko, dtype=np.uint64)
            return pk
        return cls(data, n, key_len=0, offsets=np.frombuffer(ko, dtype=np.uint64))

    def key(self, i: int) -> bytes:
        if self.key_len > 0:
            return self.data[i * self.key_len:(i + 1) * self.key_len].tobytes()
        return self.data[int(self.offsets[i]):int(self.offsets[i + 1])].tobytes()


def _ingest():
    """The packed-ingestion extension (built by pebbledb_amd/build.py; host code, no GPU)."""
    from . import _pebbleingest
    return _pebbleingest


class PackedRecords:
    """A flushed / compacted run of records in the boundary layout: keys (PackedKeys) plus value
    bytes and u64 value offsets[n+1] — what SSTableBuilder.add accumulates record by record
    (src/sstable.py:224-244), packed straight from the iterator that yields them
    (MemTableIterator / MergingIterator, src/iterators.py:24-55,144-190)."""

    __slots__ = ("keys", "values", "value_offsets", "n", "ascii")

    def __init__(self, keys: PackedKeys, values: np.ndarray, value_offsets: np.ndarray, ascii: bool = False):
        self.keys = keys
        self.values = values
        self.value_offsets = value_offsets
        self.n = keys.n
        self.ascii = bool(ascii)
        if len(value_offsets) != self.n + 1:
            raise ValueError("value offsets must have n+1 entries")

    @classmethod
    def from_iter(cls, records) -> "PackedRecords":
        """Drain `records` — Record objects (.key str, .value bytes), (key, value) pairs — in one
        C loop into packed key / value buffers."""
        kb, ko, vb, vo, n, ascii, lo, hi = _ingest().pack_records(records)
        keys = PackedKeys._from_packed(kb, ko, n, lo, hi)
        values = np.frombuffer(vb, dtype=np.uint8) if len(vb) else np.zeros(0, np.uint8)
        return cls(keys, values, np.frombuffer(vo, dtype=np.uint64), ascii=bool(ascii))

    @classmethod
    def from_encoded(cls, encoded) -> "PackedRecords":
        """Drain encoded records — the bytes the memtable stores (memtable.map values,
        Record.to_bytes, src/record.py:66-72) — split exactly as Record._from_bytes does
        (record.py:77-88), in one C loop: no Record objects are created."""
        kb, ko, vb, vo, n, ascii, lo, hi = _ingest().pack_encoded(encoded)
        keys = PackedKeys._from_packed(kb, ko, n, lo, hi)
        values = np.frombuffer(vb, dtype=np.uint8) if len(vb) else np.zeros(0, np.uint8)
        return cls(keys, values, np.frombuffer(vo, dtype=np.uint64), ascii=bool(ascii))

    def key_str(self, i: int) -> str:
        return self.keys.key(i).decode("utf-8")
