"""Packed ingestion from the flush / compaction iterators (reference
src/sstable.py:224-244 and src/iterators.py:24-55,144-190) — host code, runs on CPU.  The C
packer (csrc/ingest.c) must produce exactly the boundary layout PackedKeys.from_strs produces
from the same keys (UTF-8 of str.encode, bloom_filter.py:43), and split the memtable's encoded
records exactly as Record._from_bytes (record.py:77-88) does."""
import struct

import numpy as np
import pytest

from pebbledb_amd.keys import PackedKeys, PackedRecords


class Rec:
    """Stands in for src/record.py:Record (what MemTableIterator / MergingIterator yield)."""
    __slots__ = ("key", "value")

    def __init__(self, key, value):
        self.key, self.value = key, value


def to_bytes(key: str, value: bytes) -> bytes:
    """Record.to_bytes (record.py:66-72): key_size = len(str) — CHARACTERS (record.py:25)."""
    return struct.pack("i", len(key)) + key.encode() + struct.pack("i", len(value)) + value


def from_bytes(data: bytes):
    """Record._from_bytes (record.py:77-88), restated: the key is sliced by key_size BYTES."""
    ks = struct.unpack("i", data[:4])[0]
    key = data[4:4 + ks].decode("utf-8")
    vs = struct.unpack("i", data[4 + ks:8 + ks])[0]
    return key, data[8 + ks:8 + ks + vs]


def _same(a: PackedKeys, b: PackedKeys):
    assert a.n == b.n and a.key_len == b.key_len
    assert a.data.tobytes() == b.data.tobytes()
    if a.offsets is None:
        assert b.offsets is None
    else:
        assert np.array_equal(a.offsets, b.offsets)


@pytest.mark.parametrize("keys", [
    [f"{i:016x}" for i in range(5000)],                       # fixed width -> key_len path
    [f"k{i}" for i in range(3000)] + ["", "é", "ключ", "🔑x"],  # variable, empty, non-ASCII
    [],
    ["only"],
])
def test_pack_keys_equals_from_strs(keys):
    want = PackedKeys.from_strs(keys)
    _same(PackedKeys.from_iter(keys), want)                 # list: index walk
    _same(PackedKeys.from_iter(iter(keys)), want)           # generic iterator
    _same(PackedKeys.from_iter(k for k in keys), want)      # generator (an iterator chain)
    _same(PackedKeys.from_iter([Rec(k, b"") for k in keys]), want)  # Record-like objects


def test_pack_records_and_encoded_records():
    rng = np.random.default_rng(5)
    keys = [f"key{i:07d}" for i in range(20000)] + ["", "é✓", "a" * 300]
    vals = [rng.integers(0, 256, int(rng.integers(0, 100)), dtype=np.uint8).tobytes() for _ in keys]
    want_k = PackedKeys.from_strs(keys)
    want_v = b"".join(vals)
    want_vo = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint64)
    for src in (list(zip(keys, vals)), (Rec(k, v) for k, v in zip(keys, vals)), [[k, v] for k, v in zip(keys, vals)],
                iter([(k, memoryview(v)) for k, v in zip(keys, vals)])):
        pr = PackedRecords.from_iter(src)
        _same(pr.keys, want_k)
        assert pr.values.tobytes() == want_v and np.array_equal(pr.value_offsets, want_vo)
        assert not pr.ascii
    ascii_keys = keys[:20000]
    enc = [to_bytes(k, v) for k, v in zip(ascii_keys, vals)]
    pe = PackedRecords.from_encoded(enc)
    _same(pe.keys, PackedKeys.from_strs(ascii_keys))
    assert pe.values.tobytes() == b"".join(vals[:20000]) and pe.ascii
    assert [pe.key_str(i) for i in (0, 123, 19999)] == [ascii_keys[i] for i in (0, 123, 19999)]


def test_encoded_records_follow_the_reference_decoder():
    """Non-ASCII keys: key_size counts characters but _from_bytes slices bytes, so the reference
    reads a shifted record — the packer reproduces that split (or its decode error) exactly."""
    recs = [to_bytes("aé", b"xyz" * 90), to_bytes("plain", b"v")]
    for r in recs:
        try:
            want = from_bytes(r)
        except UnicodeDecodeError:
            with pytest.raises(UnicodeDecodeError):
                PackedRecords.from_encoded([r])
            continue
        pr = PackedRecords.from_encoded([r])
        assert pr.keys.key(0) == want[0].encode() and pr.values.tobytes() == want[1]
    with pytest.raises(UnicodeDecodeError):  # 'é' cut after its first byte
        PackedRecords.from_encoded([struct.pack("i", 2) + "aé".encode()[:2] + struct.pack("i", 0)])
    for cut in (b"\x05\x00\x00\x00ab", b"\x01\x00"):  # size fields cut short: struct.error there too
        with pytest.raises(struct.error):
            from_bytes(cut)
        with pytest.raises(struct.error):
            PackedRecords.from_encoded([cut])
    # a value longer than the data is clipped, as the reference's slice clips it
    short = struct.pack("i", 2) + b"ab" + struct.pack("i", 10) + b"xyz"
    pr = PackedRecords.from_encoded([short])
    assert (pr.keys.key(0), pr.values.tobytes()) == tuple(x.encode() if isinstance(x, str) else x
                                                          for x in from_bytes(short))
    with pytest.raises(TypeError):
        PackedKeys.from_iter([1, 2])
    with pytest.raises(TypeError):
        PackedRecords.from_iter(["bare key"])


def test_buffers_outlive_the_packer_and_are_writable():
    pk = PackedKeys.from_iter(f"{i:08d}" for i in range(100000))
    data = pk.data
    del pk  # the numpy view keeps the packer's mapping alive by itself
    import gc
    gc.collect()
    assert data.flags.writeable and data[:8].tobytes() == b"00000000"
    assert data[-8:].tobytes() == b"00099999"


def _enc_bytes(kb: bytes, value: bytes) -> bytes:
    """A record whose key_size is its byte length (what a byte-level writer would store)."""
    return struct.pack("i", len(kb)) + kb + struct.pack("i", len(value)) + value


def _outcome(fn):
    try:
        pr = fn()
    except Exception as e:  # noqa: BLE001 - the exception type is what is compared
        return type(e)
    return (pr.keys.data.tobytes(), None if pr.keys.offsets is None else pr.keys.offsets.tobytes(),
            pr.values.tobytes(), pr.value_offsets.tobytes(), pr.ascii)


TRICKY_UTF8 = [b"\xc2\x80", b"\xdf\xbf", b"\xe0\xa0\x80", b"\xed\x9f\xbf", b"\xef\xbf\xbf", b"\xf0\x90\x80\x80",
               b"\xf4\x8f\xbf\xbf", b"\xc0\x80", b"\xc1\xbf", b"\xe0\x80\x80", b"\xe0\x9f\xbf", b"\xed\xa0\x80",
               b"\xed\xbf\xbf", b"\xf0\x80\x80\x80", b"\xf0\x8f\xbf\xbf", b"\xf4\x90\x80\x80", b"\xf5\x80\x80\x80",
               b"\xff", b"\x80", b"\xe2\x82", b"\xf0\x90\x80", b"a\xc3", "ключ🔑".encode(), b"\xe2\x82\xac\x80"]


@pytest.mark.parametrize("bad", TRICKY_UTF8)
def test_parallel_encoded_packer_matches_serial(bad):
    """Lists of more than 4096 exact bytes records take the threaded packer (csrc/ingest.c
    pack_encoded_parallel); an iterator takes the serial loop.  Both must give the same buffers,
    or the same exception, for keys on every edge of CPython's strict UTF-8 decoder."""
    rng = np.random.default_rng(len(bad))
    recs = [_enc_bytes(f"k{i:06d}".encode(), rng.integers(0, 256, int(rng.integers(0, 40)),
                                                           dtype=np.uint8).tobytes()) for i in range(6000)]
    recs[4321] = _enc_bytes(b"pre" + bad + b"post", b"value")
    try:
        (b"pre" + bad + b"post").decode("utf-8")
        valid = True
    except UnicodeDecodeError:
        valid = False
    par = _outcome(lambda: PackedRecords.from_encoded(recs))
    ser = _outcome(lambda: PackedRecords.from_encoded(iter(recs)))
    assert par == ser
    assert (par is UnicodeDecodeError) == (not valid)


def test_parallel_encoded_packer_errors_and_mixed_items():
    recs = [_enc_bytes(f"key{i:05d}".encode(), b"v" * (i % 7)) for i in range(9000)]
    base = _outcome(lambda: PackedRecords.from_encoded(iter(recs)))
    assert _outcome(lambda: PackedRecords.from_encoded(recs)) == base
    assert _outcome(lambda: PackedRecords.from_encoded(tuple(recs))) == base
    mixed = list(recs)
    mixed[10] = bytearray(mixed[10])  # not exact bytes: the serial loop packs the whole list
    assert _outcome(lambda: PackedRecords.from_encoded(mixed)) == base
    for i, broken, err in ((8000, b"\x01\x00", struct.error), (5000, struct.pack("i", -1) + b"abcd", ValueError),
                           (7000, struct.pack("i", 2) + b"ab" + struct.pack("i", -5), ValueError)):
        r = list(recs)
        r[i] = broken
        assert _outcome(lambda: PackedRecords.from_encoded(r)) is err
        assert _outcome(lambda: PackedRecords.from_encoded(iter(r))) is err
    # the first bad record decides the exception, as in the reference's in-order decode
    r = list(recs)
    r[6000] = b"\x01\x00"
    r[6500] = _enc_bytes(b"\xff", b"")
    assert _outcome(lambda: PackedRecords.from_encoded(r)) is struct.error
    r[5000] = _enc_bytes(b"\xff", b"")
    assert _outcome(lambda: PackedRecords.from_encoded(r)) is UnicodeDecodeError
