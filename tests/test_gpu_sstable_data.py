"""Device SSTable build (pbf_encode_data_blocks + device bloom): byte-identical to files the
real reference's SSTableBuilder wrote (tests/golden/sstable_build.json) and to the oracle
restatement (oracle/sstable_oracle.py) on larger random record sets."""
import ctypes
import hashlib

import numpy as np
import pytest

from oracle import sstable_oracle as so
from pebbledb_amd import _native
from pebbledb_amd.keys import PackedKeys, PackedRecords
from pebbledb_amd.sstable_data import (build_sstable, encode_data_blocks, key_offsets, pack_values,
                                       plan_blocks)

from test_sstable_data_cpu import CASES

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_device_sstable_equals_reference_file(case):
    f, metas, bloom = build_sstable(case["_keys"], case["_vals"], case["block_size"])
    assert len(f) == case["file_len"]
    assert hashlib.sha256(bytes(f)).hexdigest() == case["file_sha256"]
    assert [m[2] for m in metas] == [m["offset"] for m in case["meta_blocks"]]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_packed_records_flush_equals_reference_file(case):
    """The flush without list[str]: records packed as the iterator yields them (csrc/ingest.c)
    give the same file bytes as the real reference's SSTableBuilder (sstable.py:224-288)."""
    import struct

    class Rec:
        __slots__ = ("key", "value")

        def __init__(self, k, v):
            self.key, self.value = k, v

    srcs = [PackedRecords.from_iter(zip(case["_keys"], case["_vals"])),
            PackedRecords.from_iter(Rec(k, v) for k, v in zip(case["_keys"], case["_vals"]))]
    if all(k.isascii() for k in case["_keys"]):  # encoded records split as Record._from_bytes does
        srcs.append(PackedRecords.from_encoded(
            [struct.pack("i", len(k)) + k.encode() + struct.pack("i", len(v)) + v
             for k, v in zip(case["_keys"], case["_vals"])]))
    for pr in srcs:
        f, metas, bloom = build_sstable(pr, block_size=case["block_size"])
        assert len(f) == case["file_len"]
        assert hashlib.sha256(bytes(f)).hexdigest() == case["file_sha256"]
        assert [m[2] for m in metas] == [m["offset"] for m in case["meta_blocks"]]
        assert [(m[0], m[1]) for m in metas] == [(m["first_key"], m["last_key"]) for m in case["meta_blocks"]]


def _random_records(rng, n, maxk, maxv, unicode_every=0):
    keys, vals = [], []
    for i in range(n):
        L = int(rng.integers(0, maxk + 1))
        k = "".join(chr(97 + int(x)) for x in rng.integers(0, 26, L))
        if unicode_every and i % unicode_every == 0:
            k += "é✓"
        keys.append(k)
        vals.append(rng.integers(0, 256, int(rng.integers(0, maxv + 1)), dtype=np.uint8).tobytes())
    return keys, vals


@pytest.mark.parametrize("n,bs,maxk,maxv,uni", [(20000, 4096, 40, 200, 13), (60000, 65536, 64, 512, 0),
                                                (5000, 256, 24, 60, 5), (3000, 65536, 8, 8, 0)])
def test_data_section_matches_oracle(n, bs, maxk, maxv, uni):
    rng = np.random.default_rng(n + bs)
    keys, vals = _random_records(rng, n, maxk, maxv, uni)
    pk = PackedKeys.from_strs(keys)
    vb, vo = pack_values(vals)
    bf, bo = plan_blocks(key_offsets(pk), vo, bs)
    got = encode_data_blocks(pk, vb, vo, bf, bo)
    want, _, _ = so.data_and_meta(keys, vals, bs)
    assert got.tobytes() == want


def test_device_pointers_and_bad_plans():
    keys = [f"k{i:05d}" for i in range(3000)]
    vals = [bytes([i & 0xFF]) * (i % 50) for i in range(3000)]
    pk = PackedKeys.from_strs(keys)
    vb, vo = pack_values(vals)
    ko = key_offsets(pk)
    bf, bo = plan_blocks(ko, vo, 1024)
    want, _, _ = so.data_and_meta(keys, vals, 1024)
    dev = {name: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).cuda()
           for name, a in (("k", pk.data), ("ko", ko), ("v", vb), ("vo", vo), ("bf", bf), ("bo", bo))}
    out = torch.zeros(int(bo[-1]), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    rc = _native.lib().pbf_encode_data_blocks(0, dev["k"].data_ptr(), dev["ko"].data_ptr(), dev["v"].data_ptr(),
                                              dev["vo"].data_ptr(), pk.n, dev["bf"].data_ptr(), dev["bo"].data_ptr(),
                                              len(bf) - 1, out.data_ptr(), 1)
    _native.check(rc, "encode")
    assert out.cpu().numpy().tobytes() == want
    # a host plan whose block overflows 65536 data bytes is refused before any device work
    bad = np.array([0, pk.n], dtype=np.uint64)
    big_v = [b"x" * 40 for _ in range(pk.n)]
    vb2, vo2 = pack_values(big_v)
    with pytest.raises(ValueError):
        encode_data_blocks(pk, vb2, vo2, bad, np.array([0, 10], dtype=np.uint64))


# ---------------------------------------------------------------- compaction's output split
from test_compaction_cpu import CASES as COMPACTION_CASES, case_records  # noqa: E402


@pytest.mark.parametrize("case", COMPACTION_CASES, ids=[c["name"] for c in COMPACTION_CASES])
def test_build_sstables_equals_reference_compaction(case):
    """build_sstables (one upload, one encode launch for every output, the filters on their own
    streams) writes the files the REAL reference's _compact wrote (tests/golden/
    compaction_split.json): the same number of SSTables, each byte for byte (sha256), the same
    records left out at the end; each output also equals build_sstable of its record range."""
    from pebbledb_amd.sstable_data import build_sstables
    keys, vals = case_records(case)
    outs, written = build_sstables(keys, vals, case["max_sstable_size"], case["block_size"])
    assert written == case["records_written"]
    assert len(outs) == len(case["outputs"])
    for (f, metas, bloom), o in zip(outs, case["outputs"]):
        assert len(f) == o["file_len"]
        assert hashlib.sha256(bytes(f)).hexdigest() == o["file_sha256"], o["first_record"]
        assert (bloom.nb_bytes, bloom.nb_hash_functions) == (o["nb_bytes"], o["k"])
        one, _, _ = build_sstable(keys[o["first_record"]:o["end_record"]], vals[o["first_record"]:o["end_record"]],
                                  case["block_size"])
        assert bytes(one) == bytes(f)


def test_build_sstables_packed_large_run(oracle):
    """A flush-scale run through PackedRecords: 400k records of 16-B keys + 40..103-B values,
    64 KiB blocks, 6 MB outputs (5 tables, filters built concurrently on pooled streams): every
    output equals build_sstable of its range, and its bitmap equals the C oracle's."""
    from pebbledb_amd.sstable_data import build_sstables, plan_compaction
    from pebbledb_amd.keys import splitmix_hex_keys_str
    n = 400_000
    keys = sorted(splitmix_hex_keys_str(77, 0, n))
    vals = [bytes(((i * 131 + j * 29) & 0xFF) for j in range(40 + i % 64)) for i in range(n)]
    recs = PackedRecords.from_iter(zip(keys, vals))
    outs, written = build_sstables(recs, max_sstable_size=6_000_000)
    bf, bo, tb, w = plan_compaction(np.asarray(key_offsets(recs.keys), np.uint64), recs.value_offsets, 65536, 6_000_000)
    assert written == w and len(outs) == len(tb) - 1 >= 4
    for t, (f, metas, bloom) in enumerate(outs):
        r0, r1 = int(bf[tb[t]]), int(bf[tb[t + 1]])
        one, _, b1 = build_sstable(keys[r0:r1], vals[r0:r1])
        assert bytes(one) == bytes(f), t
        want = oracle.build(bloom.nb_bytes, bloom.nb_hash_functions, PackedKeys.from_strs(keys[r0:r1]), omp=True)
        assert bloom.bitmap() == want.tobytes(), t
