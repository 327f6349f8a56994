"""SSTable data/meta encoding: the oracle restatement (oracle/sstable_oracle.py) and the host
block planner (pebbledb_amd/sstable_data.py) pinned to files the REAL reference's
SSTableBuilder wrote (tests/golden/sstable_build.json, tools/gen_golden_sstable.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import sstable_oracle as so
from oracle.oracle import sizing
from pebbledb_amd.keys import PackedKeys
from pebbledb_amd.sstable_data import key_offsets, meta_blocks, pack_values, plan_blocks

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "sstable_build.json")


def golden_cases():
    cases = json.load(open(GOLDEN))["cases"]
    for c in cases:
        if "keys" in c:
            c["_keys"] = c["keys"]
            c["_vals"] = [bytes.fromhex(v) for v in c["values_hex"]]
        else:  # default_blocks: the rules written by the generator
            c["_keys"] = [f"{i:016x}" for i in range(2500)]
            c["_vals"] = [bytes(((i * 131 + j * 29) & 0xFF) for j in range(40 + i % 90)) for i in range(2500)]
    return cases


CASES = golden_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_file(oracle, case):
    keys, vals, bs = case["_keys"], case["_vals"], case["block_size"]
    nb, k = sizing(len(keys), 0.001)
    bitmap = oracle.build(nb, k, PackedKeys.from_strs(keys))
    f = so.sstable_file(keys, vals, bs, bitmap, k)
    assert len(f) == case["file_len"]
    assert hashlib.sha256(f).hexdigest() == case["file_sha256"]
    if "file_hex" in case:
        assert f.hex() == case["file_hex"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_planner_and_meta_match_reference(case):
    keys, vals, bs = case["_keys"], case["_vals"], case["block_size"]
    pk = PackedKeys.from_strs(keys)
    _, vo = pack_values(vals)
    bf, bo = plan_blocks(key_offsets(pk), vo, bs)
    want = case["meta_blocks"]
    assert len(bf) - 1 == len(want)
    assert [int(x) for x in bo[:-1]] == [m["offset"] for m in want]
    assert int(bo[-1]) == case["meta_block_offset"]  # the data section's length
    meta, metas = meta_blocks(keys, bf, bo)
    assert [(a, b) for a, b, _ in metas] == [(m["first_key"], m["last_key"]) for m in want]
    _, want_meta, _ = so.data_and_meta(keys, vals, bs)
    assert meta == want_meta


def test_planner_rejects_what_the_reference_mishandles():
    pk = PackedKeys.from_strs(["a", "b"])
    _, vo = pack_values([b"x" * 300, b""])
    with pytest.raises(ValueError):
        plan_blocks(key_offsets(pk), vo, 256)  # record larger than the block
    with pytest.raises(ValueError):
        plan_blocks(np.zeros(1, np.uint64), np.zeros(1, np.uint64), 256)  # no records
    with pytest.raises(ValueError):
        plan_blocks(key_offsets(pk), vo, 1 << 17)  # u16 offsets


def test_record_key_size_counts_characters():
    # record.py:24 — key_size = len(str): 4 for "clé!" although it is 5 UTF-8 bytes
    assert so.record_bytes("clé!", b"v")[:4] == (4).to_bytes(4, "little")


def test_native_block_planner_equals_reference_rule():
    """pbf_plan_blocks (host C, no GPU) == the numpy restatement of DataBlockBuilder.add's rule
    (blocks.py:78-95) on random record sizes, exactly-full blocks and single-record blocks."""
    from pebbledb_amd.sstable_data import plan_blocks, plan_blocks_native
    rng = np.random.default_rng(1)
    for n, bs, maxk, maxv in ((1, 64, 8, 8), (5000, 256, 30, 100), (20000, 65536, 64, 3000), (300, 100, 40, 52)):
        kl = rng.integers(0, maxk + 1, n)
        vl = rng.integers(0, maxv + 1, n)
        kl = np.minimum(kl, bs - 8)
        vl = np.minimum(vl, bs - 8 - kl)
        ko = np.concatenate([[0], np.cumsum(kl)]).astype(np.uint64)
        vo = np.concatenate([[0], np.cumsum(vl)]).astype(np.uint64)
        a, b = plan_blocks(ko, vo, bs)
        c, d = plan_blocks_native(ko, vo, bs)
        assert np.array_equal(a, c) and np.array_equal(b, d), (n, bs)
    ko = np.array([0, 10], np.uint64)
    vo = np.array([0, 60], np.uint64)
    with pytest.raises(ValueError):
        plan_blocks_native(ko, vo, 64)  # 10 + 60 + 8 > 64
