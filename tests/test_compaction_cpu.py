"""Compaction's output split (LsmStorage._compact, src/lsm_storage.py:233-251) on the host block
plan (pebbledb_amd/sstable_data.plan_compaction), pinned to the files the REAL reference's
_compact wrote (tests/golden/compaction_split.json, tools/gen_golden_compaction.py): the number
of output SSTables, each one's record range and data-section length, and — through the oracle
restatement of the SSTable encoding and the C bloom oracle — every file's sha256."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import sstable_oracle as so
from oracle.oracle import sizing
from pebbledb_amd.keys import PackedKeys
from pebbledb_amd.sstable_data import key_offsets, pack_values, plan_compaction

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "compaction_split.json")
CASES = json.load(open(GOLDEN))["cases"]


def case_records(c):
    """The generator's inputs, rebuilt from its rules."""
    keys = [c["key"].format(i=i) for i in range(c["n"])]
    vals = [bytes(((i * 131 + j * 29) & 0xFF) for j in range(eval(c["vlen"], {"i": i}))) for i in range(c["n"])]
    return keys, vals


def plan(c, keys, vals):
    pk = PackedKeys.from_strs(keys)
    _, vo = pack_values(vals)
    return plan_compaction(np.asarray(key_offsets(pk), np.uint64), vo, c["block_size"], c["max_sstable_size"])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_plan_matches_reference_compaction(case):
    keys, vals = case_records(case)
    bf, bo, tb, written = plan(case, keys, vals)
    outs = case["outputs"]
    assert len(tb) - 1 == len(outs)
    assert written == case["records_written"]
    for t, o in enumerate(outs):
        b0, b1 = int(tb[t]), int(tb[t + 1])
        assert (int(bf[b0]), int(bf[b1])) == (o["first_record"], o["end_record"]), t
        assert int(bo[b1] - bo[b0]) == o["data_len"], t


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_files_match_reference_compaction(oracle, case):
    """Every output file, re-encoded by the oracle restatement over the planned record range,
    equals the reference's file byte for byte (sha256)."""
    keys, vals = case_records(case)
    for o in case["outputs"]:
        ks, vs = keys[o["first_record"]:o["end_record"]], vals[o["first_record"]:o["end_record"]]
        nb, k = sizing(len(ks), 0.001)
        assert (nb, k) == (o["nb_bytes"], o["k"])
        f = so.sstable_file(ks, vs, case["block_size"], oracle.build(nb, k, PackedKeys.from_strs(ks)), k)
        assert len(f) == o["file_len"] and hashlib.sha256(f).hexdigest() == o["file_sha256"]


def test_plan_empty_and_oversized_records():
    z = np.zeros(1, np.uint64)
    bf, bo, tb, w = plan_compaction(z, z, 1024, 4096)
    assert len(tb) == 1 and w == 0
    ko = np.array([0, 2000], np.uint64)
    with pytest.raises(ValueError):
        plan_compaction(ko, np.zeros(2, np.uint64), 1024, 4096)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_native_planner_equals_restatement(case):
    """pbf_plan_compaction (C, what build_sstables uses) == plan_compaction (numpy) on the golden
    runs and on random runs with many split points (host-side, no GPU)."""
    from pebbledb_amd.sstable_data import plan_compaction_native
    keys, vals = case_records(case)
    pk = PackedKeys.from_strs(keys)
    _, vo = pack_values(vals)
    ko = np.asarray(key_offsets(pk), np.uint64)
    a = plan_compaction(ko, vo, case["block_size"], case["max_sstable_size"])
    b = plan_compaction_native(ko, vo, case["block_size"], case["max_sstable_size"])
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y)
    assert a[3] == b[3]


def test_native_planner_random_runs():
    from pebbledb_amd.sstable_data import plan_compaction_native
    rng = np.random.default_rng(3)
    for trial in range(40):
        n = int(rng.integers(1, 3000))
        bs = int(rng.choice([64, 256, 1000, 4096]))
        kl = rng.integers(0, 24, n)
        vl = rng.integers(0, max(1, bs - 8 - 24), n)
        vl = np.minimum(vl, bs - 8 - kl)
        ko = np.zeros(n + 1, np.uint64)
        vo = np.zeros(n + 1, np.uint64)
        np.cumsum(kl, out=ko[1:])
        np.cumsum(vl, out=vo[1:])
        mx = int(rng.integers(1, 20 * bs))
        a = plan_compaction(ko, vo, bs, mx)
        b = plan_compaction_native(ko, vo, bs, mx)
        for x, y in zip(a[:3], b[:3]):
            assert np.array_equal(x, y), trial
        assert a[3] == b[3], trial


def test_non_positive_split_size_is_refused():
    """max_sstable_size <= 0: the reference (position tested after every add, lsm_storage.py:241)
    would build one SSTable per record; both planners refuse the size instead of silently
    splitting at the first finished block (round-4 advice)."""
    from pebbledb_amd.sstable_data import plan_compaction_native
    ko = np.array([0, 3, 6], np.uint64)
    vo = np.array([0, 10, 20], np.uint64)
    for mx in (0, -1):
        with pytest.raises(ValueError, match="max_sstable_size"):
            plan_compaction(ko, vo, 1024, mx)
        with pytest.raises(ValueError, match="max_sstable_size"):
            plan_compaction_native(ko, vo, 1024, mx)
