"""Golden compaction outputs from the REAL reference's ``LsmStorage._compact`` (build container
only):

    python tools/gen_golden_compaction.py

Writes tests/golden/compaction_split.json.  For a few record runs (inputs given by rule, the
sorted de-duplicated stream the merging iterator feeds compaction) the SSTable files the
reference's compaction writes: ``_compact`` (src/lsm_storage.py:233-251) starts a new
``SSTableBuilder`` once ``current_buffer_position >= max_sstable_size`` — a position that only
advances when a data block finishes (src/sstable.py:224-268) — and builds the last builder only
if its position is past 0, so records still in the last builder's first open block are not
written (the reference's own behaviour, kept as data here).  Per output: record range, first /
last key, file length, sha256, data-section length.  The reference's mmh3 dependency is the
stand-in of tools/mmh3_shim (see tools/gen_golden.py).
"""
from __future__ import annotations

import hashlib
import itertools
import json
import os
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden", "compaction_split.json")
sys.path.insert(0, os.path.join(HERE, "mmh3_shim"))
sys.path.insert(1, "/root/reference")

from src.lsm_storage import LsmStorage  # noqa: E402  (the reference)
from src.record import Record  # noqa: E402

# Each case: inputs by rule (tests/test_compaction_cpu.py rebuilds them from the same rules).
CASES = [
    # several splits, the last output a partial table
    {"name": "splits", "n": 3000, "key": "k{i:08d}", "vlen": "20 + i % 50", "block_size": 1024, "max_sstable_size": 16384},
    # the records after the last split fit one open block: the reference writes no last table
    {"name": "tail_dropped", "n": 1084, "key": "k{i:08d}", "vlen": "20 + i % 50", "block_size": 1024,
     "max_sstable_size": 16384},
    # a run smaller than one block: no output at all
    {"name": "one_open_block", "n": 10, "key": "k{i:08d}", "vlen": "16", "block_size": 65536, "max_sstable_size": 262144000},
    # 64-byte records into 256-byte blocks: every block exactly full; a split on every 4th block
    {"name": "exact_blocks", "n": 400, "key": "k{i:07d}", "vlen": "48", "block_size": 256, "max_sstable_size": 1040},
    # non-ASCII keys (key_size in characters, record.py:24) and the default block size
    {"name": "unicode_default_blocks", "n": 6000, "key": "clé{i:06d}", "vlen": "30 + (i * 7) % 90", "block_size": 65536,
     "max_sstable_size": 200000},
]


def value_of(i: int, n: int) -> bytes:
    return bytes(((i * 131 + j * 29) & 0xFF) for j in range(n))


def records(case):
    for i in range(case["n"]):
        yield Record(key=case["key"].format(i=i), value=value_of(i, eval(case["vlen"], {"i": i})))


def run(case):
    with tempfile.TemporaryDirectory() as d:
        counter = itertools.count()
        fake = types.SimpleNamespace(
            _configuration=types.SimpleNamespace(max_sstable_size=case["max_sstable_size"],
                                                 block_size=case["block_size"]),
            _compute_path=lambda: os.path.join(d, f"{next(counter):06d}.sst"))  # unique paths
        tables = LsmStorage._compact(fake, records(case))
        outs, at = [], 0
        keys = [case["key"].format(i=i) for i in range(case["n"])]
        for t in tables:
            with open(t.file.path, "rb") as f:
                data = f.read()
            lo = keys.index(t.first_key, at)
            hi = keys.index(t.last_key, lo) + 1
            at = hi
            outs.append({"first_record": lo, "end_record": hi, "first_key": t.first_key, "last_key": t.last_key,
                         "file_len": len(data), "file_sha256": hashlib.sha256(data).hexdigest(),
                         "data_len": t.meta_block_offset, "nb_bytes": t.bloom_filter.nb_bytes,
                         "k": t.bloom_filter.nb_hash_functions})
    return outs


def main() -> None:
    cases = []
    for c in CASES:
        outs = run(c)
        covered = outs[-1]["end_record"] if outs else 0
        cases.append(dict(c, outputs=outs, records_written=covered))
        print(c["name"], len(outs), "tables,", covered, "of", c["n"], "records written")
    with open(OUT, "w") as f:
        json.dump({"generator": "tools/gen_golden_compaction.py (reference LsmStorage._compact)",
                   "value_rule": "bytes(((i * 131 + j * 29) & 0xFF) for j in range(vlen))", "cases": cases}, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
