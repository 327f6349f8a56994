"""Generate tests/golden/lsm_get_order.json from the REAL reference's ``LsmStorage.get``.

Runs only in the build container (``/root/reference`` does not exist on the GPU box):

    python tools/gen_golden_lsm.py

A reference store (``LsmStorage.create``, src/lsm_storage.py:60-85) gets L0 and L1/L2 SSTables
whose bloom filters the reference itself builds with the product sizing
(``BloomFilter.build_from_keys_and_fp_rate(keys, 0.001)``, src/sstable.py:274 — so every table
has its own nb_bytes, as in a real LSM).  Each SSTable has no data blocks, so ``SSTable.get``
returns None and ``get`` walks every candidate; each table's ``get`` is replaced by a recorder,
the way src/__tests__/test_lsm_storage.py:287-317 wraps it with ``mock.patch.object``.  The
fixture holds the inputs (the key universe, each table's level / key slice / first and last
key), the reference's filter for each table (nb_bytes, k, sha256 and popcount of the bitmap),
and, per probe key, the tables ``get`` read, in its order.  The reference's one third-party
dependency, mmh3, is the stand-in of tools/gen_golden.py (tools/mmh3_shim).
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden", "lsm_get_order.json")
sys.path.insert(0, os.path.join(HERE, "mmh3_shim"))
sys.path.insert(1, "/root/reference")

from src.bloom_filter import BloomFilter  # noqa: E402  (the reference, bloom_filter.py:8)
from src.lsm_storage import LsmStorage  # noqa: E402  (src/lsm_storage.py:32)
from src.sstable import SSTable, SSTableFile  # noqa: E402  (src/sstable.py:116, :13)


def main():
    rng = random.Random(20261017)
    universe = ["k%05d" % i for i in range(8000)]
    universe += ["é%03d" % i for i in range(40)] + ["\U0001f511%d" % i for i in range(20)] + ["A", "zz"]
    universe = sorted(set(universe))
    U = len(universe)
    # (level, first index, last index exclusive, step): L0 newest first, overlapping; L1 disjoint
    # ranges; L2 overlapping ranges, a one-key table and one past every probe key
    specs = [
        (0, 0, 4000, 3), (0, 2000, 7000, 2), (0, 5000, U, 5), (0, 100, 900, 1),
        (1, 0, 2000, 1), (1, 2000, 4500, 1), (1, 4500, 7000, 1), (1, 7000, U, 1),
        (2, 500, 3000, 1), (2, 2500, 6000, 1), (2, 4242, 4243, 1), (2, 6000, U - 3, 1), (2, U - 2, U, 1),
    ]
    tables = []
    with tempfile.TemporaryDirectory() as tmp:
        store = LsmStorage.create(directory=tmp, nb_levels=2)
        calls: list[int] = []
        for t, (lvl, a, b, step) in enumerate(specs):
            keys = universe[a:b:step]
            bf = BloomFilter.build_from_keys_and_fp_rate(keys, 0.001)
            bm = bf.bits.to_bytes(bf.nb_bytes, "little")
            sst = SSTable(meta_blocks=[], meta_block_offset=0, bloom_filter=bf,
                          file=SSTableFile.create(path=os.path.join(tmp, f"{t}.sst"), data=b""),
                          first_key=keys[0], last_key=keys[-1])

            def recorder(key, t=t):  # SSTable.get (src/sstable.py:175-187) of a table with no blocks
                calls.append(t)
                return None
            sst.get = recorder
            if lvl == 0:
                store.state.sstables_level0.append(sst)  # appended in newest-first order
            else:
                store.state.sstables_levels[lvl - 1].append(sst)
            tables.append({"level": lvl, "start": a, "stop": b, "step": step, "first_key": keys[0],
                           "last_key": keys[-1], "n_keys": len(keys), "nb_bytes": bf.nb_bytes,
                           "k": bf.nb_hash_functions, "popcount": bin(bf.bits).count("1"),
                           "sha256": hashlib.sha256(bm).hexdigest()})
        probes = universe[::7] + ["k%05d5" % i for i in range(0, 8000, 53)] + ["", "0", "zzz", "\U0001f600"]
        probes += ["x%d" % rng.randrange(10 ** 6) for _ in range(50)]
        order = []
        for key in probes:
            calls.clear()
            assert store.get(key=key) is None
            order.append(list(calls))
    assert len({t["nb_bytes"] for t in tables}) > 6  # the product sizing gives mixed sizes
    doc = {"generated_by": "tools/gen_golden_lsm.py (reference LsmStorage.get, src/lsm_storage.py:153-181)",
           "fp_rate": 0.001, "universe": universe, "tables": tables, "probes": probes, "order": order}
    with open(OUT, "w") as fh:
        json.dump(doc, fh, ensure_ascii=True, separators=(",", ":"))
    print(f"wrote {OUT}: {len(tables)} tables, {len(probes)} probes, "
          f"{sum(len(o) for o in order)} SSTable reads")


if __name__ == "__main__":
    main()
