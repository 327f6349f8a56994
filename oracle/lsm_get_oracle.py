"""ORACLE — test infrastructure only (never imported by ``pebbledb_amd``).

Restatement of the filter stage of the reference's ``LsmStorage.get`` (src/lsm_storage.py:
153-179) for a list of keys: which SSTables it would read, in order, if none held the key.
The bloom decisions come from the C oracle's may_contain (oracle/bloom_oracle.c, itself pinned
by tests/golden); the key-range check is Python's own ``str`` comparison, exactly the
expression at lsm_storage.py:173.
"""
from __future__ import annotations

import numpy as np

from .oracle import COracle


def reference_candidates(keys: list[str], level0, levels) -> list[list[int]]:
    """level0: [(bitmap, k)] newest first; levels: [[(first_key, last_key, bitmap, k)]].
    Returns, per key, the SSTable numbers (L0 first, then level by level) in read order."""
    from pebbledb_amd.keys import PackedKeys  # the packed layout only (no device code)
    o = COracle()
    pk = PackedKeys.from_strs(keys)
    n = len(keys)

    def may_contain_all(bm, k):
        return np.unpackbits(o.probe(bm, k, pk), bitorder="little")[:n].astype(bool)

    l0_hits = [may_contain_all(bm, k) for bm, k in level0]
    lvl_hits = [[may_contain_all(bm, k) for _, _, bm, k in lvl] for lvl in levels]
    out = []
    for i, key in enumerate(keys):
        order = []
        for t in range(len(level0)):                      # lsm_storage.py:164-169
            if not l0_hits[t][i]:
                continue
            order.append(t)
        num = len(level0)
        for li, level in enumerate(levels):                # lsm_storage.py:171-178
            for j, (first_key, last_key, _, _) in enumerate(level):
                t = num + j
                if not first_key <= key <= last_key:
                    continue
                if not lvl_hits[li][j][i]:
                    continue
                order.append(t)
            num += len(level)
        out.append(order)
    return out
