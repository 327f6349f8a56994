"""Multi-GPU placement of independent SSTable filters.

Filters are independent (one per SSTable: src/sstable.py:274, built at flush
src/lsm_storage.py:200-205 and per output SSTable at compaction :238-249), so G GPUs simply
own disjoint sets of filters — no collective on the data path.  Probes (LsmStorage.get,
src/lsm_storage.py:164-179) replicate the key batch to every GPU that owns filters; each GPU
answers for its own filters and the host combines the per-filter hit masks in the reference's
order (L0 newest first, then each level's SSTables whose key range holds the key).
"""
from __future__ import annotations

import numpy as np


def filters_for_rank(n_filters: int, world: int, rank: int) -> list[int]:
    """Contiguous block partition of filter ids 0..n_filters-1 over `world` ranks."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_filters, world)
    start = rank * base + min(rank, extra)
    return list(range(start, start + base + (1 if rank < extra else 0)))


def owner_of(filter_id: int, n_filters: int, world: int) -> int:
    for r in range(world):
        if filter_id in filters_for_rank(n_filters, world, r):
            return r
    raise ValueError("filter id out of range")


def key_range(filter_id: int, keys_per_filter: int) -> tuple[int, int]:
    """Config-4 key assignment: filter g holds keys [g*K, (g+1)*K) of the global key stream."""
    return filter_id * keys_per_filter, (filter_id + 1) * keys_per_filter


def candidate_order(l0_hits: np.ndarray, level_hits: list[np.ndarray]) -> list[int]:
    """For ONE key: indices of the SSTables LsmStorage.get would read, in its order
    (lsm_storage.py:164-179) — L0 filters newest first, then each level's range-qualified
    filters — given per-filter may_contain results.  L0 entries are ids 0..len(l0)-1, level
    entries continue the numbering."""
    order = [i for i, h in enumerate(l0_hits) if h]
    off = len(l0_hits)
    for lvl in level_hits:
        order += [off + i for i, h in enumerate(lvl) if h]
        off += len(lvl)
    return order


def gather_hitmasks(per_filter: dict[int, np.ndarray], n_filters: int, n_keys: int) -> np.ndarray:
    """Stack per-filter LSB-first hit masks (from any ranks) into a bool matrix [filter, key]."""
    out = np.zeros((n_filters, n_keys), dtype=bool)
    for f, hm in per_filter.items():
        out[f] = np.unpackbits(np.asarray(hm, dtype=np.uint8), bitorder="little")[:n_keys].astype(bool)
    return out
