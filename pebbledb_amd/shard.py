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


def exchange_bitmaps(dist, torch, n_filters: int, nb_bytes: int, export, load, device: int | None = None) -> dict:
    """Give every rank every filter's bitmap, each built once by its owner (filters_for_rank):
    the key-partitioned multi-GPU probe holds all of an LSM's filters on every GPU, and pebbledb
    builds a filter once per SSTable (src/sstable.py:274, at flush src/lsm_storage.py:200-205)
    while every get probes all of them (src/lsm_storage.py:164-179) — so the others' filters
    arrive by replication, not by rebuilding.

    export(g, t): write the rank's own filter g's nb_bytes-byte bitmap into the uint8 tensor t;
    load(g, t): make filter g from t (another rank's).  With RCCL ('nccl') the tensors are on
    `device` and the exchange is ONE all-gather when every rank owns the same number of filters
    (8 filters over 1/2/4/8 GPUs), else one broadcast per filter from its owner; with gloo they
    are host tensors.  Returns {"bytes_received": ..., "collective": ...}.  One-time setup of the
    layout, never per step."""
    world, rank = dist.get_world_size(), dist.get_rank()
    on_dev = dist.get_backend() == "nccl"
    dev = torch.device("cuda", device) if on_dev else torch.device("cpu")
    owned = [filters_for_rank(n_filters, world, r) for r in range(world)]
    mine = owned[rank]
    if len({len(o) for o in owned}) == 1:
        c = len(mine)
        send = torch.empty(c * nb_bytes, dtype=torch.uint8, device=dev)
        for i, g in enumerate(mine):
            export(g, send[i * nb_bytes:(i + 1) * nb_bytes])
        recv = torch.empty(world * c * nb_bytes, dtype=torch.uint8, device=dev)
        if on_dev:
            dist.all_gather_into_tensor(recv, send)
        else:
            dist.all_gather(list(recv.chunk(world)), send)
        for r in range(world):
            if r == rank:
                continue
            for i, g in enumerate(owned[r]):
                o = (r * c + i) * nb_bytes
                load(g, recv[o:o + nb_bytes])
        return {"bytes_received": (world - 1) * c * nb_bytes,
                "collective": f"all_gather ({'RCCL' if on_dev else 'gloo'})"}
    buf = torch.empty(nb_bytes, dtype=torch.uint8, device=dev)
    got = 0
    for g in range(n_filters):
        src = owner_of(g, n_filters, world)
        if src == rank:
            export(g, buf)
        dist.broadcast(buf, src=src)
        if src != rank:
            load(g, buf.clone())
            got += nb_bytes
    return {"bytes_received": got, "collective": f"broadcast per filter ({'RCCL' if on_dev else 'gloo'})"}
