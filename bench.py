"""Benchmark: device-resident bloom build + probe (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3|c4|c5|sst] [--no-cpu-baseline]

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N ranks itself (one
child process per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, 127.0.0.1 rendezvous) before
anything touches a GPU, and exits with the worst child exit code; under torch.distributed.run
it is one of the ranks.  WORLD_SIZE != --gpus is an error.  --dry-run exercises only that
launcher and the rendezvous / barrier / max-over-ranks plumbing (gloo, no GPU, no numbers).

Config c2 (default, BASELINE.json configs[1]): per GPU one SSTable filter of m = 2^30 bits
(nb_bytes = 128 MiB), k = 6, built from 10M 16-byte keys, then probed with 20M keys (the 10M
members + 10M non-members).  A step = clear + build (10M keys) + probe (20M keys), all on the
filter's HIP stream, keys already resident in HBM.  Ranks hold independent filters over
disjoint key ranges (weak scaling, no collective on the data path: SURVEY.md §8e).

value = (build keys + probe keys) summed over ranks / max-over-ranks wall time, in Mkeys/s.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
# per-pass HBM bytes from rocprofv3 PMC passes of this same bench (tools/traffic_summary.py);
# used only when it was measured on the very kernel sources this run was built from
TRAFFIC_FILE = os.path.join(REPO, "profiles", "traffic_{config}.json")

CONFIGS = {
    # name: (n_build, nb_bytes, k, key kind)
    "c1": (1000, 1024, 4, "hex16"),
    "c2": (10_000_000, 2 ** 27, 6, "hex16"),
    "c3": (100_000_000, 2 ** 30, 8, "varlen"),
}
SEED = 0x5EEDB100
SEED_VAR = 0xC3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS) + ["c4", "c5", "c5mixed", "sst"])
    ap.add_argument("--c4-keys", type=int, default=125_000_000, help="c4: keys per filter (reference 125M)")
    ap.add_argument("--c5-probes", type=int, default=100_000_000, help="c5: probe keys (reference 100M)")
    ap.add_argument("--build-mode", type=int, default=0, help="0 auto, 1 atomic, 2 tiled")
    ap.add_argument("--probe-mode", type=int, default=0, help="0 auto, 1 direct, 2 tiled")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-events", action="store_true", help="diagnostic: time without per-step HIP events")
    ap.add_argument("--no-host-inclusive", action="store_true", help="skip the pinned host<->device leg")
    ap.add_argument("--sync-each-step", action="store_true", help="diagnostic: synchronise after every step")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the bounded CPU sample")
    ap.add_argument("--no-host-c5", action="store_true", help="c5: skip the host-resident (pinned H2D) leg")
    ap.add_argument("--no-compare", action="store_true",
                    help="c5: skip the per-filter comparison leg (PMC passes of the fused probe alone)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rendezvous check only (gloo, no GPU work, no measurement)")
    ap.add_argument("--c5-layout", default="keys", choices=["keys", "filters"],
                    help="c5 over N ranks: 'keys' = every rank holds the 8 filters and probes 1/N of the batch "
                         "through the fused path; 'filters' = 8/N filters per rank, the whole batch each")
    ap.add_argument("--sim-world", type=int, default=1,
                    help="c4/c5 on one GPU: run rank --sim-rank's share of a --sim-world-rank job (its filters, "
                         "its keys), no process group; the JSON reports that rank's rate")
    ap.add_argument("--sim-rank", type=int, default=0)
    return ap.parse_args()


def rank_plan(config: str, world: int, rank: int, local: int, c4_keys: int = 125_000_000,
              c5_probes: int = 100_000_000, c5_layout: str = "keys") -> dict:
    """What rank `rank` of `world` does (no GPU needed; tests/test_bench_launch_cpu.py checks the
    8-rank plans): its device (LOCAL_RANK), its filters and key ranges.

    c2 / c3: one filter per rank over the rank's own keys (weak scaling).
    c4: filters_for_rank(8, world, rank); filter g is built from keys [g*K, (g+1)*K) (K = 125M:
        1B keys over the 8 filters, shard.key_range).
    c5: 'keys' layout — every rank holds all 8 filters (1 GiB of bitmaps) and probes its 1/world
        slice of the 100M-key batch (whole 64-key hit-mask words) through the fused multi-filter
        path; it builds only filters_for_rank(8, world, rank) (`builds`) and receives the others
        once by replication (shard.exchange_bitmaps: an all-gather, before timing);
        'filters' layout — filters_for_rank(8, world, rank) against the whole batch.  No
        collective on the data path in either: the slices / filters are independent."""
    from pebbledb_amd.shard import filters_for_rank, key_range
    plan = {"rank": rank, "world": world, "device": local}
    if config == "c4":
        fl = filters_for_rank(8, world, rank)
        plan.update(filters=fl, key_ranges={g: key_range(g, c4_keys) for g in fl})
    elif config == "c5":
        if c5_layout == "keys":
            words = (c5_probes + 63) // 64
            a = min(c5_probes, (words * rank // world) * 64)
            b = min(c5_probes, (words * (rank + 1) // world) * 64)
            # the rank builds its own share of the filters once; the rest arrive by replication
            plan.update(filters=list(range(8)), builds=filters_for_rank(8, world, rank), probe_keys=(a, b),
                        layout="keys")
        else:
            fl = filters_for_rank(8, world, rank)
            plan.update(filters=fl, builds=fl, probe_keys=(0, c5_probes), layout="filters")
    else:
        plan.update(filters=[rank])
    return plan


def c5_probe_key_spans(nq: int, n_f: int, a: int, b: int):
    """The generator spans of probe keys [a, b) of C5's batch: (dst index, splitmix start, count).
    Keys [0, nq/2) are members, 1/8 from each filter's key range; the rest are absent keys
    (splitmix indices from 8 * n_f)."""
    half = nq // 2
    per = half // 8
    spans = []
    for g in range(8):
        lo, hi = g * per, (g * per + (per if g < 7 else half - 7 * per))
        x, y = max(a, lo), min(b, hi)
        if x < y:
            spans.append((x - a, g * n_f + (x - lo), y - x))
    x, y = max(a, half), b
    if x < y:
        spans.append((x - a, 8 * n_f + (x - half), y - x))
    return spans


def init_process_group_or_exit(dist, torch, backend: str, local: int, rank: int) -> None:
    """The timing's process group.  RCCL ('nccl') must come up or the run fails with exit code 3
    (never silently timed over another backend); gloo only when asked for (the one-GPU rehearsal)."""
    if backend == "nccl":
        try:
            dist.init_process_group(backend="nccl", init_method="env://", device_id=torch.device("cuda", local))
        except Exception as e:  # noqa: BLE001 - reported, then a non-zero exit
            print(f"rank {rank}: RCCL process group failed ({e!r}); set PBF_BENCH_BACKEND=gloo for a "
                  f"gloo-timed rehearsal", file=sys.stderr)
            sys.exit(3)
    else:
        dist.init_process_group(backend=backend, init_method="env://")


def algorithmic_bytes(n, L, k, m_bits, offsets):
    """build = n·L + 8·n·k + m/8 (+8n offsets); probe = n·L + 4·n·k + n/8."""
    build = n * L + 8 * n * k + m_bits // 8 + (8 * n if offsets else 0)
    return build


def probe_bytes(n, L, k, offsets):
    return n * L + 4 * n * k + n // 8 + (8 * n if offsets else 0)


def measured_traffic(config: str) -> dict | None:
    """{"build": bytes, "probe": bytes, "source": ...} from the committed PMC summary, or None
    when there is none for this config or it was taken on other kernel sources."""
    from pebbledb_amd.build import source_digest
    path = TRAFFIC_FILE.format(config=config)
    if not os.path.exists(path) or os.environ.get("PBF_LIB"):
        return None
    t = json.load(open(path))
    if t.get("source_sha256") != source_digest():
        return None
    out = {p: v["traffic_bytes"] for p, v in t["passes"].items()}
    out["source"] = os.path.relpath(path, REPO) + ": " + t["source"] + "; " + t["correction"]
    return out


def cpu_baseline(nb_bytes, k, kind, budget_s):
    """The reference algorithm as the reference runs it (oracle/oracle.py BigIntBloomPort: one
    Python big-int bitmap, `bits |= 1 << idx` per hashed bit) on the SAME filter size, timed on
    a bounded sample of the workload's keys; plus the C oracle on all host cores."""
    import numpy as np

    from oracle.oracle import BigIntBloomPort, COracle
    from pebbledb_amd.keys import PackedKeys, splitmix_hex_keys, splitmix_hex_keys_str, varlen_keys_str

    strs = (splitmix_hex_keys_str(SEED, 0, 64) if kind == "hex16" else varlen_keys_str(SEED_VAR, 0, 64))
    port = BigIntBloomPort(nb_bytes, k)
    t0 = time.perf_counter()
    nb = 0
    while nb < len(strs) and time.perf_counter() - t0 < budget_s / 2:
        port.add(strs[nb])
        nb += 1
    t_build = time.perf_counter() - t0
    t0 = time.perf_counter()
    npb = 0
    while npb < len(strs) and time.perf_counter() - t0 < budget_s / 2:
        port.may_contain(strs[npb] if npb % 2 == 0 else strs[npb] + "x")
        npb += 1
    t_probe = time.perf_counter() - t0
    # the workload's mix is 1 build key : 2 probe keys → keys/s = 3 / (t_add + 2·t_probe)
    tb, tp = t_build / max(nb, 1), t_probe / max(npb, 1)
    rate = 3.0 / (tb + 2.0 * tp) if nb and npb else 0.0
    # fair native number: the C oracle with OpenMP on every host core, 2M keys
    o = COracle()
    n_c = 2_000_000
    pk = PackedKeys.fixed(splitmix_hex_keys(SEED, 0, n_c))
    q = PackedKeys.fixed(splitmix_hex_keys(SEED, 0, 2 * n_c))
    t0 = time.perf_counter()
    bm = o.build(nb_bytes, k, pk, omp=True)
    o.probe(bm, k, q, omp=True)
    t_c = time.perf_counter() - t0
    return {
        "value": rate / 1e6,
        "unit": "Mkeys/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"reference algorithm (Python big-int bitmap, oracle/oracle.py BigIntBloomPort) on the "
                   f"full-size filter nb_bytes={nb_bytes}, k={k}: {nb} build keys in {t_build:.2f}s + {npb} probes "
                   f"in {t_probe:.2f}s; rate = 3/(t_add + 2*t_probe), the step's 1:2 build:probe mix"),
        "build_s_per_key": t_build / max(nb, 1),
        "probe_s_per_key": t_probe / max(npb, 1),
        "c_oracle_omp": {"value": 3 * n_c / t_c / 1e6, "unit": "Mkeys/s", "cores": o.num_threads(),
                         "sample": f"{n_c} builds + {2 * n_c} probes, same filter size"},
    }


def host_inclusive(bf, keys, n, nb_bytes, L, torch, np, reps=3):
    """The path as the reference runs it: keys start in host memory (flush / compaction
    iterator) and the bitmap ends in host memory (the SSTable file buffer).  Pinned host
    buffers, hipMemcpyAsync H2D of the packed keys, build, D2H of the bitmap; and H2D of the
    probe keys, probe, D2H of the hit mask.  Also the Python str → packed-bytes cost."""
    import ctypes
    from pebbledb_amd import _native
    from pebbledb_amd.keys import PackedKeys, splitmix_hex_keys_str

    hk = keys[: 2 * n * 16].cpu().pin_memory()
    hbm = torch.empty(nb_bytes, dtype=torch.uint8).pin_memory()
    hhm = torch.empty((2 * n + 7) // 8, dtype=torch.uint8).pin_memory()
    vp = ctypes.c_void_p
    tb, tp = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        bf.clear()
        _native.check(L.pbf_add_fixed(bf.handle, vp(hk.data_ptr()), 16, n, 0), "add")
        _native.check(L.pbf_get_bitmap(bf.handle, vp(hbm.data_ptr()), nb_bytes), "get_bitmap")
        t1 = time.perf_counter()
        _native.check(L.pbf_probe_fixed(bf.handle, vp(hk.data_ptr()), 16, 2 * n, vp(hhm.data_ptr()), 0), "probe")
        t2 = time.perf_counter()
        tb.append(t1 - t0)
        tp.append(t2 - t1)
    build_ms, probe_ms = min(tb) * 1e3, min(tp) * 1e3
    ok = bool((np.unpackbits(hhm[: n // 8].numpy(), bitorder="little") == 1).all())
    strs = splitmix_hex_keys_str(SEED, 0, 1_000_000)
    t0 = time.perf_counter()
    PackedKeys.from_strs(strs)
    pack_s = time.perf_counter() - t0
    return {
        "build_ms": round(build_ms, 3),
        "probe_ms": round(probe_ms, 3),
        "build_Mkeys_s": round(n / build_ms / 1e3, 1),
        "probe_Mkeys_s": round(2 * n / probe_ms / 1e3, 1),
        "step_Mkeys_s": round(3 * n / (build_ms + probe_ms) / 1e3, 1),
        "what": "pinned host keys -> H2D -> build -> D2H bitmap (128 MiB); pinned host probe keys -> H2D -> "
                "probe -> D2H hit mask; best of 3",
        "members_all_hit": ok,
        "py_str_packing_Mkeys_s": round(1.0 / pack_s, 2),
    }


def dropin_latency(device, reps=2000):
    """Per-call latency of the drop-in class at C1 size (BASELINE configs[0]: 1k 16-B keys,
    m = 8192, k = 4) as pebbledb calls it — add per key then a read (SSTableBuilder.build,
    sstable.py:274), may_contain per key (LsmStorage.get, lsm_storage.py:165,175), to_bytes
    (sstable.py:82) — beside the reference algorithm (BigIntBloomPort, Python big-int bitmap)."""
    from oracle.oracle import BigIntBloomPort
    from pebbledb_amd import BloomFilter
    from pebbledb_amd.keys import splitmix_hex_keys_str
    keys = splitmix_hex_keys_str(SEED, 0, 1000)
    probes = splitmix_hex_keys_str(SEED, 500, 1000)
    out = {}
    for name, cls in (("pebbledb_amd", BloomFilter), ("reference_port", BigIntBloomPort)):
        kw = {"device": device} if cls is BloomFilter else {}
        bf = cls(1024, 4, **kw)
        t0 = time.perf_counter()
        for k in keys:
            bf.add(k)
        blob = bf.to_bytes()  # the first read sends the buffered adds (one batched build)
        t_add = time.perf_counter() - t0
        for k in probes[:50]:
            bf.may_contain(k)
        st0 = _resident_stats(device) if cls is BloomFilter else None
        t0 = time.perf_counter()
        hits = 0
        for i in range(reps):
            hits += bf.may_contain(probes[i % 1000])
        t_mc = time.perf_counter() - t0
        st1 = _resident_stats(device) if cls is BloomFilter else None
        t0 = time.perf_counter()
        for _ in range(200):
            blob = bf.to_bytes()
        t_tb = time.perf_counter() - t0
        t0 = time.perf_counter()
        for _ in range(20):
            cls.build_from_keys_and_fp_rate(keys, 0.001, **kw) if cls is BloomFilter else None
        t_bk = time.perf_counter() - t0
        out[name] = {"add_us_per_key_incl_flush": round(t_add / 1000 * 1e6, 2),
                     "may_contain_us": round(t_mc / reps * 1e6, 2), "to_bytes_us": round(t_tb / 200 * 1e6, 2),
                     "hits": hits, "bitmap_sha16": __import__("hashlib").sha256(blob).hexdigest()[:16]}
        if cls is BloomFilter:
            out[name]["build_from_keys_1k_us"] = round(t_bk / 20 * 1e6, 1)
            # of the call's time, the resident wave's own (request seen -> answer written)
            out[name]["may_contain_device_us"] = round((st1[1] - st0[1]) * 1e-3 / max(1, st1[0] - st0[0]), 2)
            # where the per-key time goes: the same calls with a launch per key (the resident
            # reader off)
            L = _native_lib()
            L.pbf_resident_enable(0)
            try:
                for k in probes[:50]:
                    bf.may_contain(k)
                t0 = time.perf_counter()
                hits_l = sum(bf.may_contain(probes[i % 1000]) for i in range(reps))
                out[name]["may_contain_launch_us"] = round((time.perf_counter() - t0) / reps * 1e6, 2)
                out[name]["launch_hits_equal"] = hits_l == hits
            finally:
                L.pbf_resident_enable(1)

    out["identical"] = (out["pebbledb_amd"]["bitmap_sha16"] == out["reference_port"]["bitmap_sha16"]
                        and out["pebbledb_amd"]["hits"] == out["reference_port"]["hits"])
    out["get_16_filters"] = get_set_latency(device)
    out["reader_threads"] = reader_threads(device)
    out["batch_probe_with_gets"] = probe_with_gets(device)
    return out


def probe_with_gets(device, reps=20):
    """A batched C2 probe (20M keys against a 128 MiB filter, the tiled pipeline) alone and while
    another thread issues per-key may_contain calls on a small L0 filter (LsmStorage.get traffic
    beside a batch: the resident reader wave holds a CU slot while keys arrive, and the
    partition's workgroups each take a whole CU).  Hit masks must be identical."""
    import threading

    import numpy as np
    import torch
    from pebbledb_amd import BloomFilter, _native
    from pebbledb_amd.keys import splitmix_hex_keys_str
    L = _native.lib()
    n = 10_000_000
    keys = torch.empty(2 * n * 16, dtype=torch.uint8, device=f"cuda:{device}")
    _native.check(L.pbf_gen_splitmix_hex(device, None, keys.data_ptr(), SEED, 0, 2 * n), "gen")
    big = BloomFilter(2 ** 27, 6, device=device)
    big.add_device_fixed(keys.data_ptr(), 16, n)
    hm = torch.zeros(2 * n // 8, dtype=torch.uint8, device=f"cuda:{device}")
    small = BloomFilter.build_from_keys_and_fp_rate(splitmix_hex_keys_str(SEED, 0, 100_000), 0.001, device=device)
    probes = splitmix_hex_keys_str(SEED, 50_000, 1000)
    big.sync()

    st = torch.cuda.ExternalStream(big.stream)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(reps)]

    def batch():
        # wall time per probe, and the probes' own GPU time (HIP events around each on the
        # filter's stream: host-side delays between enqueues do not count there)
        t0 = time.perf_counter()
        for e in ev:
            e[0].record(st)
            big.probe_device_fixed(keys.data_ptr(), 16, 2 * n, hm.data_ptr())
            e[1].record(st)
        big.sync()
        wall = (time.perf_counter() - t0) / reps * 1e3
        return wall, sum(e[0].elapsed_time(e[1]) for e in ev) / reps

    batch()
    alone = batch()
    ref = hm.cpu().numpy().copy()
    stop = threading.Event()
    calls = [0]

    def gets():
        i = 0
        while not stop.is_set():
            small.may_contain(probes[i % 1000])
            i += 1
        calls[0] = i
    th = threading.Thread(target=gets)
    th.start()
    time.sleep(0.01)
    t0 = time.perf_counter()
    with_gets = batch()
    dt = time.perf_counter() - t0
    stop.set()
    th.join()
    return {"probe_ms_alone": round(alone[1], 4), "probe_ms_with_gets": round(with_gets[1], 4),
            "wall_ms_per_probe_alone": round(alone[0], 4), "wall_ms_per_probe_with_gets": round(with_gets[0], 4),
            "gets_per_s_during": round(calls[0] / max(dt, 1e-9)),
            "identical": bool(np.array_equal(ref, hm.cpu().numpy()))}


def _native_lib():
    from pebbledb_amd import _native
    return _native.lib()


def _resident_stats(device):
    """(requests answered, their device nanoseconds) of the device's resident reader so far."""
    r, d = ctypes.c_uint64(), ctypes.c_uint64()
    _native_lib().pbf_resident_stats(device, ctypes.byref(r), ctypes.byref(d))
    return r.value, d.value


def get_set_latency(device, reps=1000):
    """One LsmStorage.get's bloom checks (src/lsm_storage.py:164-179) over 10 L0 + 6 level SSTable
    filters of 16 different sizes (product sizing, sstable.py:274: 20k..170k keys, k = 10): one
    pbf_may_contain_set call (lsm_get.candidates_one; answered by the resident reader, and with it
    off by one k_may_contain_set launch) vs 16 may_contain calls; the answers must be identical."""
    from pebbledb_amd import BloomFilter
    from pebbledb_amd.keys import splitmix_hex_keys_str
    from pebbledb_amd.lsm_get import LevelTable, candidates_one
    ns = [20_000 + 10_000 * i for i in range(16)]
    tables, start = [], 0
    for n in ns:
        keys = sorted(splitmix_hex_keys_str(SEED, start, n))
        tables.append((keys[0], keys[-1], BloomFilter.build_from_keys_and_fp_rate(keys, 0.001, device=device)))
        start += n
    l0 = [bf for _, _, bf in tables[:10]]
    levels = [[LevelTable("", "\U0010ffff", bf) for _, _, bf in tables[10:]]]  # ranges that hold every probe
    flat = l0 + [t.bloom_filter for t in levels[0]]
    probes = splitmix_hex_keys_str(SEED, start - 500, 1000)  # 500 members of the last table, 500 absent
    for key in probes[:50]:
        candidates_one(key, l0, levels)
    st0 = _resident_stats(device)
    t0 = time.perf_counter()
    one = [candidates_one(probes[i % 1000], l0, levels) for i in range(reps)]
    t_set = time.perf_counter() - t0
    st1 = _resident_stats(device)
    t0 = time.perf_counter()
    loop = [[t for t, bf in enumerate(flat) if bf.may_contain(probes[i % 1000])] for i in range(reps)]
    t_loop = time.perf_counter() - t0
    L = _native_lib()
    L.pbf_resident_enable(0)  # the same gets with one k_may_contain_set launch each
    try:
        for key in probes[:50]:
            candidates_one(key, l0, levels)
        t0 = time.perf_counter()
        launched = [candidates_one(probes[i % 1000], l0, levels) for i in range(reps)]
        t_launch = time.perf_counter() - t0
    finally:
        L.pbf_resident_enable(1)
    return {"filters": len(flat), "nb_bytes": [bf.nb_bytes for bf in flat],
            "one_call_us_per_get": round(t_set / reps * 1e6, 2),
            "one_call_device_us": round((st1[1] - st0[1]) * 1e-3 / max(1, st1[0] - st0[0]), 2),
            "one_launch_us_per_get": round(t_launch / reps * 1e6, 2),
            "may_contain_x16_us_per_get": round(t_loop / reps * 1e6, 2),
            "identical": one == loop == launched}


def reader_threads(device, calls=4000):
    """Concurrent LsmStorage.get readers (src/lsm_storage.py:153-179: any thread probes a
    published filter, no lock) on ONE L0 filter (product sizing, sstable.py:274, 100k keys,
    k = 10): T threads share `calls` may_contain calls; aggregate calls/s for T = 1, 2, 4, 8 and
    whether every answer equals the single-thread answers.  One-key probes hold the handle's lock
    shared and run on per-thread reader streams; PBF_SHARED_READERS=0 (set before the library
    loads) measures the exclusive path."""
    import threading
    from pebbledb_amd import BloomFilter
    from pebbledb_amd.keys import splitmix_hex_keys_str
    keys = splitmix_hex_keys_str(SEED, 0, 100_000)
    bf = BloomFilter.build_from_keys_and_fp_rate(keys, 0.001, device=device)
    probes = splitmix_hex_keys_str(SEED, 50_000, 2000)
    want = [bf.may_contain(p) for p in probes]
    out = {"filter_nb_bytes": bf.nb_bytes, "k": bf.nb_hash_functions,
           "shared_readers": os.environ.get("PBF_SHARED_READERS", "1") != "0"}
    ok = True
    for T in (1, 2, 4, 8):
        res = [None] * T
        per = calls // T
        start = threading.Barrier(T + 1)

        def run(t):
            start.wait()
            res[t] = [bf.may_contain(probes[(t * per + i) % 2000]) for i in range(per)]

        th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
        for t in th:
            t.start()
        start.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        for t in range(T):
            ok &= res[t] == [want[(t * per + i) % 2000] for i in range(per)]
        out[f"threads_{T}_calls_per_s"] = round(T * per / dt)
    out["identical"] = bool(ok)
    return out


def all_reduce_scalar(torch, dist, value, op, dtype):
    """max / min of a scalar over ranks (RCCL: a device tensor; gloo rehearsal: a host one)."""
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=dtype, device=dev)
    dist.all_reduce(t, op=op)
    return t.item()


def c5_host_resident(args, filters, mine, hms, q, nq, k, torch, np, L, reps=2):
    """BASELINE configs[4] as LsmStorage.get batching would run it (src/lsm_storage.py:164-179):
    the probe batch starts in (pinned) host memory, every GPU copies its own replica in
    (per-GPU H2D, pbf_probe_multi with keys_on_device = 0: 256 MiB pinned chunks), probes its
    filters and the hit masks return to host memory.  Rate = key x filter probes / wall time."""
    import ctypes
    from pebbledb_amd import _native
    hq = q.cpu().pin_memory()
    outs_np = [np.zeros((nq + 7) // 8, dtype=np.uint8) for _ in mine]
    hs = (ctypes.c_void_p * len(mine))(*[filters[g].handle.value for g in mine])
    outs = (ctypes.c_void_p * len(mine))(*[a.ctypes.data for a in outs_np])
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _native.check(L.pbf_probe_multi_fixed(hs, len(mine), ctypes.c_void_p(hq.data_ptr()), 16, nq, outs, 0),
                      "probe_multi host")
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    same = all(np.array_equal(outs_np[i], hms[g].cpu().numpy()) for i, g in enumerate(mine))
    return {"ms": round(t * 1e3, 2), "Mprobes_s": round(nq * len(mine) / t / 1e6, 1),
            "h2d_GBs": round(nq * 16 / t / 1e9, 2), "equal_to_device_resident": bool(same),
            "what": f"pinned host batch of {nq} 16-B keys -> per-GPU H2D (256 MiB chunks) -> multi-filter probe of "
                    f"the rank's {len(mine)} filters -> D2H hit masks; best of {reps}"}


def c5_cpu_baseline(args, filters, mine, hms, q, n_f, nb_bytes, k, np):
    """C5's CPU baseline (rank 0, N = 1): the reference algorithm (BigIntBloomPort, Python
    big-int bitmap) probing filter 0 at full size on a bounded sample, plus the C oracle
    (OpenMP) probing a 1M-key sample against filter 0 — whose result must equal the GPU's."""
    from oracle.oracle import BigIntBloomPort, COracle
    from pebbledb_amd.keys import PackedKeys, splitmix_hex_keys
    g = mine[0]
    o = COracle()
    t0 = time.perf_counter()
    want = o.build(nb_bytes, k, PackedKeys.fixed(splitmix_hex_keys(SEED, g * n_f, n_f)), omp=True)
    t_build = time.perf_counter() - t0
    ns = 1_000_000
    a = (len(q) // 16) // 2 - ns // 2
    a -= a % 8
    qs = PackedKeys.fixed(q[a * 16:(a + ns) * 16].cpu().numpy().reshape(-1, 16))
    t0 = time.perf_counter()
    hm = o.probe(want, k, qs, omp=True)
    t_probe = time.perf_counter() - t0
    gpu = hms[g].cpu().numpy()[a // 8:(a + ns) // 8]
    # the reference's own algorithm on the full-size filter (each probe ANDs a 1<<idx big-int
    # against the 2^30-bit int): a handful of probes in the budget
    port = BigIntBloomPort(nb_bytes, k, bits=int.from_bytes(want.tobytes(), "little"))
    t0 = time.perf_counter()
    npb = 0
    while time.perf_counter() - t0 < min(args.cpu_seconds, 8.0):
        port.may_contain(qs.key(npb % ns).decode())
        npb += 1
    t_port = time.perf_counter() - t0
    return {"value": round(npb / t_port / 1e6, 9), "unit": "Mprobes/s", "cores": 1, "kind": "port",
            "sample": f"reference algorithm (BigIntBloomPort, Python big-int bitmap of 2^30 bits) probing filter {g}: "
                      f"{npb} keys in {t_port:.1f}s",
            "c_oracle_omp": {"value": round(ns / t_probe / 1e6, 2), "unit": "Mprobes/s", "cores": o.num_threads(),
                             "sample": f"{ns} probes vs filter {g} (build of its {n_f} keys: {t_build:.2f}s)"},
            "oracle_sample_equal": bool(np.array_equal(gpu, hm))}


def sets_main(args, rank, world, local, torch, dist, np):
    """Configs 4 and 5: eight independent SSTable filters spread over the ranks (8/N each,
    shard.filters_for_rank), no collective on the data path.

    c4 — BASELINE.json configs[3]: 1B 16-B keys, filter g built from keys [g*125M, (g+1)*125M)
         with pebbledb's product sizing (sstable.py:274, fp_rate 0.001 → nb_bytes 224,649,806,
         k = 10, a non-power-of-two m).  A step = clear + build of every filter the rank owns.
         value = keys built per step over all ranks / step time (strong scaling: 1B keys total).
    c5 — configs[4]: filters as C2 (m = 2^30, k = 6, 10M keys each, built before timing); 100M
         probe keys (half members, 1/8 from each filter's range; half absent) replicated to every
         rank.  A step = one multi-filter probe (pbf_probe_multi) of the batch against the
         rank's filters.  value = key x filter probes per step over all ranks / step time."""
    from math import ceil, log

    from pebbledb_amd import BloomFilter, _native, probe_multi_device
    from pebbledb_amd.bloom_filter import set_default_device
    from pebbledb_amd.shard import filters_for_rank

    set_default_device(local)
    L = _native.lib()
    # the rank's share (rank_plan); --sim-world W --sim-rank R runs rank R's share of a W-rank job
    # on this one GPU, without a process group
    sim = args.sim_world > 1
    plan = rank_plan(args.config, args.sim_world if sim else world, args.sim_rank if sim else rank, local,
                     args.c4_keys, args.c5_probes, args.c5_layout)
    mine = plan["filters"]
    if args.config == "c4":
        n = args.c4_keys
        p = 0.001
        m = (-n * log(p)) / (log(2) ** 2)  # bloom_filter.py:109-114, same expression order
        nb_bytes, k = ceil(m / 8), round((m / n) * log(2))
        keys = {}
        for g in mine:
            keys[g] = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
            _native.check(L.pbf_gen_splitmix_hex(local, None, keys[g].data_ptr(), SEED, g * n, n), "gen")
        filters = {g: BloomFilter(nb_bytes, k, device=local) for g in mine}
        s0 = filters[mine[0]]
        stream = torch.cuda.ExternalStream(s0.stream)
        torch.cuda.synchronize()

        def step(ev=None):
            for i, g in enumerate(mine):
                bf = filters[g]
                if ev is not None:
                    ev[i][0].record(torch.cuda.ExternalStream(bf.stream))
                bf.clear()
                bf.add_device_fixed(keys[g].data_ptr(), 16, n)
                if ev is not None:
                    ev[i][1].record(torch.cuda.ExternalStream(bf.stream))
        unit_total = n * (len(mine) if sim else 8)  # every rank builds its share of the 8 filters per step
    else:
        n_f = 10_000_000
        nb_bytes, k = 2 ** 27, 6
        nq_all = args.c5_probes
        qa, qb = plan["probe_keys"]  # this rank's slice of the batch
        nq = qb - qa
        filters = {}
        kb = torch.empty(n_f * 16, dtype=torch.uint8, device="cuda")

        def build_filter(g):
            _native.check(L.pbf_gen_splitmix_hex(local, None, kb.data_ptr(), SEED, g * n_f, n_f), "gen")
            torch.cuda.synchronize()
            bf = BloomFilter(nb_bytes, k, device=local)
            bf.add_device_fixed(kb.data_ptr(), 16, n_f)
            bf.sync()
            return bf
        # Each filter is built ONCE, by its owner (filters_for_rank): in the key-partitioned layout
        # the other ranks' filters arrive by replication (pebbledb builds a filter per SSTable,
        # src/sstable.py:274, and every get probes all of them, src/lsm_storage.py:164-179)
        own = plan["builds"]
        replicated = own != mine
        for g in own:
            filters[g] = build_filter(g)
        replication = None
        if replicated and sim:
            # one GPU: the other ranks' filters are built here as stand-ins (untimed), then copied
            # into this rank's set with pbf_copy_filter (same device; across GPUs of one process
            # it is a peer copy over xGMI)
            stand = {g: build_filter(g) for g in mine if g not in filters}
            torch.cuda.synchronize()
            t_r = time.perf_counter()
            for g, bf in stand.items():
                filters[g] = bf.replicate(local)
            replicate_ms = (time.perf_counter() - t_r) * 1e3
            del stand
            replication = {"replicate_ms": round(replicate_ms, 3), "filters_received": len(mine) - len(own),
                           "how": "pbf_copy_filter on this GPU (simulated rank; the real job all-gathers over RCCL)"}
        elif replicated:
            from pebbledb_amd.shard import exchange_bitmaps
            on_dev = dist.get_backend() == "nccl"

            def export(g, t):
                if on_dev:
                    filters[g].bitmap_to_device(t.data_ptr())
                    filters[g].sync()
                else:
                    t.copy_(torch.frombuffer(bytearray(filters[g].bitmap()), dtype=torch.uint8))

            def load(g, t):
                if on_dev:
                    filters[g] = BloomFilter.from_device_bitmap(t.data_ptr(), nb_bytes, k, device=local,
                                                                stream=torch.cuda.current_stream().cuda_stream)
                else:
                    filters[g] = BloomFilter.from_bytes(t.numpy().tobytes() + bytes([k]), device=local)
                filters[g].sync()
            dist.barrier()
            torch.cuda.synchronize()
            t_r = time.perf_counter()
            info = exchange_bitmaps(dist, torch, 8, nb_bytes, export, load, device=local)
            torch.cuda.synchronize()
            replicate_ms = (time.perf_counter() - t_r) * 1e3
            replicate_ms = float(all_reduce_scalar(torch, dist, replicate_ms, dist.ReduceOp.MAX, torch.float64))
            replication = {"replicate_ms": round(replicate_ms, 3), "filters_received": len(mine) - len(own),
                           "bytes_received_per_rank": info["bytes_received"], "how": info["collective"]}
        del kb
        q = torch.empty(max(nq, 1) * 16, dtype=torch.uint8, device="cuda")
        half = nq_all // 2
        per = half // 8
        # members: 1/8 of the batch's first half from each filter's range; then absent keys
        for dst, start, cnt in c5_probe_key_spans(nq_all, n_f, qa, qb):
            _native.check(L.pbf_gen_splitmix_hex(local, None, q.data_ptr() + dst * 16, SEED, start, cnt), "gen")
        hms = {g: torch.zeros((nq + 7) // 8, dtype=torch.uint8, device="cuda") for g in mine}
        fl = [filters[g] for g in mine]
        s0 = fl[0]
        stream = torch.cuda.ExternalStream(s0.stream)
        torch.cuda.synchronize()

        def step(ev=None):
            if ev is not None:
                ev[0][0].record(stream)
            probe_multi_device(fl, q.data_ptr(), nq, [hms[g].data_ptr() for g in mine], key_len=16)
            if ev is not None:
                ev[0][1].record(stream)
        # key x filter probes per step over all ranks (a simulated rank: its own share)
        unit_total = nq * len(mine) if sim else nq_all * 8

    nev = len(mine) if args.config == "c4" else 1
    events = [[[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(nev)] for _ in range(args.steps)]
    for _ in range(args.warmup):
        step()
    for bf in filters.values():
        bf.sync()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for st in range(args.steps):
        step(events[st])
    for bf in filters.values():
        bf.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    pass_ms = sum(e[i][0].elapsed_time(e[i][1]) for e in events for i in range(nev)) / (args.steps * nev)
    # correctness on the measured state
    ok = True
    fp_rate = None
    if args.config == "c4":
        g = mine[0]
        bf = filters[g]
        hm = torch.zeros((n + 7) // 8, dtype=torch.uint8, device="cuda")
        bf.probe_device_fixed(keys[g].data_ptr(), 16, n, hm.data_ptr())
        bf.sync()
        ok = bool((np.unpackbits(hm.cpu().numpy(), bitorder="little")[:n] == 1).all())
        absent = torch.empty(1_000_000 * 16, dtype=torch.uint8, device="cuda")
        _native.check(L.pbf_gen_splitmix_hex(local, None, absent.data_ptr(), SEED, 8 * n, 1_000_000), "gen")
        hm2 = torch.zeros(125_000, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        bf.probe_device_fixed(absent.data_ptr(), 16, 1_000_000, hm2.data_ptr())
        bf.sync()
        fp_rate = float(np.unpackbits(hm2.cpu().numpy()).sum()) / 1e6
    else:
        fp_total, fp_expect = 0, 0.0
        n_abs = max(0, qb - max(qa, half))  # the rank's absent keys
        for g in mine:
            bits = np.unpackbits(hms[g].cpu().numpy(), bitorder="little")[:nq]
            cnt = per if g < 7 else half - 7 * per
            lo, hi = max(qa, g * per), min(qb, g * per + cnt)  # g's members in the rank's slice
            if lo < hi:
                ok &= bool(bits[lo - qa:hi - qa].all())
            # the absent keys: false positives at the filter's own rate (fill^k)
            fill = filters[g].popcount() / (8 * nb_bytes)
            fp_total += int(bits[nq - n_abs:].sum())
            fp_expect += n_abs * fill ** k
        fp_ok = fp_total <= 3 * fp_expect + 20 * len(mine)
    host_c5 = None
    if args.config == "c5" and not args.no_host_c5:
        host_c5 = c5_host_resident(args, filters, mine, hms, q, nq, k, torch, np, L)
    if world > 1:
        elapsed = float(all_reduce_scalar(torch, dist, elapsed, dist.ReduceOp.MAX, torch.float64))
        ok = bool(all_reduce_scalar(torch, dist, 1 if ok else 0, dist.ReduceOp.MIN, torch.int32))
        if args.config == "c5":
            fp_ok = bool(all_reduce_scalar(torch, dist, 1 if fp_ok else 0, dist.ReduceOp.MIN, torch.int32))
    if rank == 0:
        ms = elapsed / args.steps * 1e3
        if args.config == "c4":
            b_pass = algorithmic_bytes(n, 16.0, k, 8 * nb_bytes, False)
            metric, unit = "Mkeys/s bloom build, 1B 16B keys into 8 product-sized SSTable filters", "Mkeys/s"
            what = (f"c4: 8 filters x {n} 16-B keys (product sizing fp 0.001: nb_bytes={nb_bytes}, k={k}); "
                    f"a step builds every filter once; filters {len(mine)}/rank")
            pk = "build pass of the rank's filters (clear + tiled build each, concurrent streams)"
        else:
            # the shared partition reads the keys ONCE for all of the rank's filters; each filter
            # then costs its k 4-B bitmap reads per key and its hit mask (SURVEY.md §8d probe
            # bytes, key term counted once): nq*L + nf*(4*nq*k + nq/8)
            b_pass = nq * 16 + len(mine) * (4 * nq * k + nq // 8)
            metric, unit = f"Mprobes/s (key x filter) batched probe, {nq_all // 1_000_000}M keys vs 8x128MiB filters", "Mprobes/s"
            what = (f"c5: {nq_all} probe keys (half members) x 8 filters (nb_bytes=2^27, k=6, 10M keys each); "
                    f"layout '{plan['layout']}': the rank probes keys [{qa}, {qb}) against its {len(mine)} filters "
                    f"in one pbf_probe_multi per step")
            pk = ("multi-filter probe (shared k_part_ring + one XCD-aware k_tile_probe_set over every filter + "
                  "one fused k_gather_ring<8>)")
        if args.config == "c4":
            # the rank's filters build concurrently on their own streams, so per-filter event
            # spans overlap: the pass rate is all of the rank's filters' bytes per step time
            b_pass *= len(mine)
            pass_ms = ms
        ach = b_pass / (pass_ms * 1e-3) / 1e9
        # PMC traffic of the same pass (profiles/traffic_c4.json: one filter's build pass, so x the
        # rank's filters; profiles/traffic_c5.json: the multi-filter probe, already x its pipelines)
        tr = measured_traffic(args.config)
        traffic = None
        if tr is not None and (args.config == "c4" or nq == nq_all):  # (measured on the whole batch)
            traffic = int(tr["build"] * len(mine)) if args.config == "c4" else int(tr["probe"])
        out = {
            "metric": metric, "value": round(unit_total / (ms * 1e-3) / 1e6, 3),
            "unit": unit, "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (splitmix64 hex keys generated on device)",
            "config": {"workload": what, "nb_bytes": nb_bytes, "k": k, "filters_per_rank": len(mine),
                       "parallelism": (f"keys-over-gpus x{world}" if args.config == "c5" and plan.get("layout") == "keys"
                                       else f"filters-over-gpus x{world}")},
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": pk,
                         "algorithmic_bytes": int(b_pass), "avg_ms": round(pass_ms, 4),
                         "traffic_source": tr["source"] if tr else None},
            "check": {"members_all_hit": ok},
            **dist_report(dist, world),
        }
        if sim:
            out["simulated_rank"] = {"rank": args.sim_rank, "world": args.sim_world,
                                     "note": "one rank's share of a --sim-world job on this GPU; value = that "
                                             "rank's units / its time (no process group)"}
        if fp_rate is not None:
            out["check"]["fp_rate_1M_absent"] = fp_rate
        if args.config == "c5":
            out["check"].update({"false_positives_rank0": fp_total, "fp_expected_rank0": round(fp_expect, 1),
                                 "fp_within_3x_expected": bool(fp_ok), "probe_detail": hex(s0.last_probe_detail)})
            if host_c5 is not None:
                out["host_resident"] = host_c5
            if replication is not None:
                # one-time: the layout's filters arrive once, then every step probes them
                replication["built_here"] = own
                out["replication"] = replication
            if world == 1 and not args.no_cpu_baseline:
                out["cpu_baseline"] = c5_cpu_baseline(args, filters, mine, hms, q, n_f, nb_bytes, k, np)
                out["check"]["oracle_sample_equal"] = out["cpu_baseline"].pop("oracle_sample_equal")
        if args.config == "c5" and not args.no_compare:
            # the same work as independent single-filter probes (no shared partition)
            tq = []
            for _ in range(2):
                t1 = time.perf_counter()
                for g in mine:
                    filters[g].probe_device_fixed(q.data_ptr(), 16, nq, hms[g].data_ptr())
                for g in mine:
                    filters[g].sync()
                tq.append(time.perf_counter() - t1)
            out["per_filter_probes_ms"] = round(min(tq) * 1e3, 3)
        print(json.dumps(out), flush=True)


def mixed_main(args, rank, world, local, torch, dist, np):
    """c5mixed — the batched LsmStorage.get filter stage (src/lsm_storage.py:164-179) over SSTable
    filters of DIFFERENT sizes, as an LSM has them (each sized from its own key count,
    sstable.py:274: fp 0.001 -> k = 10): 8 filters of 0.5M..4M keys (nb_bytes 0.9..7.2 MB) and
    a batch of 36M 16-B keys (the 18M members + 18M absent) in HBM.  A step = one
    pbf_probe_multi of the batch against the rank's filters: one k_probe_set launch that hashes
    every key once and tests every filter.  Beside it the previous behaviour, one probe pipeline
    per filter (each re-reading and re-hashing the batch).  value = key x filter probes / s."""
    from math import ceil, log

    from oracle.oracle import COracle
    from pebbledb_amd import BloomFilter, PackedKeys, _native, probe_multi_device
    from pebbledb_amd.bloom_filter import set_default_device
    from pebbledb_amd.keys import splitmix_hex_keys
    from pebbledb_amd.shard import filters_for_rank

    set_default_device(local)
    L = _native.lib()
    mine = filters_for_rank(8, world, rank)
    ns = [500_000 * (g + 1) for g in range(8)]
    starts = [sum(ns[:g]) for g in range(8)]
    total = sum(ns)
    nq = 2 * total
    q = torch.empty(nq * 16, dtype=torch.uint8, device="cuda")
    _native.check(L.pbf_gen_splitmix_hex(local, None, q.data_ptr(), SEED, 0, nq), "gen")
    torch.cuda.synchronize()
    filters = {}
    for g in mine:
        m = (-ns[g] * log(0.001)) / (log(2) ** 2)  # bloom_filter.py:109-114, same expression order
        bf = BloomFilter(ceil(m / 8), round((m / ns[g]) * log(2)), device=local)
        bf.add_device_fixed(q.data_ptr() + starts[g] * 16, 16, ns[g])
        bf.sync()
        filters[g] = bf
    fl = [filters[g] for g in mine]
    k = fl[0].nb_hash_functions
    hms = {g: torch.zeros((nq + 7) // 8, dtype=torch.uint8, device="cuda") for g in mine}
    stream = torch.cuda.ExternalStream(fl[0].stream)

    def fused():
        probe_multi_device(fl, q.data_ptr(), nq, [hms[g].data_ptr() for g in mine], key_len=16)

    def per_filter():
        for g in mine:
            filters[g].probe_device_fixed(q.data_ptr(), 16, nq, hms[g].data_ptr())

    def timed(fn):
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
        for _ in range(args.warmup):
            fn()
        for bf in fl:
            bf.sync()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for st in range(args.steps):
            evs[st][0].record(stream)
            fn()
            evs[st][1].record(stream)
        for bf in fl:
            bf.sync()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            el = float(all_reduce_scalar(torch, dist, el, dist.ReduceOp.MAX, torch.float64))
        return el / args.steps * 1e3, sum(a.elapsed_time(b) for a, b in evs) / args.steps

    ms_pf, _ = timed(per_filter)
    got_pf = {g: hms[g].cpu().numpy().copy() for g in mine}
    ms, pass_ms = timed(fused)
    got = {g: hms[g].cpu().numpy() for g in mine}
    ok = all(np.array_equal(got[g], got_pf[g]) for g in mine)
    fp_total, fp_expect = 0, 0.0
    for g in mine:
        bits = np.unpackbits(got[g], bitorder="little")[:nq]
        ok &= bool(bits[starts[g]:starts[g] + ns[g]].all())
        fill = filters[g].popcount() / (8 * filters[g].nb_bytes)
        fp_total += int(bits[total:].sum())
        fp_expect += total * fill ** k
    fp_ok = fp_total <= 3 * fp_expect + 20 * len(mine)
    if world > 1:
        ok = bool(all_reduce_scalar(torch, dist, 1 if ok else 0, dist.ReduceOp.MIN, torch.int32))
    if rank != 0:
        return
    # SURVEY.md §8d probe bytes with the key read once for the set: nq*L + nf*(4*nq*k + nq/8)
    b_pass = nq * 16 + len(mine) * (4 * nq * k + nq // 8)
    ach = b_pass / (pass_ms * 1e-3) / 1e9
    out = {
        "metric": "Mprobes/s (key x filter) batched probe, 36M keys vs 8 mixed-size product-sized filters",
        "value": round(nq * 8 / (ms * 1e-3) / 1e6, 3), "unit": "Mprobes/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (splitmix64 hex keys generated on device)",
        "config": {"workload": (f"c5mixed: {nq} probe keys (half members) x 8 product-sized filters of "
                                f"{ns[0]}..{ns[-1]} keys (fp 0.001, k={k}); filters {len(mine)}/rank"),
                   "nb_bytes": [filters[g].nb_bytes for g in mine], "k": k,
                   "parallelism": f"filters-over-gpus x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "k_probe_set (each key hashed once, every filter tested; bitmaps Infinity-Cache resident)",
                     "algorithmic_bytes": int(b_pass), "avg_ms": round(pass_ms, 4)},
        "per_filter_pipelines_ms": round(ms_pf, 4), "speedup_vs_per_filter": round(ms_pf / ms, 2),
        "check": {"members_all_hit": ok, "equal_to_per_filter_probes": ok, "false_positives": fp_total,
                  "fp_expected": round(fp_expect, 1), "fp_within_3x_expected": bool(fp_ok),
                  "probe_detail": hex(fl[0].last_probe_detail)},
        **dist_report(dist, world),
    }
    if world == 1 and not args.no_cpu_baseline:
        # the C oracle (OpenMP, all host cores) on a 2M-key sample against every filter, and the
        # sample's hit masks equal to the device's
        o = COracle()
        ns_s = 2_000_000
        sample = PackedKeys.fixed(splitmix_hex_keys(SEED, total - ns_s // 2, ns_s))
        bms = [np.frombuffer(filters[g].bitmap(), dtype=np.uint8).copy() for g in mine]
        t0 = time.perf_counter()
        hs = [o.probe(bm, k, sample, omp=True) for bm in bms]
        t_cpu = time.perf_counter() - t0
        off = (total - ns_s // 2) // 8
        same = all(np.array_equal(h, got[g][off:off + ns_s // 8]) for h, g in zip(hs, mine))
        out["cpu_baseline"] = {"value": round(ns_s * len(mine) / t_cpu / 1e6, 3), "unit": "Mprobes/s",
                               "cores": o.num_threads(), "kind": "port",
                               "sample": f"C oracle, {ns_s} keys x {len(mine)} filters (OpenMP)"}
        out["check"]["oracle_sample_equal"] = same
    print(json.dumps(out), flush=True)


def sst_main(args, rank, world, local, torch, dist, np):
    """SSTable data-section encode (sstable.py:224-268): one flush-sized
    SSTable per GPU — 3.5M records of a 16-B hex key and a 48-B value (72 B encoded, 252 MB of
    data blocks, the reference's 250 MB target), records and the host block plan already in
    HBM.  A step = one pbf_encode_data_blocks over every block.  value = records / s (all
    ranks).  Also: the host-inclusive SSTable build from Python lists (pack, plan, H2D, encode,
    D2H, meta blocks, device bloom) on a 1M-record sample, and the oracle restatement of the
    reference's builder (oracle/sstable_oracle.py) on a bounded sample as the CPU baseline."""
    import ctypes

    from pebbledb_amd import _native
    from pebbledb_amd.keys import PackedKeys, splitmix_hex_keys
    from pebbledb_amd.sstable_data import build_sstable, key_offsets, plan_blocks

    n, vlen = 3_500_000, 48
    L = _native.lib()
    kb = splitmix_hex_keys(SEED, rank * n, n)
    pk = PackedKeys.fixed(kb)
    ko = key_offsets(pk)
    rng = np.random.default_rng(rank)
    vals = rng.integers(0, 256, n * vlen, dtype=np.uint8)
    vo = np.arange(n + 1, dtype=np.uint64) * np.uint64(vlen)
    bf, bo = plan_blocks(ko, vo, 65_536)
    t = {name: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).cuda()
         for name, a in (("k", pk.data), ("ko", ko), ("v", vals), ("vo", vo), ("bf", bf), ("bo", bo))}
    out = torch.empty(int(bo[-1]), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    nblocks = len(bf) - 1

    def step():
        _native.check(L.pbf_encode_data_blocks(local, t["k"].data_ptr(), t["ko"].data_ptr(), t["v"].data_ptr(),
                                               t["vo"].data_ptr(), n, t["bf"].data_ptr(), t["bo"].data_ptr(), nblocks,
                                               out.data_ptr(), 1), "encode")
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = float(all_reduce_scalar(torch, dist, elapsed, dist.ReduceOp.MAX, torch.float64))
    if rank != 0:
        return
    ms = elapsed / args.steps * 1e3
    section = int(bo[-1])
    alg = pk.data.size + vals.size + 2 * 8 * (n + 1) + section  # read keys, values, offsets; write blocks
    ach = alg / (ms * 1e-3) / 1e9
    # host-inclusive SSTable file from Python lists, 1M records
    hn = 1_000_000
    hkeys = [format(x, "016x") for x in range(hn)]
    hvals = [bytes(vals[i * vlen:(i + 1) * vlen]) for i in range(hn)]
    th = time.perf_counter()
    f, metas, _ = build_sstable(hkeys, hvals)
    th = time.perf_counter() - th
    # the flush without list[str]: the memtable's encoded records (the
    # memtable.map iterates them in key order, Record.to_bytes) drained by the C packer into the boundary layout,
    # then the same device SSTable build -> file bytes; checked byte-identical to the list path
    import struct
    from pebbledb_amd.keys import PackedRecords
    hp = struct.pack("i", 16)
    hv = struct.pack("i", vlen)
    enc = [hp + k.encode() + hv + v for k, v in zip(hkeys, hvals)]
    tf = []
    same_file = True
    for _ in range(3):
        t0 = time.perf_counter()
        pr = PackedRecords.from_encoded(enc)
        t1 = time.perf_counter()
        f2, _, _ = build_sstable(pr)
        tf.append((time.perf_counter() - t0, t1 - t0))
        same_file = same_file and bytes(f2) == bytes(f)
        del pr, f2  # the previous flush's buffers are freed outside the next timed flush
    t_flush, t_pack = min(tf)
    # keys only, from a generator (the iterator chain shape) vs the list[str] join path
    t0 = time.perf_counter()
    PackedKeys.from_iter(k for k in hkeys)
    t_iter = time.perf_counter() - t0
    t0 = time.perf_counter()
    PackedKeys.from_strs(hkeys)
    t_strs = time.perf_counter() - t0
    compaction = compaction_leg(np, local)
    # CPU baseline: the reference builder's algorithm (oracle restatement), bounded sample
    from oracle import sstable_oracle as so
    cn = 0
    tc = time.perf_counter()
    while cn < hn and time.perf_counter() - tc < min(10.0, args.cpu_seconds):
        so.data_and_meta(hkeys[cn:cn + 20000], hvals[cn:cn + 20000], 65_536)
        cn += 20000
    tc = time.perf_counter() - tc
    out_line = {
        "metric": "Mrecords/s SSTable data-block encode (device-resident), 3.5M x (16-B key, 48-B value)",
        "value": round(n * world / (ms * 1e-3) / 1e6, 3), "unit": "Mrecords/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic (hex keys, random values)",
        "config": {"workload": f"sst: {n} records, {nblocks} data blocks of <= 64 KiB, {section} B section per GPU",
                   "parallelism": f"sstable-per-gpu x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "kernel": "k_encode_blocks",
                     "algorithmic_bytes": int(alg), "avg_ms": round(ms, 4)},
        "host_inclusive": {"records": hn, "s": round(th, 3), "Mrecords_s": round(hn / th / 1e6, 3),
                           "file_bytes": len(f), "what": "build_sstable(list[str], list[bytes]): pack, plan, H2D, "
                                                          "encode, D2H, meta blocks, device bloom, file assembly"},
        "flush_host_inclusive": {"records": hn, "s": round(t_flush, 3), "Mrecords_s": round(hn / t_flush / 1e6, 3),
                                 "pack_s": round(t_pack, 3), "pack_Mrecords_s": round(hn / t_pack / 1e6, 2),
                                 "file_identical_to_list_path": same_file,
                                 "keys_from_generator_Mkeys_s": round(hn / t_iter / 1e6, 2),
                                 "keys_from_list_join_Mkeys_s": round(hn / t_strs / 1e6, 2),
                                 "what": "records -> file bytes: memtable-encoded records (Record.to_bytes) -> "
                                         "PackedRecords.from_encoded (C packer) -> build_sstable (plan, H2D, device "
                                         "encode, D2H, meta, device bloom, trailer); best of 3, the previous flush freed outside the timing"},
        "cpu_baseline": {"value": round(cn / tc / 1e6, 4), "unit": "Mrecords/s", "cores": 1, "kind": "port",
                         "sample": f"oracle/sstable_oracle.py data_and_meta (the reference builder's algorithm) "
                                   f"on {cn} records in {tc:.1f}s"},
        "compaction": compaction,
    }
    print(json.dumps(out_line), flush=True)


def compaction_leg(np, device, n=4_000_000, vlen=48, max_sstable_size=100_000_000, reps=3):
    """Compaction's output SSTables (LsmStorage._compact, src/lsm_storage.py:233-251) for a merged
    run of n records (sorted 16-B hex keys, 48-B values; packed beforehand, as the merging
    iterator's output would be by the C packer): build_sstables (the split planned on the host,
    ONE upload, one encode launch for every output, the outputs' filters built side by side on
    pooled streams) vs one build_sstable call per output over the same ranges, run after run.
    Host-inclusive (records in host memory -> file bytes of every output); best of `reps`; the
    files of both paths must be identical."""
    from pebbledb_amd.keys import PackedKeys, PackedRecords, splitmix_hex_keys
    from pebbledb_amd.sstable_data import build_sstable, build_sstables, key_offsets, plan_compaction
    kb = np.sort(splitmix_hex_keys(SEED, 0, n).view("S16").reshape(-1)).view(np.uint8).reshape(n, 16)
    vals = np.random.default_rng(5).integers(0, 256, n * vlen, dtype=np.uint8)
    vo = np.arange(n + 1, dtype=np.uint64) * np.uint64(vlen)
    run = PackedRecords(PackedKeys.fixed(kb), vals, vo, ascii=True)
    bf, bo, tb, written = plan_compaction(np.asarray(key_offsets(run.keys), np.uint64), vo, 65_536, max_sstable_size)
    parts = []
    for t in range(len(tb) - 1):
        r0, r1 = int(bf[tb[t]]), int(bf[tb[t + 1]])
        parts.append(PackedRecords(PackedKeys.fixed(kb[r0:r1]), vals[r0 * vlen:r1 * vlen], vo[:r1 - r0 + 1], ascii=True))
    t_one, t_seq = [], []
    same = True
    for _ in range(reps):
        t0 = time.perf_counter()
        outs, w = build_sstables(run, max_sstable_size=max_sstable_size, device=device)
        t_one.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        seq = [build_sstable(p, device=device) for p in parts]
        t_seq.append(time.perf_counter() - t0)
        same = same and len(seq) == len(outs) and all(bytes(a[0]) == bytes(b[0]) for a, b in zip(outs, seq))
        del outs, seq
    a, b = min(t_one), min(t_seq)
    return {"records": n, "written": written, "outputs": len(tb) - 1, "max_sstable_size": max_sstable_size,
            "build_sstables_s": round(a, 4), "build_sstables_Mrecords_s": round(written / a / 1e6, 2),
            "sequential_build_sstable_s": round(b, 4), "sequential_Mrecords_s": round(written / b / 1e6, 2),
            "speedup": round(b / a, 3), "files_identical": bool(same),
            "what": "host-inclusive: packed run -> every output's file bytes (plan, H2D, device encode + filters, "
                    "D2H, meta, trailer); best of 3"}


def spawn_ranks(args) -> int:
    """--gpus N without a launcher: start N ranks of this script (one per GPU) and wait.  Runs
    before anything in this process touches a GPU (children are started, never exec'd into).
    A rank that fails ends the others (they would wait at a barrier forever)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or code
                for other in live:
                    other.terminate()
        time.sleep(0.05)
    return rc


def dist_report(dist, world):
    """The process group the timing went over: its backend and the world size it saw.
    `rccl_world_size` is always present (1 for a single-GPU run, the RCCL world otherwise; null
    for a gloo rehearsal, which is not RCCL); `world_size_seen` is what the group saw."""
    if world == 1:
        return {"backend": None, "rccl_world_size": 1, "world_size_seen": 1}
    be = dist.get_backend()
    ws = dist.get_world_size()
    return {"backend": be, "rccl_world_size": ws if be == "nccl" else None, "world_size_seen": ws}


def dry_run(args, rank, world, dist):
    """Launcher and plumbing check without a GPU: gloo rendezvous on 127.0.0.1, the barrier
    and the max-over-ranks of the timed region as a real run does them.  Reports no number."""
    import torch
    if world > 1:
        dist.init_process_group(backend="gloo", init_method="env://")
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    elapsed = time.perf_counter() - t0
    seen = 1
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        seen = dist.get_world_size()
    # every rank's placement as its own process computed it (LOCAL_RANK -> device, filters, keys)
    plan = rank_plan(args.config, world, rank, int(os.environ.get("LOCAL_RANK", "0")), args.c4_keys,
                     args.c5_probes, args.c5_layout)
    plans = [plan]
    if world > 1:
        plans = [None] * world
        dist.all_gather_object(plans, plan)
    if rank == 0:
        print(json.dumps({"dry_run": True, "metric": None, "value": None, "n_gpus": world, "world_size_seen": seen,
                          "backend": "gloo" if world > 1 else None, "max_elapsed_s": round(elapsed, 4),
                          "config": {"workload": args.config}, "plans": plans}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus={args.gpus}: launch {args.gpus} ranks "
              f"(or run without a launcher and let --gpus start them)", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        import torch.distributed as dist
        dry_run(args, rank, world, dist)
        return
    # rehearsal of the N-rank path on a one-GPU box: every rank on device PBF_BENCH_DEVICE,
    # rendezvous / max-over-ranks over gloo (PBF_BENCH_BACKEND=gloo); the driver's runs use
    # one GPU per rank over RCCL
    if os.environ.get("PBF_BENCH_DEVICE"):
        local = int(os.environ["PBF_BENCH_DEVICE"])

    import torch
    import torch.distributed as dist
    import numpy as np

    torch.cuda.set_device(local)
    if world > 1:
        # RCCL carries only the timing plumbing (barrier, max over ranks): the data path has no
        # collective.  If RCCL cannot start the run fails (exit 3) rather than
        # silently timing over another backend; gloo only when asked for (PBF_BENCH_BACKEND=gloo,
        # the one-GPU rehearsal).
        init_process_group_or_exit(dist, torch, os.environ.get("PBF_BENCH_BACKEND", "nccl"), local, rank)

    if args.config == "c5mixed":
        mixed_main(args, rank, world, local, torch, dist, np)
        if world > 1:
            dist.destroy_process_group()
        return
    if args.config == "sst":
        sst_main(args, rank, world, local, torch, dist, np)
        if world > 1:
            dist.destroy_process_group()
        return
    if args.config in ("c4", "c5"):
        sets_main(args, rank, world, local, torch, dist, np)
        if world > 1:
            dist.destroy_process_group()
        return

    from pebbledb_amd import BloomFilter, _native
    from pebbledb_amd.bloom_filter import set_default_device

    set_default_device(local)
    n, nb_bytes, k, kind = CONFIGS[args.config]
    m_bits = 8 * nb_bytes
    # this rank's SSTable: keys [rank*2n, rank*2n + n) are members, [.. + n, .. + 2n) are absent
    start = rank * 2 * n
    L = _native.lib()
    if kind == "hex16":
        keys = torch.empty(2 * n * 16, dtype=torch.uint8, device="cuda")
        _native.check(L.pbf_gen_splitmix_hex(local, None, keys.data_ptr(), SEED, start, 2 * n), "gen")
        offs = None
        key_bytes = 16.0
    else:
        from pebbledb_amd.keys import _splitmix64_np
        idx = np.arange(start, start + 2 * n, dtype=np.uint64)
        with np.errstate(over="ignore"):
            h = _splitmix64_np((np.uint64(SEED_VAR) << np.uint64(32)) + idx)
        lens = (8 + h % np.uint64(57)).astype(np.int64)
        o = np.zeros(2 * n + 1, dtype=np.int64)
        np.cumsum(lens, out=o[1:])
        offs = torch.from_numpy(o).cuda()
        keys = torch.empty(int(o[-1]), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        _native.check(L.pbf_gen_varlen(local, None, keys.data_ptr(), offs.data_ptr(), SEED_VAR, start, 2 * n), "gen")
        key_bytes = float(o[n]) / n
        del h, lens, idx
    hitmask = torch.zeros((2 * n + 7) // 8, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    bf = BloomFilter(nb_bytes, k, device=local)
    if args.build_mode:
        bf.set_build_mode(args.build_mode)
    if args.probe_mode:
        bf.set_probe_mode(args.probe_mode)
    stream = torch.cuda.ExternalStream(bf.stream)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        bf.clear()  # the build's time includes zeroing the bitmap (a memset, or the tile pass)
        if offs is None:
            bf.add_device_fixed(keys.data_ptr(), 16, n)
        else:
            bf.add_device(keys.data_ptr(), offs.data_ptr(), n)
        if ev is not None:
            ev[1].record(stream)
        if offs is None:
            bf.probe_device_fixed(keys.data_ptr(), 16, 2 * n, hitmask.data_ptr())
        else:
            bf.probe_device(keys.data_ptr(), offs.data_ptr(), 2 * n, hitmask.data_ptr())
        if ev is not None:
            ev[2].record(stream)

    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    span = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    # warm-up right before the timed region: the GPU is never idle long before t0 (a queue left
    # idle for ~100 ms was seen to start its next submission up to ~20 ms late)
    for _ in range(args.warmup):
        step()
    bf.sync()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    bf.sync()
    t0 = time.perf_counter()
    span[0].record(stream)
    for s in range(args.steps):
        step(None if args.no_events else events[s])
        if args.sync_each_step:
            bf.sync()
    span[1].record(stream)
    t_enq = time.perf_counter()
    bf.sync()
    t_done = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    gpu_span_ms = span[0].elapsed_time(span[1])
    # correctness guard on the measured data (the last step's hit mask): every member must hit
    hm = hitmask.cpu().numpy()
    members_ok = bool((np.unpackbits(hm, bitorder="little")[:n] == 1).all())
    fp = int(np.unpackbits(hm, bitorder="little")[n:2 * n].sum())
    # a corrupted bitmap (e.g. all ones) still lets every member hit: the absent half must show
    # false positives at the filter's own rate, fill^k (fill measured on the device)
    # positions a signed 32-bit hash can reach: all m, or 2^32 of them when m > 2^32
    # (bloom_filter.py:47 floor-mod)
    fill = bf.popcount() / min(m_bits, 2 ** 32)
    fp_expect = n * fill ** k
    fp_ok = fp <= 3 * fp_expect + 20
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if args.no_events:
        for s in range(min(args.steps, 5)):  # time a few steps separately for the roofline
            step(events[s])
        bf.sync()
        events = events[:min(args.steps, 5)]
    build_ms = sum(e[0].elapsed_time(e[1]) for e in events) / len(events)
    probe_ms = sum(e[1].elapsed_time(e[2]) for e in events) / len(events)
    # GPU time of a step (build + probe events) averaged over each quarter of the timed steps: shows
    # whether the first steps of a short run are slower (clocks still ramping under sustained load)
    quarters = None
    if not args.no_events and len(events) >= 4:
        per = [e[0].elapsed_time(e[2]) for e in events]
        q = len(per) // 4
        quarters = [round(sum(per[i * q:(i + 1) * q]) / q, 4) for i in range(4)]
    if world > 1:
        elapsed = float(all_reduce_scalar(torch, dist, elapsed, dist.ReduceOp.MAX, torch.float64))
        members_ok = bool(all_reduce_scalar(torch, dist, 1 if members_ok else 0, dist.ReduceOp.MIN, torch.int32))
        fp_ok = bool(all_reduce_scalar(torch, dist, 1 if fp_ok else 0, dist.ReduceOp.MIN, torch.int32))

    host_inc = None
    if rank == 0 and offs is None and not args.no_host_inclusive:
        host_inc = host_inclusive(bf, keys, n, nb_bytes, L, torch, np)

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        keys_per_step = 3 * n * world
        value = keys_per_step * args.steps / elapsed / 1e6
        offsets = offs is not None
        b_build = algorithmic_bytes(n, key_bytes, k, m_bits, offsets)
        b_probe = probe_bytes(2 * n, key_bytes, k, offsets)
        ach_build = b_build / (build_ms * 1e-3) / 1e9
        ach_probe = b_probe / (probe_ms * 1e-3) / 1e9
        if build_ms >= probe_ms:
            dom = {"kernel": f"build pass ({'tiled' if bf.last_build_mode == 2 else 'atomic'}: "
                             f"{'k_part+k_tile_build+k_ovf_build' if bf.last_build_mode == 2 else 'k_build_atomic'})",
                   "achieved": ach_build, "ms": build_ms, "bytes": b_build}
        else:
            dom = {"kernel": ("probe pass (tiled: k_part<probe>+k_tile_probe+k_gather)" if bf.last_probe_mode == 2
                              else "k_probe"), "achieved": ach_probe, "ms": probe_ms, "bytes": b_probe}
        traffic = measured_traffic(args.config)
        dom_pass = "build" if build_ms >= probe_ms else "probe"
        out = {
            "metric": ("Mkeys/s bloom build+probe (device-resident), 10M 16B keys; 1/2/4/8 GPU" if args.config == "c2"
                       else f"Mkeys/s bloom build+probe (device-resident), {n} "
                            f"{'16B' if kind == 'hex16' else 'variable-length (8-64 B)'} keys"),
            "value": round(value, 3),
            "unit": "Mkeys/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": ("synthetic (splitmix64 hex keys generated on device)" if kind == "hex16" else
                     "synthetic (splitmix64-derived [0-9a-z] keys of 8-64 B generated on device)"),
            "config": {"workload": f"{args.config}: build {n} keys of {key_bytes:.1f} B into m=2^{m_bits.bit_length() - 1}"
                                   f" bits (nb_bytes={nb_bytes}), k={k}; probe {2 * n} keys ({n} members + {n} absent)"
                                   f"; one filter per GPU", "n_build": n, "n_probe": 2 * n, "nb_bytes": nb_bytes, "k": k,
                       "keys_per_step_per_gpu": 3 * n, "parallelism": f"filter-per-gpu x{world}"},
            "host_enqueue_ms_per_step": round((t_enq - t0) / args.steps * 1e3, 4),
            "gpu_span_ms_per_step": round(gpu_span_ms / args.steps, 4),
            "gpu_ms_per_step_by_quarter": quarters,
            "host_wait_ms": {"stream_done": round((t_done - t_enq) * 1e3, 3), "device_sync": round((t1 - t_done) * 1e3, 3)},
            "build_ms": round(build_ms, 4),
            "probe_ms": round(probe_ms, 4),
            "build_Mkeys_s_per_gpu": round(n / build_ms / 1e3, 1),
            "probe_Mkeys_s_per_gpu": round(2 * n / probe_ms / 1e3, 1),
            "build_mode": bf.last_build_mode,
            "probe_mode": bf.last_probe_mode,
            "roofline": {"bound": "hbm", "achieved": round(dom["achieved"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(dom["achieved"] / HBM_PEAK_GBS, 4),
                         "traffic": int(traffic[dom_pass]) if traffic else None, "kernel": dom["kernel"],
                         "algorithmic_bytes": int(dom["bytes"]), "avg_ms": round(dom["ms"], 4)},
            "roofline_build": {"achieved": round(ach_build, 1), "frac": round(ach_build / HBM_PEAK_GBS, 4),
                               "algorithmic_bytes": int(b_build), "traffic": int(traffic["build"]) if traffic else None},
            "roofline_probe": {"achieved": round(ach_probe, 1), "frac": round(ach_probe / HBM_PEAK_GBS, 4),
                               "algorithmic_bytes": int(b_probe), "traffic": int(traffic["probe"]) if traffic else None},
            "traffic_source": traffic["source"] if traffic else "no PMC summary for this library build",
            "check": {"members_all_hit": members_ok, "false_positives": fp, "probes_absent": n,
                      "fp_expected": round(fp_expect, 2), "fp_within_3x_expected": bool(fp_ok)},
            **dist_report(dist, world),
        }
        if host_inc is not None:
            out["host_inclusive"] = host_inc
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(nb_bytes, k, kind, args.cpu_seconds)
            if args.config == "c1":
                out["dropin_latency"] = dropin_latency(local)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    del bf


if __name__ == "__main__":
    main()
