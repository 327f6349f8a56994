"""The N-rank path with the HIP library doing each rank's filter work (`-m gpu`): two ranks on
the one GPU of the box, rendezvous over gloo on 127.0.0.1, each rank builds and probes ITS
SSTable filters (shard.filters_for_rank, independent filters, no collective on the data path:
src/lsm_storage.py:200-205,238-249), and every hit mask gathered from both ranks equals the
oracle's.  The driver's 8-GPU runs use one GPU per rank over RCCL; this checks the sharding
and the bookkeeping with real device results."""
import json
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_WORKER = textwrap.dedent("""
    import json, os, sys
    sys.path.insert(0, '.')
    import numpy as np
    import torch.distributed as dist
    from pebbledb_amd import BloomFilter, PackedKeys, may_contain_multi
    from pebbledb_amd.keys import splitmix_hex_keys
    from pebbledb_amd.shard import filters_for_rank, key_range
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", init_method="env://")
    n_filters, kpf, nb, k = 8, 40_000, 2 ** 18, 6
    mine = filters_for_rank(n_filters, world, rank)
    probe = PackedKeys.fixed(splitmix_hex_keys(77, 0, n_filters * kpf + 5000))
    fs = []
    for f in mine:
        a, b = key_range(f, kpf)
        bf = BloomFilter(nb, k, device=0)
        bf.add_many(PackedKeys.fixed(splitmix_hex_keys(77, a, b - a)))
        fs.append(bf)
    masks = may_contain_multi(fs, probe)  # this rank's filters, one shared pipeline
    local = {f: masks[i].tobytes().hex() for i, f in enumerate(mine)}
    objs = [None] * world
    dist.all_gather_object(objs, local)
    merged = {}
    for d in objs:
        merged.update(d)
    dist.barrier()
    if rank == 0:
        print("RESULT " + json.dumps({"world": dist.get_world_size(), "masks": merged}), flush=True)
    dist.destroy_process_group()
""")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_one_gpu_hip_filters_equal_oracle(oracle):
    from pebbledb_amd.keys import PackedKeys, splitmix_hex_keys
    from pebbledb_amd.shard import gather_hitmasks, key_range
    world, port = 2, _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", _WORKER], env=env, cwd=REPO, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    res = json.loads([x for x in outs[0][0].splitlines() if x.startswith("RESULT ")][0][7:])
    assert res["world"] == 2
    masks = {int(f): np.frombuffer(bytes.fromhex(h), np.uint8) for f, h in res["masks"].items()}
    assert sorted(masks) == list(range(8))
    probe = PackedKeys.fixed(splitmix_hex_keys(77, 0, 8 * 40_000 + 5000))
    mat = gather_hitmasks(masks, 8, probe.n)
    for f in range(8):
        a, b = key_range(f, 40_000)
        want = oracle.build(2 ** 18, 6, PackedKeys.fixed(splitmix_hex_keys(77, a, b - a)))
        assert np.array_equal(masks[f], oracle.probe(want, 6, probe)), f
        assert mat[f, a:b].all()


_KEYS_WORKER = textwrap.dedent("""
    import importlib.util, json, os, sys
    sys.path.insert(0, '.')
    import numpy as np
    import torch.distributed as dist
    from pebbledb_amd import BloomFilter, PackedKeys, may_contain_multi
    from pebbledb_amd.keys import splitmix_hex_keys
    from pebbledb_amd.shard import key_range
    spec = importlib.util.spec_from_file_location("bench_mod", "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", init_method="env://")
    n_filters, kpf, nb, k, nq = 8, 40_000, 2 ** 18, 6, 8 * 40_000 + 5003
    plan = bench.rank_plan("c5", world, rank, 0, c5_probes=nq)  # key-partitioned layout
    a, b = plan["probe_keys"]
    fs = []
    for f in plan["filters"]:
        lo, hi = key_range(f, kpf)
        bf = BloomFilter(nb, k, device=0)
        bf.add_many(PackedKeys.fixed(splitmix_hex_keys(77, lo, hi - lo)))
        fs.append(bf)
    probe = PackedKeys.fixed(splitmix_hex_keys(77, a, b - a))  # only this rank's slice
    masks = may_contain_multi(fs, probe)
    objs = [None] * world
    dist.all_gather_object(objs, {"a": a, "b": b, "masks": [m.tobytes().hex() for m in masks]})
    dist.barrier()
    if rank == 0:
        print("RESULT " + json.dumps(objs), flush=True)
    dist.destroy_process_group()
""")


def test_two_ranks_key_partitioned_probe_equals_oracle(oracle):
    """C5's key-partitioned layout (bench.rank_plan 'keys'): every rank holds the 8 filters and
    probes its slice of the batch through the fused multi-filter path; the slices' masks,
    concatenated, equal the oracle's whole-batch masks for every filter."""
    from pebbledb_amd.keys import PackedKeys, splitmix_hex_keys
    from pebbledb_amd.shard import key_range
    world, port = 2, _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", _KEYS_WORKER], env=env, cwd=REPO, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    parts = json.loads([x for x in outs[0][0].splitlines() if x.startswith("RESULT ")][0][7:])
    nq = 8 * 40_000 + 5003
    assert parts[0]["a"] == 0 and parts[-1]["b"] == nq and parts[0]["b"] == parts[1]["a"] and parts[0]["b"] % 64 == 0
    probe = PackedKeys.fixed(splitmix_hex_keys(77, 0, nq))
    for f in range(8):
        got = np.concatenate([np.frombuffer(bytes.fromhex(p["masks"][f]), np.uint8) for p in parts])
        lo, hi = key_range(f, 40_000)
        want = oracle.probe(oracle.build(2 ** 18, 6, PackedKeys.fixed(splitmix_hex_keys(77, lo, hi - lo))), 6, probe)
        assert np.array_equal(got, want), f
