"""The RCCL branch of the multi-GPU code on a one-GPU box (`-m gpu`): an RCCL process group of one
rank (RCCL refuses two ranks on one device, so world 1 is what a single MI355X can run).  The
8-GPU job's collectives are the bench's barrier and max-over-ranks (bench.py all_reduce_scalar)
and, for C5's key-partitioned layout, the one-time replication of the filters
(shard.exchange_bitmaps: pbf_get_bitmap_device into a device buffer, all_gather_into_tensor,
pbf_set_bitmap_device from the gathered buffer).  Here each runs over RCCL on device tensors, and
bitmaps that went through the all-gather and back into filters equal their sources and the
oracle.  (Ranks on several devices run only on the driver's 8-GPU node.)"""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, '.')
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    from pebbledb_amd import BloomFilter, PackedKeys
    from pebbledb_amd.keys import splitmix_hex_keys
    from pebbledb_amd.shard import exchange_bitmaps
    from oracle.oracle import COracle

    torch.cuda.set_device(0)
    dist.init_process_group(backend="nccl", init_method="env://", device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    o = COracle()
    nb, k, nf = 1 << 20, 6, 3
    sets = [PackedKeys.fixed(splitmix_hex_keys(50 + f, 0, 200000)) for f in range(nf)]
    filters = []
    for s in sets:
        bf = BloomFilter(nb, k, device=0)
        bf.add_many(s)
        bf.sync()
        filters.append(bf)
    want = [o.build(nb, k, s, omp=True).tobytes() for s in sets]
    assert [bf.bitmap() for bf in filters] == want

    # the bench's timing plumbing over RCCL
    dist.barrier()
    assert bench.all_reduce_scalar(torch, dist, 2.5, dist.ReduceOp.MAX, torch.float64) == 2.5

    # the replication exactly as bench.py's C5 keys layout drives it
    stream = torch.cuda.current_stream().cuda_stream
    def export(g, t):
        filters[g].bitmap_to_device(t.data_ptr())
        filters[g].sync()
    def load(g, t):
        filters[g] = BloomFilter.from_device_bitmap(t.data_ptr(), nb, k, device=0, stream=stream)
        filters[g].sync()
    info = exchange_bitmaps(dist, torch, nf, nb, export, load, device=0)
    assert info["collective"] == "all_gather (RCCL)" and info["bytes_received"] == 0, info

    # the same primitives with the gathered buffer loaded back (at world 1 exchange_bitmaps has
    # no other rank's filter to load)
    send = torch.empty(nf * nb, dtype=torch.uint8, device="cuda")
    for g in range(nf):
        export(g, send[g * nb:(g + 1) * nb])
    recv = torch.empty_like(send)
    dist.all_gather_into_tensor(recv, send)
    torch.cuda.synchronize()
    back = [BloomFilter.from_device_bitmap(recv[g * nb:(g + 1) * nb].data_ptr(), nb, k, device=0, stream=stream)
            for g in range(nf)]
    for g, bf in enumerate(back):
        bf.sync()
        assert bf.bitmap() == want[g], g
        q = sets[g]
        assert np.array_equal(bf.may_contain_many(q, packed=True), o.probe(np.frombuffer(want[g], dtype=np.uint8), k, q))
    dist.barrier()
    dist.destroy_process_group()
    print("ok")
""")


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_one_rank_barrier_max_and_replication():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
