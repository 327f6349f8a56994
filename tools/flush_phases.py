"""Phase times of the device SSTable flush (diagnostic; run on the GPU box):
encoded records -> PackedRecords -> plan -> meta -> filter create -> pbf_build_sstable -> file."""
import ctypes
import struct
import sys
import time
from math import ceil, log

import numpy as np

sys.path.insert(0, ".")
from pebbledb_amd import BloomFilter, _native  # noqa: E402
from pebbledb_amd.keys import PackedRecords  # noqa: E402
from pebbledb_amd.sstable_data import key_offsets, meta_blocks, plan_blocks_native  # noqa: E402
from pebbledb_amd.sstable_bloom import sstable_size  # noqa: E402

n, vlen = 1_000_000, 48
rng = np.random.default_rng(0)
vals = rng.integers(0, 256, n * vlen, dtype=np.uint8).tobytes()
enc = [struct.pack("i", 16) + format(i, "016x").encode() + struct.pack("i", vlen) + vals[i * vlen:(i + 1) * vlen]
       for i in range(n)]
state = {}
for rep in range(3):
    t = {}
    t0 = time.perf_counter()
    state.clear()  # drop the previous rep's records, filter and file first (freeing is timed here)
    t["free_previous"] = time.perf_counter()
    pr = PackedRecords.from_encoded(enc)
    t["pack"] = time.perf_counter()
    pk, vb, vo = pr.keys, pr.values, pr.value_offsets
    ko = np.ascontiguousarray(key_offsets(pk), dtype=np.uint64)
    t["key_offsets"] = time.perf_counter()
    bf, bo = plan_blocks_native(ko, vo, 65536)
    t["plan"] = time.perf_counter()
    meta, metas = meta_blocks(pk, bf, bo)
    t["meta"] = time.perf_counter()
    m = (-n * log(0.001)) / (log(2) ** 2)
    nb, k = ceil(m / 8), round((m / n) * log(2))
    bloom = BloomFilter(nb, k)
    t["filter_create"] = time.perf_counter()
    state.update(pr=pr, pk=pk, vb=vb, vo=vo, ko=ko, bloom=bloom)
    del pr, pk, vb, vo, ko, bloom
    pk, vb, vo, ko, bloom = state["pk"], state["vb"], state["vo"], state["ko"], state["bloom"]
    data_len = int(bo[-1])
    out = np.empty(sstable_size(data_len, len(meta), nb), dtype=np.uint8)
    t["file_alloc"] = time.perf_counter()
    buf = out
    vp = ctypes.c_void_p
    _native.check(_native.lib().pbf_build_sstable(bloom.handle, vp(pk.data.ctypes.data), vp(ko.ctypes.data),
                                                  vp(vb.ctypes.data), vp(vo.ctypes.data), n, vp(bf.ctypes.data),
                                                  vp(bo.ctypes.data), len(bf) - 1, vp(buf.ctypes.data),
                                                  vp(buf.ctypes.data + data_len + len(meta))), "build")
    t["device_build"] = time.perf_counter()
    out[data_len:data_len + len(meta)] = np.frombuffer(meta, dtype=np.uint8)
    t["assemble"] = time.perf_counter()
    state["out"] = out
    del out, pk, vb, vo, ko, bloom, buf
    prev = t0
    parts = []
    for name, v in t.items():
        parts.append(f"{name} {1e3 * (v - prev):.1f}")
        prev = v
    print(f"rep {rep}: total {1e3 * (prev - t0):.1f} ms: " + ", ".join(parts), flush=True)
