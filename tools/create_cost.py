"""Diagnostic: what a filter's creation costs (pbf_create pieces), on the GPU box."""
import ctypes
import sys
import time

sys.path.insert(0, ".")
from pebbledb_amd import BloomFilter, _native  # noqa: E402

L = _native.lib()
keep = []
for nb in (1024, 1_797_199, 2 ** 27):
    ts = []
    for i in range(6):
        t0 = time.perf_counter()
        h = ctypes.c_void_p()
        _native.check(L.pbf_create(0, nb, 10, ctypes.byref(h)), "create")
        t1 = time.perf_counter()
        _native.check(L.pbf_sync(h), "sync")
        t2 = time.perf_counter()
        keep.append(h)
        ts.append((1e3 * (t1 - t0), 1e3 * (t2 - t1)))
    print(f"nb_bytes {nb}: create / sync ms: " + " ".join(f"{a:.2f}/{b:.2f}" for a, b in ts), flush=True)
t0 = time.perf_counter()
bfs = [BloomFilter(1_797_199, 10) for _ in range(10)]
print(f"10 x BloomFilter(1797199, 10): {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
