"""Diagnostic (GPU): replicate a filter, then change the source; report whether the replica
changed and whether the two handles share a bitmap."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle.oracle import COracle  # noqa: E402
from pebbledb_amd import BloomFilter, PackedKeys, _native  # noqa: E402
from pebbledb_amd.keys import splitmix_hex_keys  # noqa: E402

o = COracle()
L = _native.lib()
n, nb, k = 300_000, 2 ** 20 + 12, 7
host = PackedKeys.fixed(splitmix_hex_keys(31, 0, n))
want = o.build(nb, k, host).tobytes()
src = BloomFilter(nb, k)
src.add_many(host)
print("src ok", src.bitmap() == want)
for bounce in (False, True, False):
    r = src.replicate(0, bounce=bounce)
    print("bounce", bounce, "replica ok", r.bitmap() == want,
          "ptrs", hex(L.pbf_device_bitmap(src.handle) or 0), hex(L.pbf_device_bitmap(r.handle) or 0))
src.add_many(PackedKeys.fixed(splitmix_hex_keys(31, 10 ** 9, 50_000)))
a, b = np.frombuffer(r.bitmap(), np.uint8), np.frombuffer(src.bitmap(), np.uint8)
w = np.frombuffer(want, np.uint8)
d = np.flatnonzero(a != w)
print("after src change: replica == want", len(d) == 0, "diff bytes", len(d), "first", d[:10],
      "replica == src", bool((a == b).all()), "src changed", bool((b != w).any()))
if len(d):
    print("replica bytes at diff", a[d[:10]], "want", w[d[:10]], "src", b[d[:10]])
