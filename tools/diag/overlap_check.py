"""Would a build and a probe on different streams overlap?  C2's build pass (10M keys into filter A)
and C2's probe pass (20M keys against an already built filter B), each on its filter's own pooled
stream: issued one after the other with a sync between, and issued together (both in flight).
If together ~= the sum, the kernels (each a whole-CU-LDS partition or a tile pass over every CU)
serialise on the device and there is nothing to gain from overlapping them in one filter's step."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from pebbledb_amd import BloomFilter, _native  # noqa: E402

L = _native.lib()
n = 10_000_000
keys = torch.empty(2 * n * 16, dtype=torch.uint8, device="cuda")
_native.check(L.pbf_gen_splitmix_hex(0, None, keys.data_ptr(), 0x5EEDB100, 0, 2 * n), "gen")
keys_b = torch.empty(2 * n * 16, dtype=torch.uint8, device="cuda")
_native.check(L.pbf_gen_splitmix_hex(0, None, keys_b.data_ptr(), 0x5EEDB100, 2 * n, 2 * n), "gen")
hm = torch.zeros((2 * n + 7) // 8, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
A = BloomFilter(1 << 27, 6, device=0)
B = BloomFilter(1 << 27, 6, device=0)
B.add_device_fixed(keys_b.data_ptr(), 16, n)
B.sync()
print("streams differ:", A.stream != B.stream)


def build():
    A.clear()
    A.add_device_fixed(keys.data_ptr(), 16, n)


def probe():
    B.probe_device_fixed(keys_b.data_ptr(), 16, 2 * n, hm.data_ptr())


for _ in range(5):
    build(); probe(); A.sync(); B.sync()
res = {}
for name in ("build alone", "probe alone", "sequential", "together"):
    ts = []
    for _ in range(30):
        torch.cuda.synchronize()
        t = time.perf_counter()
        if name == "build alone":
            build(); A.sync()
        elif name == "probe alone":
            probe(); B.sync()
        elif name == "sequential":
            build(); A.sync(); probe(); B.sync()
        else:
            build(); probe(); A.sync(); B.sync()
        ts.append((time.perf_counter() - t) * 1e3)
    ts.sort()
    res[name] = ts[len(ts) // 2]
    print("%-12s %.3f ms (median of 30, wall)" % (name, res[name]))

# steady state, no host syncs inside: 50 x (build A, probe B) on two streams vs 50 x (build A,
# probe A) on A's stream (the bench step)
for name in ("one stream (build A, probe A)", "two streams (build A, probe B)"):
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(50):
            build()
            if name.startswith("one"):
                A.probe_device_fixed(keys.data_ptr(), 16, 2 * n, hm.data_ptr())
            else:
                probe()
        A.sync(); B.sync()
        ms = (time.perf_counter() - t) * 1e3 / 50
    print("%-32s %.3f ms per build+probe (wall, steady state)" % (name, ms))
