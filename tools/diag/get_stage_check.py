"""Which path one get's filter stage takes (lsm_get.candidates_one: the C stage or the Python
loop) and what each costs, on the bench's 16-filter set (bench.py get_set_latency).

Needs tools/microbench/get_latency.so (the same call loop in C, loaded into this process):
    gcc -O2 -fPIC -shared -DGET_LATENCY_LIB -o tools/microbench/get_latency.so \
        tools/microbench/get_latency.c -Iinclude -Lpebbledb_amd -lpebblebloom \
        -Wl,-rpath,'$ORIGIN/../../pebbledb_amd'
"""
import sys
import time

sys.path.insert(0, ".")
from pebbledb_amd import BloomFilter, bloom_filter  # noqa: E402
from pebbledb_amd.keys import splitmix_hex_keys_str  # noqa: E402
from pebbledb_amd.lsm_get import LevelTable, candidates_one, may_contain_set_bits  # noqa: E402

SEED = 0x5EEDB100
ns = [20_000 + 10_000 * i for i in range(16)]
tables, start = [], 0
for n in ns:
    keys = sorted(splitmix_hex_keys_str(SEED, start, n))
    tables.append((keys[0], keys[-1], BloomFilter.build_from_keys_and_fp_rate(keys, 0.001, device=0)))
    start += n
l0 = [bf for _, _, bf in tables[:10]]
levels = [[LevelTable("", "\U0010ffff", bf) for _, _, bf in tables[10:]]]
flat = l0 + [t.bloom_filter for t in levels[0]]
probes = splitmix_hex_keys_str(SEED, start - 500, 1000)
fast = bloom_filter._FAST or bloom_filter._fast()
print("fast handles:", [bf._fast != 0 for bf in flat])
print("C stage result:", fast.candidates_one(probes[0], l0, levels), "python:", candidates_one(probes[0], l0, levels))
import ctypes  # noqa: E402
from pebbledb_amd import _native  # noqa: E402
L = _native.lib()
hs16 = (ctypes.c_void_p * 16)(*[bf._fast for bf in flat])
hs1 = (ctypes.c_void_p * 1)(flat[-1]._fast)
bits = (ctypes.c_uint8 * 8)()
tup16 = tuple(bf._fast for bf in flat)
enc = [p.encode() for p in probes]
for name, fn in (("ctypes set 16", lambda k: L.pbf_may_contain_set(hs16, 16, k.encode(), len(k), bits)),
                 ("ctypes set 1", lambda k: L.pbf_may_contain_set(hs1, 1, k.encode(), len(k), bits)),
                 ("fast.may_contain_set 1", lambda k: fast.may_contain_set((flat[-1]._fast,), k)),
                 ("fast.may_contain_set tuple16", lambda k: fast.may_contain_set(tup16, k)),
                 ("fast.may_contain 1", lambda k: fast.may_contain(flat[-1]._fast, k)),
                 ("C stage", lambda k: fast.candidates_one(k, l0, levels)),
                 ("candidates_one", lambda k: candidates_one(k, l0, levels)),
                 ("may_contain_set_bits", lambda k: may_contain_set_bits(flat, k)),
                 ("fast.may_contain_set", lambda k: fast.may_contain_set([bf._fast for bf in flat], k))):
    for _ in range(200):
        fn(probes[_ % 1000])
    t = time.perf_counter()
    for i in range(5000):
        fn(probes[i % 1000])
    print("%-22s %.2f us" % (name, (time.perf_counter() - t) / 5000 * 1e6))

# the same library call loop in C, inside this process, over these filters
lib = ctypes.CDLL("tools/microbench/get_latency.so")
lib.loop_set.restype = ctypes.c_double
lib.loop_set.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
kb = b"".join(enc)
print("C loop in-process, 16: %.2f us" % lib.loop_set(hs16, 16, kb, 1000, 20000))
print("C loop in-process, 1:  %.2f us" % lib.loop_set(hs1, 1, kb, 1000, 20000))
lib.loop_set_gap.restype = ctypes.c_double
lib.loop_set_gap.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_double]
for gap in (0.0, 0.5, 1.0, 2.0, 4.0):
    print("C loop, gap %.1f us: 16 filters %.2f us, 1 filter %.2f us" % (
        gap, lib.loop_set_gap(hs16, 16, kb, 1000, 20000, gap), lib.loop_set_gap(hs1, 1, kb, 1000, 20000, gap)))
same16 = (flat[-1]._fast,) * 16
for _ in range(200):
    fast.may_contain_set(same16, probes[_])
t = time.perf_counter()
for i in range(5000):
    fast.may_contain_set(same16, probes[i % 1000])
print("fast.may_contain_set one filter x16: %.2f us" % ((time.perf_counter() - t) / 5000 * 1e6))


def dev_stats():
    r, d = ctypes.c_uint64(), ctypes.c_uint64()
    L.pbf_resident_stats(0, ctypes.byref(r), ctypes.byref(d))
    return r.value, d.value


for name, fn in (("fast.may_contain_set tuple16", lambda k: fast.may_contain_set(tup16, k)),
                 ("fast.may_contain 1", lambda k: fast.may_contain(flat[-1]._fast, k))):
    r0, d0 = dev_stats()
    t = time.perf_counter()
    for i in range(5000):
        fn(probes[i % 1000])
    dt = (time.perf_counter() - t) / 5000 * 1e6
    r1, d1 = dev_stats()
    print("%-30s %.2f us per call, device %.2f us" % (name, dt, (d1 - d0) * 1e-3 / max(1, r1 - r0)))
r0, d0 = dev_stats()
print("C loop in-process, 16: %.2f us" % lib.loop_set(hs16, 16, kb, 1000, 20000), end="")
r1, d1 = dev_stats()
print(", device %.2f us" % ((d1 - d0) * 1e-3 / max(1, r1 - r0)))
