"""Diagnostic (GPU box): the cost of BloomFilter creation inside a flush-sized process, with and
without Python's cyclic GC, next to a bare create loop (profiles/r02/s9/create_in_flush.txt)."""
import gc
import struct
import sys
import time

sys.path.insert(0, ".")
from pebbledb_amd import BloomFilter  # noqa: E402

nb, k = 1797198, 10
for rep in range(3):
    t = time.perf_counter(); b = BloomFilter(nb, k); b.sync() if hasattr(b, "sync") else None
    print(f"bare create {1e3 * (time.perf_counter() - t):.2f} ms"); del b
enc = [struct.pack("i", 16) + format(i, "016x").encode() + struct.pack("i", 48) + bytes(48) for i in range(1_000_000)]
for mode in ("gc on", "gc off"):
    if mode == "gc off":
        gc.disable()
    for rep in range(3):
        junk = [[i] for i in range(20000)]  # container allocations, as the flush's Python code makes
        t = time.perf_counter(); b = BloomFilter(nb, k)
        print(f"{mode}: create {1e3 * (time.perf_counter() - t):.2f} ms"); del b, junk
    t = time.perf_counter(); gc.collect(); print(f"{mode}: full gc.collect {1e3 * (time.perf_counter() - t):.2f} ms")
