"""Resident reader under filter churn: reader threads run gets (may_contain_set over the current
filters) while a writer thread keeps building new filters of other sizes and dropping old ones,
as flushes and compactions do to an LSM's SSTables.  A dropped filter is destroyed once the last
reader holding it lets go (Python references), its descriptor-table index goes back to the board
and the epoch moves on; new filters take freed indexes.  Every answer is checked against the
oracle's answer for that filter, computed when the filter was published.

    python tools/diag/reader_churn.py [seconds] [readers]
"""
import sys
import threading
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

from oracle.oracle import COracle  # noqa: E402
from pebbledb_amd import BloomFilter, PackedKeys, may_contain_set  # noqa: E402
from pebbledb_amd.keys import splitmix_hex_keys  # noqa: E402

K = 7
NPROBE = 64
NLIVE = 24


def run(seconds: float = 10.0, readers: int = 8) -> dict:
    o = COracle()
    probe_arr = splitmix_hex_keys(900, 0, NPROBE)
    probe_pk = PackedKeys.fixed(probe_arr)
    probe_keys = [probe_pk.key(i).decode() for i in range(NPROBE)]
    lock = threading.Lock()
    gen = [0]

    def make(i):
        nb = 300 + 97 * (i % 50) + 13 * i
        members = np.concatenate([splitmix_hex_keys(1000 + i, 0, 400), probe_arr[i % 8::8]])
        pk = PackedKeys.fixed(members)
        bf = BloomFilter(nb, K)
        bf.add_many(pk)
        bf.sync()
        want = np.unpackbits(o.probe(o.build(nb, K, pk), K, probe_pk), bitorder="little")[:NPROBE].astype(bool)
        return bf, want

    live = [make(i) for i in range(NLIVE)]
    gen[0] = NLIVE
    stop = threading.Event()
    stats = {"gets": 0, "churn": 0, "errors": []}

    def reader(seed):
        rng = np.random.default_rng(seed)
        n = 0
        try:
            while not stop.is_set():
                with lock:
                    snap = list(live)
                sub = [snap[j] for j in rng.choice(len(snap), size=int(rng.integers(1, 20)), replace=False)]
                q = int(rng.integers(0, NPROBE))
                got = may_contain_set([bf for bf, _ in sub], probe_keys[q])
                exp = [bool(w[q]) for _, w in sub]
                if got != exp:
                    stats["errors"].append((q, got, exp))
                    stop.set()
                n += 1
        except Exception as e:  # noqa: BLE001
            stats["errors"].append(repr(e))
            stop.set()
        with lock:
            stats["gets"] += n

    def writer():
        try:
            while not stop.is_set():
                f = make(gen[0])
                gen[0] += 1
                with lock:
                    live[gen[0] % NLIVE] = f  # the replaced filter dies with its last reference
                stats["churn"] += 1
        except Exception as e:  # noqa: BLE001
            stats["errors"].append(repr(e))
            stop.set()

    ts = [threading.Thread(target=reader, args=(s,)) for s in range(readers)] + [threading.Thread(target=writer)]
    for t in ts:
        t.start()
    t0 = time.time()
    while time.time() - t0 < seconds and not stop.is_set():
        time.sleep(0.2)
    stop.set()
    for t in ts:
        t.join()
    return stats


if __name__ == "__main__":
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    st = run(secs, nr)
    print(f"gets {st['gets']}, filters replaced {st['churn']}, errors {len(st['errors'])}: {st['errors'][:3]}")
    sys.exit(1 if st["errors"] else 0)
