"""The drop-in surface under the reference's calling patterns (runs on an MI355X, `-m gpu`):
per-key may_contain (LsmStorage.get, src/lsm_storage.py:165,175) through the one-key launch,
reader threads sharing one filter without a lock (lsm_storage.py:153-179), host staging in
chunks smaller than one hit-mask byte's worth of keys, and the pooled working memory."""
import os
import subprocess
import sys
import textwrap
import threading

import numpy as np
import pytest

from pebbledb_amd import BloomFilter, PackedKeys, may_contain_multi
from pebbledb_amd import _native
from pebbledb_amd.keys import splitmix_hex_keys, varlen_keys

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _strs(pk: PackedKeys) -> list[str]:
    return [pk.key(i).decode("utf-8") for i in range(pk.n)]


def test_one_key_may_contain_matches_oracle(oracle):
    """pbf_may_contain (one launch, key via mapped pinned memory) == the oracle, over fixed,
    variable-length, empty, non-ASCII and > 4096-byte keys, for power-of-two and floor-mod m."""
    d, o = varlen_keys(5, 0, 3000)
    members = PackedKeys(d, 3000, offsets=o)
    extra = ["", "é", "ключ", "🔑" * 3, "x" * 5000, "y" * 4096, "z" * 4097]
    # the resident reader's head carries keys of up to 76 bytes; longer ones (to 1 KiB) come from
    # the slot body, longer still take the launch
    extra += [("%d-" % n) + "k" * (n - len("%d-" % n)) for n in (15, 16, 17, 47, 48, 49, 75, 76, 77, 78, 100, 1023,
                                                                   1024, 1025)]
    extra += ["é" * 38, "é" * 39]  # 76 / 78 UTF-8 bytes
    keys = _strs(members) + extra
    probes = keys + [s + "!" for s in keys[:1500]] + ["absent-%d" % i for i in range(500)]
    for nb, k in ((2 ** 14, 6), (100_003, 7), (777, 3), (64, 40)):
        bf = BloomFilter(nb, k)
        bf.add_many(keys)
        want = oracle.build(nb, k, PackedKeys.from_strs(keys))
        assert bf.bitmap() == want.tobytes()
        want_hm = np.unpackbits(oracle.probe(want, k, PackedKeys.from_strs(probes)), bitorder="little")
        got = [bf.may_contain(s) for s in probes]
        assert got == [bool(x) for x in want_hm[:len(probes)]], (nb, k)
        assert bf.last_probe_detail & _native.PBF_DETAIL_ONE_KEY or len(probes[-1]) > 4096
        if k <= 32:  # a short key of a built filter: the resident reader answered (no launch)
            assert bf.may_contain(keys[0])
            assert bf.last_probe_detail & _native.PBF_DETAIL_RESIDENT


def test_reader_threads_share_one_filter(oracle):
    """Eight threads call may_contain / may_contain_many on ONE filter at once (the reference's
    reader threads, no lock) while a ninth adds keys to another filter: every answer equals the
    oracle's."""
    n = 50_000
    pk = PackedKeys.fixed(splitmix_hex_keys(11, 0, n))
    bf = BloomFilter(2 ** 16, 5)
    bf.add_many(pk)
    want = oracle.build(2 ** 16, 5, pk)
    q = PackedKeys.fixed(splitmix_hex_keys(11, n // 2, n))
    want_hm = oracle.probe(want, 5, q)
    want_bits = np.unpackbits(want_hm, bitorder="little")[:n]
    qs = _strs(q)
    errors = []

    def reader(t):
        try:
            for rep in range(3):
                if (t + rep) % 2:
                    got = bf.may_contain_many(q, packed=True)
                    if not np.array_equal(got, want_hm):
                        errors.append(("batch", t))
                else:
                    for i in range(t, n, 97):
                        if bf.may_contain(qs[i]) != bool(want_bits[i]):
                            errors.append(("key", t, i))
                            break
        except Exception as e:  # pragma: no cover - reported below
            errors.append(("exc", t, repr(e)))

    other = BloomFilter(2 ** 16, 5)

    def writer():
        for i in range(0, n, 5000):
            other.add_many(PackedKeys.fixed(splitmix_hex_keys(11, i, 5000)))

    th = [threading.Thread(target=reader, args=(t,)) for t in range(8)] + [threading.Thread(target=writer)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errors, errors[:5]
    assert other.bitmap() == want.tobytes()
    # concurrent add() buffering on one filter from several threads
    shared = BloomFilter(2 ** 16, 5)
    strs = _strs(pk)

    def adder(t):
        for s in strs[t::4]:
            shared.add(s)

    th = [threading.Thread(target=adder, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert shared.bitmap() == want.tobytes()


def test_stage_chunks_smaller_than_a_hitmask_byte(oracle):
    """PBF_STAGE_BYTES smaller than 64 keys' worth of bytes: every host-staged chunk but the last
    still holds a multiple of 64 keys, so hit-mask bytes never straddle chunks (single and
    multi-filter probes; fixed and variable-length keys)."""
    code = textwrap.dedent("""
        import numpy as np, sys
        sys.path.insert(0, '.')
        from pebbledb_amd import BloomFilter, PackedKeys, may_contain_multi
        from pebbledb_amd.keys import splitmix_hex_keys, varlen_keys
        from oracle.oracle import COracle
        o = COracle()
        fx = PackedKeys.fixed(splitmix_hex_keys(3, 0, 3001))
        d, off = varlen_keys(3, 0, 3001)
        vr = PackedKeys(d, 3001, offsets=off)
        for pk in (fx, vr):
            fs = []
            for mode in (1, 2):
                bf = BloomFilter(50000, 6); bf.set_build_mode(mode); bf.add_many(pk)
                want = o.build(50000, 6, pk)
                assert bf.bitmap() == want.tobytes()
                for pm in (1, 2):
                    bf.set_probe_mode(pm)
                    assert np.array_equal(bf.may_contain_many(pk, packed=True), o.probe(want, 6, pk))
                fs.append(bf)
            m = may_contain_multi(fs, pk)
            assert np.array_equal(m[0], o.probe(want, 6, pk)) and np.array_equal(m[1], m[0])
        print('ok')
    """)
    env = dict(os.environ, PBF_STAGE_BYTES="200")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_scratch_is_pooled_not_per_filter(oracle):
    """Working memory is a per-device pool: building and probing many filters leaves the pool at
    the size of the largest single pipeline (not growing with the number of filters), each
    filter holding only its bitmap; pbf_trim releases the pool and later calls still work."""
    L = _native.lib()

    def pool_bytes():
        v = _native._u64(0)
        _native.check(L.pbf_scratch_bytes(0, __import__("ctypes").byref(v)), "scratch")
        return v.value

    pk = PackedKeys.fixed(splitmix_hex_keys(4, 0, 300_000))
    want = oracle.build(2 ** 20, 6, pk)
    fs = []
    sizes = []
    for i in range(12):
        bf = BloomFilter(2 ** 20, 6)
        bf.set_build_mode(2)
        bf.set_probe_mode(2)
        bf.add_many(pk)
        assert np.array_equal(bf.may_contain_many(pk, packed=True)[:1000], np.full(1000, 0xFF, np.uint8))
        fs.append(bf)
        sizes.append(pool_bytes())
    assert max(sizes[4:]) <= max(sizes[:4]), sizes  # bounded by the pipeline, not by the filter count
    _native.check(L.pbf_trim(0), "trim")
    assert pool_bytes() == 0
    for bf in fs[:3]:
        assert bf.bitmap() == want.tobytes()
        assert bf.may_contain_many(pk).all()


def test_shared_readers_beside_a_writer_on_the_same_filter(oracle):
    """Readers hold a built filter's lock shared (one-key probes on reader streams) while a writer
    on the SAME handle re-adds keys that are already members and runs batch probes (exclusive);
    every one-key and set answer equals the oracle's, and the handle records the one-key path."""
    from pebbledb_amd import may_contain_set
    n = 40_000
    pk = PackedKeys.fixed(splitmix_hex_keys(21, 0, n))
    bf = BloomFilter(2 ** 17, 6)
    bf.add_many(pk)
    small = BloomFilter(4099, 3)
    small.add_many(PackedKeys.fixed(splitmix_hex_keys(21, 0, 1000)))
    want = oracle.build(2 ** 17, 6, pk)
    want_small = oracle.build(4099, 3, PackedKeys.fixed(splitmix_hex_keys(21, 0, 1000)))
    q = PackedKeys.fixed(splitmix_hex_keys(21, n // 2, n))
    wb = np.unpackbits(oracle.probe(want, 6, q), bitorder="little")[:n]
    ws = np.unpackbits(oracle.probe(want_small, 3, q), bitorder="little")[:n]
    qs = _strs(q)
    errors = []
    stop = threading.Event()

    def reader(t):
        try:
            for i in range(t, n, 53):
                if bf.may_contain(qs[i]) != bool(wb[i]):
                    errors.append(("key", t, i))
                    return
                if i % 5 == 0:
                    got = may_contain_set([bf, small, bf], qs[i])
                    if got != [bool(wb[i]), bool(ws[i]), bool(wb[i])]:
                        errors.append(("set", t, i, got))
                        return
        except Exception as e:  # pragma: no cover
            errors.append(("exc", t, repr(e)))

    def writer():
        try:
            while not stop.is_set():
                bf.add_many(PackedKeys.fixed(splitmix_hex_keys(21, 0, 2000)))  # members again: no bit changes
                if not np.array_equal(bf.may_contain_many(q, packed=True)[:100], oracle.probe(want, 6, q)[:100]):
                    errors.append(("batch",))
        except Exception as e:  # pragma: no cover
            errors.append(("wexc", repr(e)))

    w = threading.Thread(target=writer)
    th = [threading.Thread(target=reader, args=(t,)) for t in range(8)]
    w.start()
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    stop.set()
    w.join(timeout=300)
    assert not errors, errors[:5]
    assert bf.bitmap() == want.tobytes()
    assert bf.may_contain(qs[0]) == bool(wb[0])
    # a built, idle filter: the one-key probe ran under the shared lock, answered by the
    # resident reader wave
    assert bf.last_probe_detail == (_native.PBF_DETAIL_ONE_KEY | _native.PBF_DETAIL_SHARED
                                    | _native.PBF_DETAIL_RESIDENT)


def test_shared_readers_see_keys_a_writer_added(oracle):
    """Round-4 advice: a writer adds NEW keys (bits change) and then signals; reader threads then
    probe those keys and must all hit — whether their call finds the add still queued on the
    filter's stream (the exclusive path, ordered after it) or finished (the shared path)."""
    n0, n1 = 50_000, 20_000
    bf = BloomFilter(2 ** 18, 6)
    bf.add_many(PackedKeys.fixed(splitmix_hex_keys(91, 0, n0)))
    bf.sync()
    new = _strs(PackedKeys.fixed(splitmix_hex_keys(91, n0, n1)))
    rounds = 6
    added = [threading.Event() for _ in range(rounds)]
    errors = []

    def writer():
        for r in range(rounds):
            bf.add_many(new[r * (n1 // rounds):(r + 1) * (n1 // rounds)])
            added[r].set()

    def reader(t):
        try:
            for r in range(rounds):
                added[r].wait(timeout=120)
                for i in range(r * (n1 // rounds) + t, (r + 1) * (n1 // rounds), 97):
                    if not bf.may_contain(new[i]):
                        errors.append((t, r, i))
                        return
        except Exception as e:  # pragma: no cover
            errors.append(("exc", t, repr(e)))

    th = [threading.Thread(target=reader, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    w = threading.Thread(target=writer)
    w.start()
    w.join(timeout=300)
    for t in th:
        t.join(timeout=300)
    assert not errors, errors[:5]
    want = oracle.build(2 ** 18, 6, PackedKeys.fixed(splitmix_hex_keys(91, 0, n0 + (n1 // rounds) * rounds)))
    assert bf.bitmap() == want.tobytes()


def test_one_key_probe_exclusive_fallback_in_a_subprocess():
    """PBF_SHARED_READERS=0 sends one-key probes through the exclusive path: the handle records
    the one-key launch without the shared flag (the same answers)."""
    code = ("import sys; sys.path.insert(0, '.'); from pebbledb_amd import BloomFilter, _native\n"
            "bf = BloomFilter(4096, 4); bf.add('a'); bf.sync()\n"
            "assert bf.may_contain('a')\n"
            "print(bf.last_probe_detail == _native.PBF_DETAIL_ONE_KEY)")
    env = dict(os.environ, PBF_SHARED_READERS="0")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == "True"


def test_wait_stream_orders_a_torch_producer_without_sync(oracle):
    """Device keys produced by torch on a side stream (behind a queue of long matmuls, so the copy
    lands late): pbf_wait_stream orders the filter's add after them with no torch.cuda.synchronize;
    the bitmap equals the oracle's.  pbf_signal_stream hands the probe's device hit mask back to
    a torch stream, which reads it without waiting on the host."""
    torch = pytest.importorskip("torch")
    n = 300_000
    host = splitmix_hex_keys(31, 0, n)
    src = torch.from_numpy(host.reshape(-1)).cuda()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda")
    dst = torch.zeros_like(src)
    with torch.cuda.stream(side):
        for _ in range(20):  # ~ms of work ahead of the copy on the producer's stream
            a = a @ a
            a = a / a.norm()
        dst.copy_(src)
    bf = BloomFilter(2 ** 20, 6)
    bf.set_build_mode(_native.PBF_BUILD_ATOMIC)
    bf.wait_stream(side.cuda_stream)
    bf.add_device_fixed(dst.data_ptr(), 16, n)
    want = oracle.build(2 ** 20, 6, PackedKeys.fixed(host))
    assert bf.bitmap() == want.tobytes()
    # consumer side: the hit mask produced on the filter's stream, read on a torch stream
    q = torch.from_numpy(splitmix_hex_keys(31, n // 2, n).reshape(-1)).cuda()
    torch.cuda.synchronize()
    hm = torch.zeros((n + 7) // 8, dtype=torch.uint8, device="cuda")
    consumer = torch.cuda.Stream()
    bf.probe_device_fixed(q.data_ptr(), 16, n, hm.data_ptr())
    bf.signal_stream(consumer.cuda_stream)
    with torch.cuda.stream(consumer):
        copy = hm.clone()
    consumer.synchronize()
    want_hm = oracle.probe(want, 6, PackedKeys.fixed(splitmix_hex_keys(31, n // 2, n)))
    assert np.array_equal(copy.cpu().numpy(), want_hm)
    bf.sync()


def _run_py(code: str, env_extra: dict) -> str:
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.strip().splitlines()[-1]


def test_resident_reader_off_launches_per_key_in_a_subprocess():
    """PBF_RESIDENT_READER=0: the shared one-key probe launches per key (no resident flag), with
    the same answers."""
    code = ("import sys; sys.path.insert(0, '.'); from pebbledb_amd import BloomFilter, _native\n"
            "bf = BloomFilter(4096, 4); bf.add_many(['a', 'b']); bf.sync()\n"
            "assert bf.may_contain('a') and bf.may_contain('b')\n"
            "print(bf.last_probe_detail == _native.PBF_DETAIL_ONE_KEY | _native.PBF_DETAIL_SHARED)")
    assert _run_py(code, {"PBF_RESIDENT_READER": "0"}) == "True"


def test_resident_reader_relaunches_after_idle_in_a_subprocess():
    """With a 50 us idle time the resident wave leaves between keys separated by 2 ms sleeps and
    is relaunched by the next key: every answer still equals the per-key launch's, and the wave
    was started more than once."""
    code = textwrap.dedent("""
        import sys, time, ctypes; sys.path.insert(0, '.')
        from pebbledb_amd import BloomFilter, _native
        from pebbledb_amd.keys import splitmix_hex_keys_str
        keys = splitmix_hex_keys_str(7, 0, 2000)
        bf = BloomFilter(2 ** 12, 5); bf.add_many(keys); bf.sync()
        probes = splitmix_hex_keys_str(7, 1000, 200)
        got = []
        for i, p in enumerate(probes):
            got.append(bf.may_contain(p))
            assert bf.last_probe_detail & _native.PBF_DETAIL_RESIDENT
            if i % 20 == 0:
                time.sleep(0.002)
        n = ctypes.c_uint32(0)
        _native.check(_native.lib().pbf_resident_launches(bf.device, ctypes.byref(n)))
        print(n.value, ''.join('1' if g else '0' for g in got))
    """)
    out = _run_py(code, {"PBF_RESIDENT_IDLE_US": "50"})
    launches, bits = out.split()
    code0 = textwrap.dedent("""
        import sys; sys.path.insert(0, '.')
        from pebbledb_amd import BloomFilter
        from pebbledb_amd.keys import splitmix_hex_keys_str
        keys = splitmix_hex_keys_str(7, 0, 2000)
        bf = BloomFilter(2 ** 12, 5); bf.add_many(keys); bf.sync()
        print(''.join('1' if bf.may_contain(p) else '0' for p in splitmix_hex_keys_str(7, 1000, 200)))
    """)
    assert _run_py(code0, {"PBF_RESIDENT_READER": "0"}) == bits
    assert bits == "1" * 200  # probes are keys 1000..1199 of the 2000 members
    assert int(launches) >= 2


def test_more_threads_than_resident_slots(oracle):
    """80 threads probe one filter at once: the first 64 hold resident slots, the rest launch per
    key; every answer equals the oracle's."""
    n = 20_000
    pk = PackedKeys.fixed(splitmix_hex_keys(17, 0, n))
    bf = BloomFilter(2 ** 15, 6)
    bf.add_many(pk)
    bf.sync()
    want = np.unpackbits(oracle.probe(oracle.build(2 ** 15, 6, pk), 6, pk), bitorder="little")[:n]
    qs = _strs(pk)
    errors = []
    barrier = threading.Barrier(80)

    def reader(t):
        try:
            barrier.wait(timeout=120)
            for i in range(t, n, 397):
                if bf.may_contain(qs[i]) != bool(want[i]):
                    errors.append((t, i))
                    return
        except Exception as e:  # pragma: no cover
            errors.append(("exc", t, repr(e)))

    th = [threading.Thread(target=reader, args=(t,)) for t in range(80)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errors, errors[:5]


def test_partitions_planned_around_a_live_reader_in_a_subprocess(oracle):
    """While the resident reader is live the tiled build / probe plan 31 partition workgroups per
    XCD (groups_cap); PBF_SPARE_CU=1 forces that planning: builds equal the oracle and tiled probes
    equal direct ones, for the ring (m = 2^30) and the counting-sort (variable-length) partitions."""
    code = textwrap.dedent("""
        import sys, numpy as np; sys.path.insert(0, '.')
        from pebbledb_amd import BloomFilter, PackedKeys
        from pebbledb_amd.keys import splitmix_hex_keys, varlen_keys
        from oracle.oracle import COracle
        o = COracle()
        fx = PackedKeys.fixed(splitmix_hex_keys(61, 0, 3_000_000))
        q = PackedKeys.fixed(splitmix_hex_keys(61, 1_500_000, 3_000_000))
        d, off = varlen_keys(62, 0, 600_000)
        vr = PackedKeys(d, 600_000, offsets=off)
        for nb, k, keys, probes in ((2 ** 27, 6, fx, q), (3 * 2 ** 22 + 5, 8, vr, vr)):
            bf = BloomFilter(nb, k); bf.set_build_mode(2); bf.add_many(keys)
            assert bf.bitmap() == o.build(nb, k, keys, omp=True).tobytes(), nb
            bf.set_probe_mode(2); t = bf.may_contain_many(probes, packed=True)
            bf.set_probe_mode(1); dr = bf.may_contain_many(probes, packed=True)
            assert np.array_equal(t, dr), nb
        print('ok')
    """)
    assert _run_py(code, {"PBF_SPARE_CU": "1"}) == "ok"


def test_resident_descriptor_indexes_cached_and_reused(oracle):
    """The resident reader names filters by descriptor-table index and caches their descriptors
    in LDS (reader_service.hpp): 300 filters of different sizes (more than the 256 cache entries,
    so indexes collide), gets over sets of 64 (indexes past the 16th travel in the slot body), then
    100 filters destroyed and 100 new ones of OTHER sizes built, which take the freed indexes: the
    epoch must keep the cache from answering with a destroyed filter's descriptor.  Every answer
    equals the oracle's."""
    import gc
    from pebbledb_amd import may_contain_set
    k = 7

    def make(i, gen):
        nb = 211 + 37 * i + 1009 * gen  # every filter a different m, and a new one per generation
        members = PackedKeys.fixed(splitmix_hex_keys(70 + gen, 1000 * i, 150))
        bf = BloomFilter(nb, k)
        bf.add_many(members)
        return bf, oracle.build(nb, k, members)

    def check(filters, bitmaps, probes):
        q = PackedKeys.fixed(probes)
        want = [np.unpackbits(oracle.probe(bm, k, q), bitorder="little")[:q.n] for bm in bitmaps]
        keys = _strs(q)
        for j, key in enumerate(keys):
            f = j % len(filters)
            assert filters[f].may_contain(key) == bool(want[f][j]), (f, key)
        for j, key in enumerate(keys[:60]):
            base = (7 * j) % (len(filters) - 64)
            got = may_contain_set(filters[base:base + 64], key)
            assert got == [bool(want[base + t][j]) for t in range(64)], (base, key)

    pairs = [make(i, 0) for i in range(300)]
    filters, bitmaps = [p[0] for p in pairs], [p[1] for p in pairs]
    # probes: members of some filters and keys of none
    probes = np.concatenate([splitmix_hex_keys(70, 1000 * i, 3) for i in range(0, 300, 2)] +
                            [splitmix_hex_keys(99, 0, 300)])
    check(filters, bitmaps, probes)
    del pairs
    for i in range(100):  # destroy: the indexes go back to the table
        filters[i] = None
    gc.collect()
    fresh = [make(i, 1) for i in range(100)]
    for i in range(100):
        filters[i], bitmaps[i] = fresh[i]
    del fresh
    probes = np.concatenate([splitmix_hex_keys(71, 1000 * i, 3) for i in range(100)] +
                            [splitmix_hex_keys(70, 1000 * i, 2) for i in range(100, 300, 3)] +
                            [splitmix_hex_keys(98, 0, 300)])
    import ctypes
    r0, d0 = ctypes.c_uint64(), ctypes.c_uint64()
    _native.check(_native.lib().pbf_resident_stats(filters[0].device, ctypes.byref(r0), ctypes.byref(d0)))
    check(filters, bitmaps, probes)
    assert filters[0].last_probe_detail & _native.PBF_DETAIL_RESIDENT
    r1, d1 = ctypes.c_uint64(), ctypes.c_uint64()
    _native.check(_native.lib().pbf_resident_stats(filters[0].device, ctypes.byref(r1), ctypes.byref(d1)))
    # every probe above was answered by the wave, each in well under a millisecond of its time
    assert r1.value - r0.value >= probes.shape[0] + 60
    assert 0 < d1.value - d0.value < (r1.value - r0.value) * 1_000_000


def test_resident_reader_under_filter_churn():
    """Reader threads run gets over the current filters while a writer keeps replacing them with
    filters of other sizes (an LSM's flushes and compactions): replaced filters are destroyed when
    their last reader lets go, their descriptor indexes are reused under a new epoch, and every
    answer equals the oracle's (tools/diag/reader_churn.py; 20 s runs: ~1M gets, ~40k
    replacements, no error -- profiles/r06/perkey/s25_churn.log)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("reader_churn", os.path.join(REPO, "tools", "diag", "reader_churn.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    st = mod.run(seconds=4.0, readers=8)
    assert not st["errors"], st["errors"][:3]
    assert st["gets"] > 1000 and st["churn"] > 50, st
