"""Multi-filter probe (pbf_probe_multi): one key batch against several SSTable filters, the
batched form of LsmStorage.get's filter checks (src/lsm_storage.py:164-175; SURVEY.md §8 a-14,
config C5).  Every hit mask must equal the filter's own single probe and the oracle's."""
import numpy as np
import pytest

from pebbledb_amd import BloomFilter, PackedKeys, may_contain_multi, may_contain_set, probe_multi_device
from pebbledb_amd import _native
from pebbledb_amd._native import PBF_PROBE_DIRECT, PBF_PROBE_TILED
from pebbledb_amd.keys import splitmix_hex_keys, varlen_keys

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SEED = 0x5EEDB100


def _filters(oracle, nb, k, n_per, count, mode=None, seed=SEED):
    fs, want = [], []
    for f in range(count):
        pk = PackedKeys.fixed(splitmix_hex_keys(seed, f * n_per, n_per))
        bf = BloomFilter(nb, k)
        bf.add_many(pk)
        if mode is not None:
            bf.set_probe_mode(mode)
        fs.append(bf)
        want.append(oracle.build(nb, k, pk))
    return fs, want


@pytest.mark.parametrize("mode", [PBF_PROBE_TILED, PBF_PROBE_DIRECT, None])
def test_multi_same_size_matches_oracle(oracle, mode):
    nb, k, n_per, count = 2 ** 20, 6, 40000, 5
    fs, want = _filters(oracle, nb, k, n_per, count, mode)
    q = PackedKeys.fixed(splitmix_hex_keys(SEED, n_per // 2, count * n_per))  # members of all + absent
    got = may_contain_multi(fs, q)
    for i in range(count):
        assert np.array_equal(got[i], oracle.probe(want[i], k, q)), i
        assert np.array_equal(got[i], fs[i].may_contain_many(q, packed=True)), i
    if mode == PBF_PROBE_TILED:
        assert all(bf.last_probe_mode == PBF_PROBE_TILED for bf in fs)


def test_multi_more_than_eight_filters_and_ragged_n(oracle):
    nb, k, n_per, count = 2 ** 19, 5, 20000, 11  # two groups of the shared pipeline (8 + 3)
    fs, want = _filters(oracle, nb, k, n_per, count, PBF_PROBE_TILED)
    q = PackedKeys.fixed(splitmix_hex_keys(SEED, 3, count * n_per + 13))
    got = may_contain_multi(fs, q)
    for i in range(count):
        assert np.array_equal(got[i], oracle.probe(want[i], k, q)), i


def test_multi_mixed_sizes_k0_and_varlen(oracle):
    """Filters of different (nb_bytes, k), a k = 0 filter (always True) and variable-length keys:
    the set falls back to per-filter probes with identical results."""
    d, o = varlen_keys(0xC3, 0, 30000)
    pk = PackedKeys(d, 30000, offsets=o)
    shapes = [(2 ** 18, 6), (100003, 7), (2 ** 18, 6), (777, 3)]
    fs, want = [], []
    for nb, k in shapes:
        bf = BloomFilter(nb, k)
        bf.add_many(pk)
        fs.append(bf)
        want.append(oracle.build(nb, k, pk))
    zero = BloomFilter(64, 0)
    dq, oq = varlen_keys(0xC3, 15000, 30000)
    q = PackedKeys(dq, 30000, offsets=oq)
    got = may_contain_multi(fs + [zero], q)
    for i, (nb, k) in enumerate(shapes):
        assert np.array_equal(got[i], oracle.probe(want[i], k, q)), i
    assert (got[-1][:-1] == 0xFF).all() and got[-1][-1] == 0xFF
    # same-size subset with variable-length keys takes the shared pipeline
    fs[0].set_probe_mode(PBF_PROBE_TILED)
    fs[2].set_probe_mode(PBF_PROBE_TILED)
    got2 = may_contain_multi([fs[0], fs[2]], q)
    assert np.array_equal(got2[0], got[0]) and np.array_equal(got2[1], got[2])


def _product_filters(oracle, ns, seed=SEED):
    """SSTable filters as pebbledb sizes them (sstable.py:274: fp 0.001 -> k = 10, nb_bytes from
    each table's own key count): every filter a different nb_bytes."""
    fs, want, start = [], [], 0
    for n in ns:
        pk = PackedKeys.fixed(splitmix_hex_keys(seed, start, n))
        bf = BloomFilter.build_from_keys_and_fp_rate(pk, 0.001)
        fs.append(bf)
        want.append(oracle.build(bf.nb_bytes, bf.nb_hash_functions, pk))
        start += n
    return fs, want, start


def test_multi_mixed_product_sizes_one_hash_pass(oracle):
    """8 product-sized filters of different n (different nb_bytes, k = 10): one k_probe_set launch
    hashes every key once for all eight; each hit mask equals the filter's own probe and the
    oracle, host- and device-resident.  Then a set mixing them with a large filter (its own tiled
    pipeline) and a k = 7 filter (its own fused group)."""
    ns = [150_000 * (i + 1) for i in range(8)]  # 150k .. 1.2M keys: 270 KB .. 2.2 MB filters
    fs, want, total = _product_filters(oracle, ns)
    assert len({bf.nb_bytes for bf in fs}) == 8 and {bf.nb_hash_functions for bf in fs} == {10}
    q = PackedKeys.fixed(splitmix_hex_keys(SEED, total // 2, total + 37))  # members of the later filters + absent
    got = may_contain_multi(fs, q)
    assert all(bf.last_probe_detail == (_native.PBF_DETAIL_SET | (8 << 8)) for bf in fs)
    for i, bf in enumerate(fs):
        assert np.array_equal(got[i], oracle.probe(want[i], 10, q)), i
        assert np.array_equal(got[i], bf.may_contain_many(q, packed=True)), i
    assert got[-1].any() and not got[-1].all()
    # device-resident keys and hit masks
    qd = torch.from_numpy(q.data.copy()).cuda()
    hm = torch.zeros((len(fs), (q.n + 7) // 8), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    probe_multi_device(fs, qd.data_ptr(), q.n, [hm[i].data_ptr() for i in range(len(fs))], key_len=16)
    fs[0].sync()
    assert np.array_equal(hm.cpu().numpy(), got)
    # mixed with a large filter (tiled: its own pipeline and stream) and a k = 7 one
    big_pk = PackedKeys.fixed(splitmix_hex_keys(SEED + 1, 0, 3_000_000))
    big = BloomFilter(2 ** 25, 6)
    big.add_many(big_pk)
    seven = BloomFilter(300_007, 7)
    seven.add_many(PackedKeys.fixed(splitmix_hex_keys(SEED + 2, 0, 200_000)))
    want7 = oracle.build(300_007, 7, PackedKeys.fixed(splitmix_hex_keys(SEED + 2, 0, 200_000)))
    wantb = oracle.build(2 ** 25, 6, big_pk)
    mixed = [fs[3], big, seven, fs[0], fs[7]]
    got2 = may_contain_multi(mixed, q)
    assert big.last_probe_mode == PBF_PROBE_TILED
    assert np.array_equal(got2[0], got[3]) and np.array_equal(got2[3], got[0]) and np.array_equal(got2[4], got[7])
    assert np.array_equal(got2[1], oracle.probe(wantb, 6, q))
    assert np.array_equal(got2[2], oracle.probe(want7, 7, q))


def test_may_contain_set_one_key_many_sizes(oracle):
    """pbf_may_contain_set: one key against 16 L0-like and 6 level-like filters of different sizes
    (product sizing), a k = 7 and a k = 0 filter and a repeated filter, in one launch per k;
    every answer equals the filter's own may_contain and the oracle's.  Keys: members, absent
    keys, empty, non-ASCII, and a key longer than the 4 KiB mapped stage."""
    ns = [20_000 + 7_919 * i for i in range(22)]
    fs, want, total = _product_filters(oracle, ns, seed=SEED + 5)
    seven = BloomFilter(50_021, 7)
    seven.add_many(["k%d" % i for i in range(3000)])
    zero = BloomFilter(64, 0)
    mixed = fs[:10] + [seven, zero] + fs[10:] + [fs[4]]
    keys = [bytes(k).decode() for k in splitmix_hex_keys(SEED + 5, 0, total)[::997]]
    keys += [bytes(k).decode() for k in splitmix_hex_keys(SEED + 6, 0, 120)] + ["", "é\U0001f511", "x" * 5000]
    keys += ["k%d" % i for i in range(0, 4000, 37)]
    for key in keys:
        got = may_contain_set(mixed, key)
        assert got == [bf.may_contain(key) for bf in mixed], key
    w7 = oracle.build(50_021, 7, PackedKeys.from_strs(["k%d" % i for i in range(3000)]))
    pk = PackedKeys.from_strs(keys)
    for bf, w in zip(fs + [seven], want + [w7]):
        hits = np.unpackbits(oracle.probe(w, bf.nb_hash_functions, pk), bitorder="little")[:len(keys)]
        assert [bool(h) for h in hits] == [may_contain_set([bf], key)[0] for key in keys]
    assert may_contain_set([], "a") == []


def test_multi_rejects_bad_sets():
    a = BloomFilter(4096, 3)
    a.add("x")
    with pytest.raises(ValueError):
        may_contain_multi([a, a], ["x", "y"])
    b = BloomFilter(0, 3)
    with pytest.raises(ZeroDivisionError):
        may_contain_multi([a, b], ["x"])


def _dev_hex(seed, start, n, out=None, at=0):
    t = out if out is not None else torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    _native.check(_native.lib().pbf_gen_splitmix_hex(0, None, t.data_ptr() + at * 16, seed, start, n), "gen")
    return t


def test_multi_device_c5_shape(oracle):
    """C5 at reduced size: 8 filters (m = 2^27, k = 6) over disjoint 1M-key SSTables, probed with
    8M keys (half members spread evenly over the 8 sets, half absent) in one device call; each
    hit mask equals that filter's single device probe; members all hit; the oracle agrees on
    every filter for a 200k-key sample."""
    nf, nb, k, n_per = 8, 2 ** 24, 6, 1_000_000
    keys = _dev_hex(SEED, 0, nf * n_per)
    fs = []
    for f in range(nf):
        bf = BloomFilter(nb, k)
        bf.add_device_fixed(keys.data_ptr() + f * n_per * 16, 16, n_per)
        bf.set_probe_mode(PBF_PROBE_TILED)
        fs.append(bf)
    for bf in fs:
        bf.sync()
    nq = 8 * n_per
    half = nq // 2
    q = torch.empty(nq * 16, dtype=torch.uint8, device="cuda")
    for f in range(nf):  # members: the first half of each filter's key range
        _dev_hex(SEED, f * n_per, half // nf, q, f * (half // nf))
    _dev_hex(SEED, nf * n_per, half, q, half)  # absent
    hms = [torch.zeros(nq // 8, dtype=torch.uint8, device="cuda") for _ in range(nf)]
    torch.cuda.synchronize()
    probe_multi_device(fs, q.data_ptr(), nq, [h.data_ptr() for h in hms], key_len=16)
    fs[0].sync()
    assert all(bf.last_probe_mode == PBF_PROBE_TILED for bf in fs)
    single = torch.zeros(nq // 8, dtype=torch.uint8, device="cuda")
    qh = q[: 200_000 * 16].cpu().numpy().reshape(-1, 16)
    per = half // nf
    for f, bf in enumerate(fs):
        single.zero_()
        torch.cuda.synchronize()
        bf.probe_device_fixed(q.data_ptr(), 16, nq, single.data_ptr())
        bf.sync()
        h = hms[f].cpu().numpy()
        assert np.array_equal(h, single.cpu().numpy()), f
        bits = np.unpackbits(h, bitorder="little")
        assert bits[f * per:(f + 1) * per].all(), f  # its own members
        want = oracle.build(nb, k, PackedKeys.fixed(splitmix_hex_keys(SEED, f * n_per, n_per)), omp=True)
        assert np.array_equal(h[:25_000], oracle.probe(want, k, PackedKeys.fixed(qh), omp=True)), f


# ---------------------------------------------------------------- C5 as benchmarked
def _c5_filters(oracle, nf, n_per, nb=2 ** 27, k=6):
    """nf SSTable filters of the C5 geometry (m = 2^30, k = 6), filter f built on device from
    keys [f*n_per, (f+1)*n_per); plus the oracle's bitmaps (OpenMP C restatement)."""
    keys = _dev_hex(SEED, 0, nf * n_per)
    fs = []
    for f in range(nf):
        bf = BloomFilter(nb, k)
        bf.add_device_fixed(keys.data_ptr() + f * n_per * 16, 16, n_per)
        fs.append(bf)
    for bf in fs:
        bf.sync()
    host = keys.cpu().numpy().reshape(-1, 16)
    del keys
    want = [oracle.build(nb, k, PackedKeys.fixed(host[f * n_per:(f + 1) * n_per]), omp=True) for f in range(nf)]
    for f, bf in enumerate(fs):
        got = bf.bitmap()
        if got != want[f].tobytes():
            g = np.frombuffer(got, dtype=np.uint8)
            missing = int(np.unpackbits(want[f] & ~g).sum())
            extra = int(np.unpackbits(g & ~want[f]).sum())
            tiles = np.unique(np.flatnonzero(g != want[f]) // (1 << 17))  # 2^20-bit tiles
            raise AssertionError(f"filter {f}/{nf}: {missing} bits missing, {extra} extra, in tiles "
                                 f"{tiles[:20].tolist()} ({len(tiles)} tiles); build detail "
                                 f"{hex(bf.last_build_detail)} stream {bf.stream:#x}, streams "
                                 f"{[hex(b.stream) for b in fs]}")
    return fs, want


def _c5_probe_and_check(oracle, fs, want, q, nq, k=6, sample=(0, 1_000_000), samples=None):
    """One device multi-probe of q (nq 16-B keys) against fs; every filter's hit mask equals
    its own single-filter probe over the whole batch and the oracle's on [sample) (or on each
    range of `samples`)."""
    nf = len(fs)
    hms = [torch.zeros((nq + 7) // 8, dtype=torch.uint8, device="cuda") for _ in range(nf)]
    torch.cuda.synchronize()
    probe_multi_device(fs, q.data_ptr(), nq, [h.data_ptr() for h in hms], key_len=16)
    fs[0].sync()
    detail = fs[0].last_probe_detail
    got = [h.cpu().numpy() for h in hms]
    del hms
    single = torch.zeros((nq + 7) // 8, dtype=torch.uint8, device="cuda")
    ranges = []
    for a, b in (samples or [sample]):
        a, b = max(0, a - a % 8), min(nq, b) - min(nq, b) % 8  # whole hit-mask bytes
        ranges.append((a, b, PackedKeys.fixed(q[a * 16:b * 16].cpu().numpy().reshape(-1, 16))))
    for f, bf in enumerate(fs):
        single.zero_()
        torch.cuda.synchronize()
        bf.probe_device_fixed(q.data_ptr(), 16, nq, single.data_ptr())
        bf.sync()
        assert np.array_equal(got[f], single.cpu().numpy()), f
        for a, b, qh in ranges:
            assert np.array_equal(got[f][a // 8:b // 8], oracle.probe(want[f], k, qh, omp=True)[: (b - a) // 8]), (f, a)
    return got, detail


@pytest.fixture(scope="module")
def c5_full(oracle):
    """BASELINE.json configs[4]'s filter set: 8 SSTable filters of nb_bytes = 2^27, k = 6, 10M
    keys each (built once for the module's full-size C5 tests), plus the oracle's bitmaps."""
    fs, want = _c5_filters(oracle, 8, 10_000_000)
    yield fs, want
    fs.clear()  # the handles go with their last reference
    torch.cuda.empty_cache()


def _c5_queries(nq, nf=8, n_per=10_000_000):
    """C5's probe batch: the first half members spread evenly over the nf SSTables (filter f's
    block of `per` keys), the second half absent keys."""
    half = nq // 2
    per = half // nf
    q = torch.empty(nq * 16, dtype=torch.uint8, device="cuda")
    for f in range(nf):
        cnt = per if f < nf - 1 else half - (nf - 1) * per
        _dev_hex(SEED, f * n_per, cnt, q, f * per)
    _dev_hex(SEED, nf * n_per, nq - half, q, half)
    return q, half, per


@pytest.mark.timeout(300)
def test_c5_full_geometry_fused_ring_gather(oracle, c5_full):
    """BASELINE.json configs[4] on one GPU as bench.py runs it: 8 filters (nb_bytes = 2^27,
    k = 6, 10M keys each) and one device multi-probe of 20M + 37 keys (half members spread over
    the 8 SSTables, half absent): B = 1024 tiles takes the RING partition, the XCD-aware fused
    tile test and ONE fused k_gather_ring<8> (checked via last_probe_detail).  Every filter's
    mask == its single probe over the whole batch == the oracle on a 1M-key sample; members all
    hit; the false-positive count is at the theoretical rate."""
    nf = 8
    fs, want = c5_full
    nq = 20_000_037
    q, half, per = _c5_queries(nq)
    got, detail = _c5_probe_and_check(oracle, fs, want, q, nq, sample=(half - 500_000, half + 500_000))
    assert detail & _native.PBF_DETAIL_RING and (detail >> 8) & 0xFF == nf, hex(detail)
    for f in range(nf):
        bits = np.unpackbits(got[f], bitorder="little")[:nq]
        cnt = per if f < nf - 1 else half - (nf - 1) * per
        assert bits[f * per:f * per + cnt].all(), f
        fill = fs[f].popcount() / (8 * 2 ** 27)
        fp = int(bits[half:].sum())
        assert fp <= 3 * (nq - half) * fill ** 6 + 20, (f, fp)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("nq,p", [(100_000_000, 1), (100_000_037, 1), (200_000_037, 2)])
def test_c5_full_size_100m_pipelines(oracle, c5_full, nq, p):
    """C5 at its own size (BASELINE.json configs[4]: 100M lookup keys vs 8 x 128 MiB filters)
    under -m gpu.  100M keys take the fused 8-filter path in ONE pipeline: the gather's key
    bitmaps for 8 filters would cap a pipeline at ~33M keys with one partition workgroup per CU,
    so the plan takes 3 rounds of workgroups and the tile test walks its table in region chunks.
    200M keys take 2 pipelines, the second offsetting every filter's hit mask by i0 / 8.  Every
    filter's mask == its own single probe over the whole batch; the oracle agrees on samples
    around the pipeline boundary, the middle and the batch's ragged end for all 8 filters;
    members all hit; false positives at the filters' rate.  The *_037 cases are ragged: not a
    multiple of 8, 64 or p x 64."""
    nf = 8
    fs, want = c5_full
    q, half, per = _c5_queries(nq)
    # pipelines of equal size, multiples of 64 keys (tiled_probe_batch)
    pl = (((nq + p - 1) // p) + 63) // 64 * 64
    b1, b2 = (pl, nq // 4) if p > 1 else (nq // 3, 2 * nq // 3)
    samples = [(b1 - 100_000, b1 + 100_000), (b2 - 100_000, b2 + 100_000), (nq - 100_003, nq)]
    got, detail = _c5_probe_and_check(oracle, fs, want, q, nq, samples=samples)
    del q
    assert detail & _native.PBF_DETAIL_RING, hex(detail)
    assert (detail >> 8) & 0xFF == nf, hex(detail)
    assert detail >> 16 == p, f"{detail >> 16} pipelines, expected {p} ({hex(detail)})"
    for f in range(nf):
        bits = np.unpackbits(got[f], bitorder="little")[:nq]
        cnt = per if f < nf - 1 else half - (nf - 1) * per
        cnt = min(cnt, 10_000_000)  # (a block past the filter's 10M keys holds other filters' keys)
        assert bits[f * per:f * per + cnt].all(), f
        # the last byte's padding bits stay clear
        if nq % 8:
            assert got[f][-1] >> (nq % 8) == 0, f
        fill = fs[f].popcount() / (8 * 2 ** 27)
        fp = int(bits[half:].sum())
        assert fp <= 3 * (nq - half) * fill ** 6 + 20, (f, fp)


@pytest.mark.timeout(150)
@pytest.mark.parametrize("nf", [2, 5])
def test_c5_geometry_small_sets_ragged_and_spills(oracle, nf):
    """The same ring + fused path with 2 and 5 filters, a ragged batch, and keys repeated 60k and
    50k times so the multi-filter partition's rings and regions overflow (spilled positions are
    tested against every filter's bitmap inside the partition)."""
    n_per = 2_000_000
    fs, want = _c5_filters(oracle, nf, n_per)
    base = nf * n_per // 2 + 3
    rep_member = np.repeat(splitmix_hex_keys(SEED, 5, 1), 60_000, axis=0)           # member of filter 0
    rep_absent = np.repeat(splitmix_hex_keys(SEED + 1, 0, 1), 50_000, axis=0)
    qh = np.concatenate([splitmix_hex_keys(SEED, 0, base), rep_member,
                         splitmix_hex_keys(SEED, nf * n_per, 777_777), rep_absent])
    nq = len(qh)
    q = torch.from_numpy(qh.reshape(-1)).cuda()
    got, detail = _c5_probe_and_check(oracle, fs, want, q, nq, sample=(0, nq // 8 * 8))
    assert detail & _native.PBF_DETAIL_RING and (detail >> 8) & 0xFF == nf, hex(detail)
    b0 = np.unpackbits(got[0], bitorder="little")[:nq]
    assert b0[base:base + 60_000].all()  # the repeated member hits filter 0 every time


def test_multi_placement_groups_one_thread_each(oracle):
    """A filter set in placement groups (LsmStorage.get's filters placed one per GPU, probed from
    one process: pbf_probe_multi_placed): each group runs on its own host thread and stages the
    host batch to its device itself.  On the one-GPU box every group is on device 0 (the 8-GPU
    shape is one group per device); masks come back in the set's (get) order and equal the
    single-group probe and the oracle, for same-size filters (shared pipelines per group),
    mixed sizes and variable-length keys."""
    nb, k, n_per, count = 2 ** 21, 6, 60_000, 8
    fs, want = _filters(oracle, nb, k, n_per, count)
    small = BloomFilter(50_021, 7)
    small_keys = PackedKeys.fixed(splitmix_hex_keys(SEED, 5, 3000))
    small.add_many(small_keys)
    fs.append(small)
    want.append(oracle.build(50_021, 7, small_keys))
    q = PackedKeys.fixed(splitmix_hex_keys(SEED, n_per // 3, count * n_per + 11))
    groups = [i % 4 for i in range(len(fs))]
    got = may_contain_multi(fs, q, groups=groups)
    ref = may_contain_multi(fs, q)
    assert np.array_equal(got, ref)
    kk = [k] * count + [7]
    for i in range(len(fs)):
        assert np.array_equal(got[i], oracle.probe(want[i], kk[i], q)), i
    d, o = varlen_keys(0xC3, 0, 20_000)
    vq = PackedKeys(d, 20_000, offsets=o)
    gv = may_contain_multi(fs, vq, groups=[3, 2, 1, 0, 3, 2, 1, 0, 5])
    for i in range(len(fs)):
        assert np.array_equal(gv[i], oracle.probe(want[i], kk[i], vq)), i
    with pytest.raises(ValueError):
        may_contain_multi([fs[0], fs[0]], q, groups=[0, 1])  # a filter twice


def _device_count():
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


@pytest.mark.skipif(_device_count() < 2, reason="needs two GPUs (the driver's multi-GPU node)")
def test_filters_on_two_devices_from_one_process(oracle):
    """Round-4 advice: the cross-device fan-out with filters REALLY on two devices — a host batch
    against filters on devices 0 and 1 (by device: one host thread per device; with explicit
    groups; and the one-key set probe, one launch per device) equals the oracle."""
    nb, k, n_per = 2 ** 20, 6, 30_000
    fs, want = [], []
    for i in range(6):
        keys = PackedKeys.fixed(splitmix_hex_keys(SEED, i * n_per, n_per))
        bf = BloomFilter(nb, k, device=i % 2)
        bf.add_many(keys)
        fs.append(bf)
        want.append(oracle.build(nb, k, keys))
    assert {bf.device for bf in fs} == {0, 1}
    q = PackedKeys.fixed(splitmix_hex_keys(SEED, n_per // 2, 6 * n_per))
    for got in (may_contain_multi(fs, q), may_contain_multi(fs, q, groups=[0, 1, 2, 3, 2, 3])):
        for i in range(len(fs)):
            assert np.array_equal(got[i], oracle.probe(want[i], k, q)), i
    qs = [bytes(x).decode() for x in splitmix_hex_keys(SEED, n_per - 50, 100)]
    for key in qs:
        exp = [bool(np.unpackbits(oracle.probe(w, k, PackedKeys.from_strs([key])), bitorder="little")[0]) for w in want]
        assert may_contain_set(fs, key) == exp
