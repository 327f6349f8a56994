"""Device-resident path (keys and hit masks in HBM, torch as the allocator) and full-size
properties at BASELINE.json's config-2 scale.  Runs on an MI355X (`-m gpu`)."""
import numpy as np
import pytest

from pebbledb_amd import BloomFilter, PackedKeys
from pebbledb_amd import _native
from pebbledb_amd._native import PBF_BUILD_ATOMIC, PBF_BUILD_TILED, PBF_PROBE_DIRECT, PBF_PROBE_TILED
from pebbledb_amd.keys import splitmix_hex_keys, varlen_keys

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def dev_keys_hex(seed, start, n):
    t = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    _native.check(_native.lib().pbf_gen_splitmix_hex(0, None, t.data_ptr(), seed, start, n), "gen")
    torch.cuda.synchronize()
    return t


def test_device_keygen_matches_numpy():
    t = dev_keys_hex(0x5EEDB100, 12345, 5000)
    assert np.array_equal(t.cpu().numpy().reshape(-1, 16), splitmix_hex_keys(0x5EEDB100, 12345, 5000))
    d, o = varlen_keys(0xC3, 777, 3000)
    od = torch.from_numpy(o.view(np.int64)).cuda()
    out = torch.empty(int(o[-1]), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    _native.check(_native.lib().pbf_gen_varlen(0, None, out.data_ptr(), od.data_ptr(), 0xC3, 777, 3000), "gen")
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), d)


@pytest.mark.parametrize("mode", [PBF_BUILD_ATOMIC, PBF_BUILD_TILED])
def test_device_resident_equals_host_path(oracle, mode):
    n = 200000
    keys = dev_keys_hex(9, 0, n)
    host = PackedKeys.fixed(splitmix_hex_keys(9, 0, n))
    bf = BloomFilter(2 ** 18, 6)
    bf.set_build_mode(mode)
    bf.add_device_fixed(keys.data_ptr(), 16, n)
    q = dev_keys_hex(9, n // 2, n)
    hm = torch.zeros((n + 7) // 8, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    want = oracle.build(2 ** 18, 6, host)
    qh = PackedKeys.fixed(splitmix_hex_keys(9, n // 2, n))
    want_hm = oracle.probe(want, 6, qh)
    for pm in (PBF_PROBE_DIRECT, PBF_PROBE_TILED):
        hm.zero_()
        torch.cuda.synchronize()
        bf.set_probe_mode(pm)
        bf.probe_device_fixed(q.data_ptr(), 16, n, hm.data_ptr())
        bf.sync()
        assert bf.bitmap() == want.tobytes()
        assert np.array_equal(hm.cpu().numpy(), want_hm), pm
    # variable-length on device, offsets not starting at 0 (a slice of a larger batch)
    d, o = varlen_keys(21, 0, 30001)
    od = torch.from_numpy(o.view(np.int64)).cuda()
    dd = torch.from_numpy(d).cuda()
    torch.cuda.synchronize()
    sl = 1000  # keys [1000, 30001): offsets pointer shifted, data pointer at offsets[1000]
    bfv = BloomFilter(40000, 7)
    bfv.set_build_mode(mode)
    bfv.add_device(dd.data_ptr() + int(o[sl]), od.data_ptr() + 8 * sl, 30001 - sl)
    bfv.sync()
    sub = PackedKeys(d[int(o[sl]):], 30001 - sl, offsets=o[sl:] - o[sl])
    assert bfv.bitmap() == oracle.build(40000, 7, sub).tobytes()


def test_config2_full_size_properties(oracle):
    """C2: 10M 16-B keys, m = 2^30 (128 MiB), k = 6 — bit-exact vs the OpenMP oracle,
    atomic == tiled, no false negatives, FPR at the theoretical value."""
    n, nb, k = 10_000_000, 2 ** 27, 6
    keys = dev_keys_hex(0x5EEDB100, 0, n)
    a = BloomFilter(nb, k)
    a.set_build_mode(PBF_BUILD_TILED)
    a.add_device_fixed(keys.data_ptr(), 16, n)
    b = BloomFilter(nb, k)
    b.set_build_mode(PBF_BUILD_ATOMIC)
    b.add_device_fixed(keys.data_ptr(), 16, n)
    a.sync()
    b.sync()
    ba, bb = a.bitmap(), b.bitmap()
    assert ba == bb
    host = PackedKeys.fixed(keys.cpu().numpy().reshape(-1, 16))
    want = oracle.build(nb, k, host, omp=True)
    assert ba == want.tobytes()
    # probes: n members + n non-members
    q = dev_keys_hex(0x5EEDB100, 0, 2 * n)
    hm = torch.zeros(2 * n // 8, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    a.set_probe_mode(PBF_PROBE_TILED)
    a.probe_device_fixed(q.data_ptr(), 16, 2 * n, hm.data_ptr())
    a.sync()
    assert a.last_probe_mode == PBF_PROBE_TILED
    h = hm.cpu().numpy()
    hm2 = torch.zeros(2 * n // 8, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    a.set_probe_mode(PBF_PROBE_DIRECT)
    a.probe_device_fixed(q.data_ptr(), 16, 2 * n, hm2.data_ptr())
    a.sync()
    assert np.array_equal(hm2.cpu().numpy(), h)  # direct == tiled at full size
    assert (h[: n // 8] == 0xFF).all()  # no false negatives
    fp = int(np.unpackbits(h[n // 8:]).sum())
    fill = a.popcount() / (8 * nb)
    expect = n * fill ** k
    assert fp <= 3 * expect + 20, (fp, expect)
    # the non-member hit mask equals the oracle's on a 1M sample
    qs = PackedKeys.fixed(splitmix_hex_keys(0x5EEDB100, n, 1_000_000))
    assert np.array_equal(h[n // 8: n // 8 + 125000], oracle.probe(want, k, qs, omp=True))


@pytest.mark.timeout(150)
def test_config4_full_size_product_sizing(oracle):
    """C4: one of the eight 125M-key SSTable filters with pebbledb's product sizing
    (sstable.py:274, fp 0.001 → nb_bytes 224,649,806, k = 10: non-power-of-two m, the
    Lemire-fastmod floor-mod path).  Tiled build == the C oracle bit for bit; members all hit."""
    from math import ceil, log
    n = 125_000_000
    m = (-n * log(0.001)) / (log(2) ** 2)
    nb, k = ceil(m / 8), round((m / n) * log(2))
    assert (nb, k) == (224_649_806, 10)
    keys = dev_keys_hex(0x5EEDB100, 3 * n, n)  # filter 3's key range
    bf = BloomFilter(nb, k)
    bf.set_build_mode(PBF_BUILD_TILED)
    bf.add_device_fixed(keys.data_ptr(), 16, n)
    hm = torch.zeros(n // 8, dtype=torch.uint8, device="cuda")
    bf.probe_device_fixed(keys.data_ptr(), 16, n, hm.data_ptr())
    bf.sync()
    assert bf.last_build_mode == PBF_BUILD_TILED
    assert bool((hm == 0xFF).all().item())
    got = bf.bitmap()
    host = PackedKeys.fixed(keys.cpu().numpy().reshape(-1, 16))
    del keys, hm
    want = oracle.build(nb, k, host, omp=True)
    assert got == want.tobytes()


@pytest.mark.timeout(150)
def test_config4_eight_concurrent_builds_and_absent_keys(oracle):
    """C4 as bench.py runs it (BASELINE configs[3]): the eight 125M-key product-sized filters
    (nb_bytes 224,649,806, k = 10) cleared and built back to back on their own pooled streams with
    no wait between them, twice.  Filters 0 and 6 == the C oracle bit for bit; filter 6's hit
    mask of 1M absent keys == the oracle's bitwise (the reference's non-uniform floor-mod for a
    non-power-of-two m shows in its false-positive rate)."""
    from math import ceil, log
    n = 125_000_000
    m = (-n * log(0.001)) / (log(2) ** 2)
    nb, k = ceil(m / 8), round((m / n) * log(2))
    keys = [dev_keys_hex(0x5EEDB100, g * n, n) for g in range(8)]
    fs = [BloomFilter(nb, k) for _ in range(8)]
    assert len({bf.stream for bf in fs}) > 1  # the pool deals distinct streams
    for _ in range(2):
        for g, bf in enumerate(fs):
            bf.clear()
            bf.add_device_fixed(keys[g].data_ptr(), 16, n)
    absent = dev_keys_hex(0x5EEDB100, 8 * n, 1_000_000)
    hm = torch.zeros(1_000_000 // 8, dtype=torch.uint8, device="cuda")
    fs[6].probe_device_fixed(absent.data_ptr(), 16, 1_000_000, hm.data_ptr())
    for bf in fs:
        bf.sync()
    assert all(bf.last_build_mode == PBF_BUILD_TILED for bf in fs)
    got = {g: fs[g].bitmap() for g in (0, 6)}
    host = {g: PackedKeys.fixed(keys[g].cpu().numpy().reshape(-1, 16)) for g in (0, 6)}
    hm_got = hm.cpu().numpy()
    del keys, absent, hm
    for g in (0, 6):
        want = oracle.build(nb, k, host[g], omp=True)
        assert got[g] == want.tobytes(), g
        if g == 6:
            qs = PackedKeys.fixed(splitmix_hex_keys(0x5EEDB100, 8 * n, 1_000_000))
            want_hm = oracle.probe(want, k, qs, omp=True)
            assert np.array_equal(hm_got, want_hm)
            fp = int(np.unpackbits(hm_got).sum())
            assert 500 < fp < 2500, fp  # ~0.0013 (the floor-mod's edge tiles), not 0.001


@pytest.mark.timeout(150)
def test_config3_full_size_varlen_large_m(oracle):
    """C3 as bench.py runs it (BASELINE configs[2]): 100M variable-length keys (8..64 B) into
    m = 2^33 bits (nb_bytes = 2^30), k = 8 — the m > 2^32 index map where only [0, 2^31) and
    [m - 2^31, m) are reachable — then ONE probe of 200M keys (the 100M members + 100M absent:
    two tiled pipelines, the counting-sort partition at 4096 tiles).  Build == the C oracle bit
    for bit, the unreachable middle stays zero, members all hit, and the absent half's hit mask
    == the oracle's bitwise (every false positive the same)."""
    from pebbledb_amd.keys import _splitmix64_np
    n, nb, k = 100_000_000, 2 ** 30, 8
    idx = np.arange(2 * n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = _splitmix64_np((np.uint64(0xC3) << np.uint64(32)) + idx)
    o = np.zeros(2 * n + 1, dtype=np.uint64)
    np.cumsum((np.uint64(8) + h % np.uint64(57)), out=o[1:])
    del h, idx
    od = torch.from_numpy(o.view(np.int64)).cuda()
    d = torch.empty(int(o[-1]), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    _native.check(_native.lib().pbf_gen_varlen(0, None, d.data_ptr(), od.data_ptr(), 0xC3, 0, 2 * n), "gen")
    torch.cuda.synchronize()
    bf = BloomFilter(nb, k)
    bf.set_build_mode(PBF_BUILD_TILED)
    bf.add_device(d.data_ptr(), od.data_ptr(), n)
    hm = torch.zeros(2 * n // 8, dtype=torch.uint8, device="cuda")
    bf.probe_device(d.data_ptr(), od.data_ptr(), 2 * n, hm.data_ptr())
    bf.sync()
    assert bf.last_probe_mode == PBF_PROBE_TILED
    h_all = hm.cpu().numpy()
    assert (h_all[: n // 8] == 0xFF).all()
    got = np.frombuffer(bf.bitmap(), dtype=np.uint8)
    assert not got[2 ** 28: nb - 2 ** 28].any()  # bits [2^31, m - 2^31) are unreachable
    hd = d.cpu().numpy()
    del d, od, hm
    want = oracle.build(nb, k, PackedKeys(hd[: int(o[n])], n, offsets=o[: n + 1]), omp=True)
    assert np.array_equal(got, want)
    absent = PackedKeys(hd[int(o[n]):], n, offsets=o[n:] - o[n])
    want_hm = oracle.probe(want, k, absent, omp=True)
    assert np.array_equal(h_all[n // 8:], want_hm)
    assert 30 < int(np.unpackbits(want_hm).sum()) < 300  # ~116 at these seeds (~70 expected)


@pytest.mark.timeout(150)
def test_ring_probe_with_regions_past_4gib(oracle):
    """A ring-partition probe whose regions exceed 4 GiB (264M keys, k = 4, one pipeline of a
    2^30-bit filter: G x B x cap x 4 B ~ 4.7 GB).  A flush with no complete group writes the
    workgroup's dummy line after ALL regions; as a 32-bit offset from the workgroup's regions it
    wrapped into another workgroup's live entries (round-5 advisor).  Tiled == direct probe over
    the whole batch, members all hit, a sample == the oracle."""
    n_m, nq, nb, k = 10_000_000, 264_000_000, 2 ** 27, 4
    keys = dev_keys_hex(0x77, 0, nq)
    bf = BloomFilter(nb, k)
    bf.set_build_mode(PBF_BUILD_TILED)
    bf.add_device_fixed(keys.data_ptr(), 16, n_m)
    hm_t = torch.zeros(nq // 8, dtype=torch.uint8, device="cuda")
    hm_d = torch.zeros(nq // 8, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    bf.set_probe_mode(PBF_PROBE_TILED)
    bf.probe_device_fixed(keys.data_ptr(), 16, nq, hm_t.data_ptr())
    bf.sync()
    detail = bf.last_probe_detail
    assert detail & _native.PBF_DETAIL_RING and (detail >> 16) == 1, hex(detail)  # one ring pipeline
    sb = __import__("ctypes").c_uint64()
    _native.check(_native.lib().pbf_scratch_bytes(0, __import__("ctypes").byref(sb)), "scratch")
    assert sb.value > 4 * 2 ** 30 + 2 ** 28  # the regions alone pass 4 GiB
    bf.set_probe_mode(PBF_PROBE_DIRECT)
    bf.probe_device_fixed(keys.data_ptr(), 16, nq, hm_d.data_ptr())
    bf.sync()
    assert bool(torch.equal(hm_t, hm_d))
    assert bool((hm_t[: n_m // 8] == 0xFF).all().item())
    want = oracle.build(nb, k, PackedKeys.fixed(keys[: n_m * 16].cpu().numpy().reshape(-1, 16)), omp=True)
    assert bf.bitmap() == want.tobytes()
    s0 = nq - 1_000_000  # the batch's last workgroups: the regions' far end
    qs = PackedKeys.fixed(keys[s0 * 16:].cpu().numpy().reshape(-1, 16))
    assert np.array_equal(hm_t[s0 // 8:].cpu().numpy(), oracle.probe(want, k, qs, omp=True))
    del keys, hm_t, hm_d
    _native.check(_native.lib().pbf_trim(0), "trim")


def test_replicate_and_device_bitmaps(oracle):
    """BloomFilter.replicate (pbf_copy_filter: device to device, or through pinned host memory)
    and the device-memory from_bytes / to_bytes (pbf_set_bitmap_device / pbf_get_bitmap_device):
    each replica is the source's bitmap and k bit for bit (== the oracle), answers its probes
    identically, and is independent of later changes to the source."""
    n, nb, k = 300_000, 2 ** 20 + 12, 7
    host = PackedKeys.fixed(splitmix_hex_keys(31, 0, n))
    want = oracle.build(nb, k, host)
    src = BloomFilter(nb, k)
    src.add_many(host)
    probes = PackedKeys.fixed(splitmix_hex_keys(31, n // 2, n))
    want_hm = oracle.probe(want, k, probes)
    for bounce in (False, True):
        r = src.replicate(0, bounce=bounce)
        assert r.nb_hash_functions == k and r.nb_bytes == nb and r.handle.value != src.handle.value
        assert r.bitmap() == want.tobytes() and r == src
        assert np.array_equal(r.may_contain_many(probes, packed=True), want_hm)
        assert r.may_contain(f"{0:016x}") == src.may_contain(f"{0:016x}")
    # the replica does not follow the source
    r = src.replicate()
    src.add_many(PackedKeys.fixed(splitmix_hex_keys(31, 10 ** 9, 50_000)))
    assert r.bitmap() == want.tobytes() and src.bitmap() != want.tobytes()
    # a pristine (cleared) filter replicates to all zeros, including m > 2^32 (unreachable middle)
    big = BloomFilter(2 ** 29 + 2 ** 16, 3)
    big.add_many([f"k{i}" for i in range(1000)])
    big.clear()
    assert not any(big.replicate().bitmap())
    big.add_many([f"k{i}" for i in range(1000)])
    rb = big.replicate()
    assert rb.bitmap() == big.bitmap() and rb.may_contain("k7") and not rb.may_contain("zz")
    del big, rb
    # device-memory to_bytes / from_bytes through a torch tensor
    t = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    r.bitmap_to_device(t.data_ptr())
    r.sync()
    assert t.cpu().numpy().tobytes() == want.tobytes()
    f2 = BloomFilter.from_device_bitmap(t.data_ptr(), nb, k, device=0,
                                        stream=torch.cuda.current_stream().cuda_stream)
    f2.sync()
    assert f2.bitmap() == want.tobytes()
    assert np.array_equal(f2.may_contain_many(probes, packed=True), want_hm)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs 2 GPUs (the driver's 8-GPU node)")
def test_replicate_to_another_device(oracle):
    """pbf_copy_filter across devices (peer copy over xGMI, and the pinned-host bounce)."""
    n, nb, k = 200_000, 2 ** 22, 6
    host = PackedKeys.fixed(splitmix_hex_keys(41, 0, n))
    want = oracle.build(nb, k, host)
    src = BloomFilter(nb, k, device=0)
    src.add_many(host)
    for bounce in (False, True):
        r = src.replicate(1, bounce=bounce)
        assert r.device == 1 and r.bitmap() == want.tobytes()
        probes = PackedKeys.fixed(splitmix_hex_keys(41, n // 2, n))
        assert np.array_equal(r.may_contain_many(probes, packed=True), oracle.probe(want, k, probes))
