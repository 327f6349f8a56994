"""GPU parity: the HIP path (through the C-ABI) against the oracle and the reference's golden
vectors.  Bit-exact for every bitmap, hit mask and index.  Runs on an MI355X (`-m gpu`)."""
import hashlib

import numpy as np
import pytest

from conftest import load_golden
from pebbledb_amd import BloomFilter, PackedKeys, _native
from pebbledb_amd._native import (PBF_BUILD_ATOMIC, PBF_BUILD_AUTO, PBF_BUILD_TILED, PBF_PROBE_DIRECT,
                                  PBF_PROBE_TILED)
from pebbledb_amd.keys import splitmix_hex_keys, varlen_keys

pytestmark = pytest.mark.gpu

MODES = [PBF_BUILD_ATOMIC, PBF_BUILD_TILED]
PROBE_MODES = [PBF_PROBE_DIRECT, PBF_PROBE_TILED]


def probe_both(bf, keys):
    """Hit mask from the direct AND the tiled probe; they must agree bit for bit."""
    pk = keys if isinstance(keys, PackedKeys) else PackedKeys.from_strs(list(keys))
    out = []
    for pm in PROBE_MODES:
        try:
            bf.set_probe_mode(pm)
        except ValueError:  # the tiled probe needs k <= 32 (register budget of k_part)
            assert pm == PBF_PROBE_TILED and bf.nb_hash_functions > 32
            continue
        out.append(bf.may_contain_many(pk, packed=True))
        if pk.n:
            assert bf.last_probe_mode == pm
    bf.set_probe_mode(0)
    assert all(np.array_equal(out[0], o) for o in out[1:]), "direct and tiled probes disagree"
    return out[0]


def built(nb, k, keys, mode=PBF_BUILD_AUTO):
    bf = BloomFilter(nb, k)
    if mode != PBF_BUILD_AUTO:
        try:
            bf.set_build_mode(mode)
        except ValueError:  # the tiled build needs k <= 32
            assert mode == PBF_BUILD_TILED and k > 32
    bf.add_many(keys)
    if mode != PBF_BUILD_AUTO and len(keys if not isinstance(keys, PackedKeys) else range(keys.n)) and k <= 32:
        assert bf.last_build_mode == mode
    bf.add_many(keys)
    return bf


def bits_of(hm, n):
    return [bool(hm[i >> 3] >> (i & 7) & 1) for i in range(n)]


# ---------------------------------------------------------------- the reference's own tests
def test_reference_test_lookups():
    # src/__tests__/test_bloom_filter.py:4-20
    bf = BloomFilter(nb_bytes=4, nb_hash_functions=3)
    for key in ["foo", "bar", "baz"]:
        bf.add(key=key)
    for key in ["foo", "bar", "baz"]:
        assert bf.may_contain(key=key) is True
    for key in ["not_in_bloom_filter", "missing"]:
        assert bf.may_contain(key=key) is False


def test_reference_build_from_keys():
    bf = BloomFilter.build_from_keys_and_fp_rate(["key1", "key2"], 0.001)
    assert bf.may_contain("key1") is True and bf.may_contain("key2") is True


@pytest.mark.parametrize("nb,expected", [(1, b"3"), (3, b"\x003\x10")])
def test_reference_encode(nb, expected):
    # test_bloom_filter.py:32-61
    bf = BloomFilter(nb_bytes=nb, nb_hash_functions=2)
    for key in ["key1", "key2", "key3"]:
        bf.add(key)
    assert bf.to_bytes() == expected + b"\x02"
    assert BloomFilter.from_bytes(bf.to_bytes()) == bf  # :64-91


def test_reference_equality():
    # test_bloom_filter.py:94-140
    keys = ["key1", "key2", "key3"]
    a, b = BloomFilter(8, 3), BloomFilter(8, 3)
    c = BloomFilter(8, 4)
    for key in keys:
        a.add(key)
        b.add(key)
        c.add(key)
    assert (a == b) is True
    assert (a == c) is False
    d = BloomFilter(8, 4)
    for key in keys[:2]:
        d.add(key)
    assert (a == d) is False
    # __eq__ ignores nb_bytes (bloom_filter.py:36)
    e = BloomFilter(16, 3, bits=a.bits)
    assert e == a


def test_reference_lsm_negative():
    # test_lsm_storage.py:287-317: m=16, k=3, "baz" must be a negative
    bf = BloomFilter(nb_bytes=2, nb_hash_functions=3)
    for key in ["foo", "bar"]:
        bf.add(key=key)
    assert bf.may_contain("foo") and bf.may_contain("bar")
    assert bf.may_contain("baz") is False


def test_golden_kats_all():
    for c in load_golden("reference_kats.json")["cases"]:
        bf = BloomFilter(c["nb_bytes"], c["k"])
        for key in c["keys"]:
            bf.add(key)
        assert bf.to_bytes().hex() == c["to_bytes_hex"]
        assert bf.bits == int(c["bits"])
        assert [bf.may_contain(p) for p in c["probes"]] == c["probe_results"]


# ---------------------------------------------------------------- index math (any m)
def test_index_math_golden():
    for c in load_golden("index_math.json")["cases"]:
        bf = BloomFilter(c["nb_bytes"], c["k"])
        for key, want in zip(c["keys"], c["indices"]):
            assert bf._hash(key) == want, (c["nb_bytes"], key)
        del bf


def test_large_m_set_bits_both_modes():
    for c in load_golden("large_m.json")["cases"]:
        keys = [f"{i:016d}" for i in range(64)]
        for mode in MODES:
            bf = built(c["nb_bytes"], c["k"], keys, mode)
            bm = np.frombuffer(bf.bitmap(), dtype=np.uint8)
            bits = np.unpackbits(bm, bitorder="little")
            got = np.flatnonzero(bits).tolist()
            assert got == c["set_bits"], (c["nb_bytes"], mode)
            del bf, bm, bits


# ---------------------------------------------------------------- golden bitmaps
def _check_desc(bf, d):
    b = bf.bitmap()
    assert hashlib.sha256(b).hexdigest() == d["sha256"]
    assert bf.popcount() == d["popcount"]
    if "to_bytes_hex" in d:
        assert bf.to_bytes().hex() == d["to_bytes_hex"]


@pytest.mark.parametrize("mode", MODES)
def test_config1_golden(mode):
    g = load_golden("config1.json")
    keys = [f"{i:016d}" for i in range(1000)]
    bf = built(1024, 4, keys, mode)
    _check_desc(bf, g["config1"])
    hm = probe_both(bf, [f"{i:016d}" for i in range(11000)])
    assert hm.tobytes().hex() == g["config1"]["probe_hitmask_hex"]
    bfp = BloomFilter.build_from_keys_and_fp_rate(keys, 0.001)
    _check_desc(bfp, g["product_p0001"])


@pytest.mark.parametrize("mode", MODES)
def test_splitmix_golden(mode):
    g = load_golden("splitmix16.json")
    members = PackedKeys.fixed(splitmix_hex_keys(g["seed"], 0, g["members"]))
    non = PackedKeys.fixed(splitmix_hex_keys(g["seed"], g["nonmember_start"], g["nonmembers"]))
    bf = built(8192, 6, members, mode)
    _check_desc(bf, g["pow2"])
    assert probe_both(bf, non).tobytes().hex() == g["pow2"]["hitmask_nonmembers_hex"]
    bf2 = built(6007, 7, PackedKeys.fixed(splitmix_hex_keys(g["seed"], 0, 5000)), mode)
    _check_desc(bf2, g["odd"])
    assert probe_both(bf2, non).tobytes().hex() == g["odd"]["hitmask_nonmembers_hex"]


@pytest.mark.parametrize("mode", MODES)
def test_varlen_and_unicode_golden(mode):
    g = load_golden("varlen.json")
    d, o = varlen_keys(g["seed"], 0, g["members"])
    bf = built(8192, 8, PackedKeys(d, g["members"], offsets=o), mode)
    _check_desc(bf, g["varlen"])
    d2, o2 = varlen_keys(g["seed"], g["nonmember_start"], g["nonmembers"])
    hm = probe_both(bf, PackedKeys(d2, g["nonmembers"], offsets=o2))
    assert hm.tobytes().hex() == g["varlen"]["hitmask_nonmembers_hex"]
    sk = [(f"{i:08d}" * 8)[:8 + i % 57] for i in range(1000)]
    _check_desc(built(1024, 8, sk, mode), g["survey_family"])
    u = load_golden("unicode.json")
    bfu = built(u["nb_bytes"], u["nb_hash_functions"], u["keys"], mode)
    _check_desc(bfu, u)
    hm = probe_both(bfu, u["keys"] + [f"absent-{i}" for i in range(200)])
    assert hm.tobytes().hex() == u["hitmask_hex"]


# ---------------------------------------------------------------- oracle sweeps
CASES = [
    # (nb_bytes, k, key kind, n)
    (1, 1, "hex16", 100), (3, 2, "hex16", 50), (1000, 3, "hex16", 3000), (6007, 7, "var", 4000),
    (123457, 6, "hex16", 200000), (2 ** 20 + 3, 10, "hex16", 300000), (2 ** 20, 8, "var", 100000),
    (77777, 17, "hex16", 20000), (5000, 33, "var", 3000), (4096, 40, "fixed7", 2000),
    (2 ** 24, 6, "fixed7", 500000), (2 ** 27, 6, "hex16", 1000000), (17971985, 10, "hex16", 1000000),
    # one tile of 2^10..2^12 positions filling its 32..128 words exactly (ceil(m/32) == W): the tile
    # test's bitmap load must not take the 1 KiB LDS-DMA pieces (round-5 advisor)
    (125, 4, "hex16", 600), (128, 3, "var", 500), (253, 5, "hex16", 1200), (256, 4, "fixed7", 1500),
    (509, 6, "var", 2500), (512, 3, "hex16", 3000),
]


def make_keys(kind, n, start=0):
    if kind == "hex16":
        return PackedKeys.fixed(splitmix_hex_keys(11, start, n))
    if kind == "fixed7":
        return PackedKeys.fixed(splitmix_hex_keys(13, start, n)[:, 3:10])
    d, o = varlen_keys(17, start, n)
    return PackedKeys(d, n, offsets=o)


@pytest.mark.parametrize("nb,k,kind,n", CASES)
def test_sweep_against_oracle(oracle, nb, k, kind, n):
    keys = make_keys(kind, n)
    want = oracle.build(nb, k, keys, omp=True)
    probes = make_keys(kind, n // 2 + 7, start=n - n // 4)
    want_hm = oracle.probe(want, k, probes, omp=True)
    for mode in MODES:
        bf = built(nb, k, keys, mode)
        got = np.frombuffer(bf.bitmap(), dtype=np.uint8)
        assert np.array_equal(got, want), (mode, int((got != want).sum()))
        assert np.array_equal(probe_both(bf, probes), want_hm)
        del bf


def test_unaligned_and_odd_lengths(oracle):
    raw = splitmix_hex_keys(5, 0, 5001)
    buf = np.zeros(raw.size + 1, dtype=np.uint8)
    buf[1:] = raw.reshape(-1)
    pk = PackedKeys(buf[1:], 5001, key_len=16)  # 16-byte keys at an odd address → generic path
    assert pk.data.ctypes.data % 16 != 0
    want = oracle.build(3001, 5, pk)
    for mode in MODES:
        assert np.array_equal(np.frombuffer(built(3001, 5, pk, mode).bitmap(), np.uint8), want)
    for L in (1, 2, 3, 4, 5, 9, 15, 31, 33, 63, 64, 65, 200):
        keys = [("x" * L + str(i))[:L] if L else "" for i in range(300)]
        pk = PackedKeys.from_strs(keys)
        want = oracle.build(999, 4, pk)
        for mode in MODES:
            assert np.array_equal(np.frombuffer(built(999, 4, pk, mode).bitmap(), np.uint8), want), L


def test_empty_keys_and_empty_batches(oracle):
    keys = ["", "", "a", ""]
    pk = PackedKeys.from_strs(keys)
    want = oracle.build(64, 5, pk)
    bf = BloomFilter(64, 5)
    bf.add_many(keys)
    assert bf.bitmap() == want.tobytes()
    assert bf.may_contain("") is True
    only_empty = BloomFilter(64, 5)
    only_empty.add_many(["", ""])
    assert only_empty.bitmap() == oracle.build(64, 5, PackedKeys.from_strs([""])).tobytes()
    bf.add_many([])
    assert bf.may_contain_many([]).size == 0
    with pytest.raises(ZeroDivisionError):
        BloomFilter.build_from_keys_and_fp_rate([], 0.001)
    z = BloomFilter(0, 3)
    with pytest.raises(ZeroDivisionError):
        z.add("a")
    assert BloomFilter(0, 0).may_contain("x") is True  # no hash function → vacuous AND
    assert BloomFilter(8, 0).may_contain("x") is True
    with pytest.raises(Exception):  # struct.error, as bloom_filter.py:80
        BloomFilter(8, 300).to_bytes()


@pytest.mark.parametrize("mode", MODES)
def test_incremental_batches(oracle, mode):
    keys = make_keys("hex16", 300000)
    want = oracle.build(2 ** 20, 6, keys, omp=True)
    bf = BloomFilter(2 ** 20, 6)
    bf.set_build_mode(mode)
    for s in range(0, 300000, 70001):
        e = min(300000, s + 70001)
        bf.add_many(PackedKeys.fixed(keys.data.reshape(-1, 16)[s:e]))
    assert np.array_equal(np.frombuffer(bf.bitmap(), np.uint8), want)
    # from_bytes then more adds (non-pristine tiled path)
    half = PackedKeys.fixed(keys.data.reshape(-1, 16)[:150000])
    rest = PackedKeys.fixed(keys.data.reshape(-1, 16)[150000:])
    bf2 = BloomFilter.from_bytes(built(2 ** 20, 6, half).to_bytes())
    bf2.set_build_mode(mode)
    bf2.add_many(rest)
    assert np.array_equal(np.frombuffer(bf2.bitmap(), np.uint8), want)
    bf2.clear()
    assert bf2.popcount() == 0
    bf2.add_many(keys)
    assert np.array_equal(np.frombuffer(bf2.bitmap(), np.uint8), want)


def test_hitmask_tails(oracle):
    keys = make_keys("hex16", 1000)
    want = oracle.build(4096, 6, keys)
    bf = built(4096, 6, keys)
    for n in (1, 7, 8, 9, 63, 64, 65, 127, 129, 1000):
        q = PackedKeys.fixed(keys.data.reshape(-1, 16)[:n])
        assert np.array_equal(probe_both(bf, q), oracle.probe(want, 6, q)), n
        assert bf.may_contain_many(q).all()


def test_stale_region_entries_after_a_larger_probe(oracle):
    """The tile test does not mask a region's last word past its fill (the gather reads only the
    filled entries): a small probe after a larger one on the same scratch — its regions' tails
    hold the larger batch's entries — must still equal the oracle, for one filter and for a
    shared-pipeline set of three (k_tile_probe_set), at an odd key count (partial hit-mask
    words, the hw -> mask conversion)."""
    from pebbledb_amd import may_contain_multi
    nb, k = 2 ** 24, 6  # 128 tiles of 2^20 bits
    members = [PackedKeys.fixed(splitmix_hex_keys(0x57A1E + f, 0, 400_000)) for f in range(3)]
    wants = [oracle.build(nb, k, m, omp=True) for m in members]
    fs = []
    for m in members:
        bf = BloomFilter(nb, k)
        bf.set_build_mode(PBF_BUILD_TILED)
        bf.add_many(m)
        bf.set_probe_mode(PBF_PROBE_TILED)
        fs.append(bf)
    big = PackedKeys.fixed(np.concatenate([splitmix_hex_keys(0x57A1E, 0, 1_500_000),
                                           splitmix_hex_keys(0x99, 0, 1_500_000)]))
    small = PackedKeys.fixed(np.concatenate([splitmix_hex_keys(0x57A1E, 7, 150_000),
                                             splitmix_hex_keys(0x98, 0, 150_001)]))
    for q in (big, small, big, small):
        assert np.array_equal(fs[0].may_contain_many(q, packed=True), oracle.probe(wants[0], k, q, omp=True))
        assert fs[0].last_probe_mode == PBF_PROBE_TILED
        got = may_contain_multi(fs, q)
        for i in range(3):
            assert np.array_equal(got[i], oracle.probe(wants[i], k, q, omp=True)), (q.n, i)


def test_small_host_stage_chunks(oracle, monkeypatch):
    """The host→device chunking path (PBF_STAGE_BYTES) in a child process."""
    import subprocess, sys, os, textwrap
    code = textwrap.dedent("""
        import numpy as np, sys
        sys.path.insert(0, '.')
        from pebbledb_amd import BloomFilter, PackedKeys
        from pebbledb_amd.keys import splitmix_hex_keys, varlen_keys
        from oracle.oracle import COracle
        o = COracle()
        fx = PackedKeys.fixed(splitmix_hex_keys(3, 0, 20000))
        d, off = varlen_keys(3, 0, 20000)
        vr = PackedKeys(d, 20000, offsets=off)
        for pk in (fx, vr):
            for mode in (1, 2):
                bf = BloomFilter(50000, 6); bf.set_build_mode(mode); bf.add_many(pk)
                want = o.build(50000, 6, pk)
                assert bf.bitmap() == want.tobytes()
                for pm in (1, 2):
                    bf.set_probe_mode(pm)
                    assert np.array_equal(bf.may_contain_many(pk, packed=True), o.probe(want, 6, pk))
        print('ok')
    """)
    env = dict(os.environ, PBF_STAGE_BYTES="4099")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_sstable_section_roundtrip_golden():
    """encode_sstable / decode_bloom_section against the reference's own SSTable bytes
    (src/sstable.py:80-100, via tests/golden/sstable_section.json)."""
    from pebbledb_amd.sstable_bloom import decode_bloom_section, encode_sstable
    g = load_golden("sstable_section.json")
    bf = BloomFilter.build_from_keys_and_fp_rate(g["keys"], g["fp_rate"])
    out = encode_sstable(bytes.fromhex(g["data_hex"]), bytes.fromhex(g["meta_hex"]), bf)
    assert bytes(out) == bytes.fromhex(g["sstable_hex"])
    back = decode_bloom_section(out)
    assert back == bf and back.nb_bytes == bf.nb_bytes
    assert all(back.may_contain(k) for k in g["keys"])
    # a big filter through the same path (bitmap copied device → file buffer → device)
    keys = PackedKeys.fixed(splitmix_hex_keys(3, 0, 200000))
    big = BloomFilter.build_from_keys_and_fp_rate(keys, 0.001)
    blob = encode_sstable(b"x" * 1000, b"m" * 77, big)
    again = decode_bloom_section(blob)
    assert again.bitmap() == big.bitmap() and again.nb_hash_functions == big.nb_hash_functions


_PART_CHILD = """
import numpy as np, os, sys
sys.path.insert(0, '.')
from pebbledb_amd import BloomFilter, PackedKeys, _native
from pebbledb_amd.keys import splitmix_hex_keys, varlen_keys
from oracle.oracle import COracle
o = COracle()
# distinct keys, plus one key repeated 60k times: its tiles' regions / rings overflow
distinct = splitmix_hex_keys(21, 0, 200000)
same = np.repeat(splitmix_hex_keys(22, 0, 1), 60000, axis=0)
fx = PackedKeys.fixed(np.concatenate([distinct, same, distinct[:1000]]))
d, off = varlen_keys(23, 0, 100000)
vr = PackedKeys(d, 100000, offsets=off)
# variable-length keys with one key repeated 60k times (the 4096-key sub-chunks' stage windows and
# region overflow together)
k0 = d[int(off[0]):int(off[1])]
vd = PackedKeys(np.concatenate([d, np.tile(k0, 60000)]), 160000,
                offsets=np.concatenate([off, off[-1] + np.uint64(len(k0)) * np.arange(1, 60001, dtype=np.uint64)]))
probes = PackedKeys.fixed(np.concatenate([splitmix_hex_keys(21, 150000, 100000), same,
                                          np.repeat(splitmix_hex_keys(24, 0, 1), 50000, axis=0)]))
# B = 1024 tiles (C2 geometry), 768 (non-power-of-two m), 16 (rings overflow constantly)
for nb, pk, q in ((2 ** 27, fx, probes), (3 * 2 ** 25, vr, vr), (2 ** 21, fx, probes), (2 ** 27 + 12, vr, vr),
                  (2 ** 27, vd, vd)):
    want = o.build(nb, 6, pk, omp=True)
    want_hm = o.probe(want, 6, q, omp=True)
    bf = BloomFilter(nb, 6); bf.set_build_mode(2); bf.add_many(pk)
    assert bf.bitmap() == want.tobytes(), nb
    bf.add_many(pk)  # a second batch onto a non-pristine bitmap
    assert bf.bitmap() == want.tobytes(), nb
    bf.set_probe_mode(2)
    assert np.array_equal(bf.may_contain_many(q, packed=True), want_hm), nb
    assert bf.last_probe_mode == 2 and bf.last_build_mode == 2
    if os.environ.get('PBF_PART') == 'sort':  # exact k = 6: packed entries unless disabled
        assert bool(bf.last_build_detail & _native.PBF_DETAIL_PACKED) == (os.environ.get('PBF_PK3') != '0'), hex(bf.last_build_detail)
# the spill path of a shared multi-filter pipeline (every spilled position tested against each
# filter of the set, ring_kernels.hpp spill_one / tiled_kernels.hpp spill_probe): three filters of
# 16 tiles whose rings overflow constantly, against the oracle
from pebbledb_amd import may_contain_multi
sets = [PackedKeys.fixed(np.concatenate([splitmix_hex_keys(40, f * 10 ** 6, 150000), same])) for f in range(3)]
wants = [o.build(2 ** 21, 6, m, omp=True) for m in sets]
fs = []
for m in sets:
    bf = BloomFilter(2 ** 21, 6); bf.set_build_mode(2); bf.add_many(m); bf.set_probe_mode(2)
    fs.append(bf)
got = may_contain_multi(fs, probes)
assert fs[0].last_probe_mode == 2 and (fs[0].last_probe_detail >> 8) & 0xFF == 3, hex(fs[0].last_probe_detail)
for i in range(3):
    assert np.array_equal(got[i], o.probe(wants[i], 6, probes, omp=True)), i
print('ok')
"""


@pytest.mark.parametrize("part,pk3", [("sort", "1"), ("sort", "0"), ("ring", "1")])
def test_tiled_partition_strategies_and_region_overflow(part, pk3):
    """Both partition passes of the tiled build / probe (PBF_PART forces one; the counting sort's
    build with packed and plain region entries, PBF_PK3), with a key repeated enough to overflow
    its tiles' regions and rings (build overflow list, probe in-place test)."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, PBF_PART=part, PBF_PK3=pk3)
    r = subprocess.run([sys.executable, "-c", _PART_CHILD], env=env, capture_output=True, text=True, timeout=600,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_murmur3_documented_values_and_goldens():
    """pbf_murmur3_x86_32 on the device: mmh3's documented values and the
    reference's own hash of 'key1' with seeds 0..3 (tests/golden)."""
    from pebbledb_amd.bloom_filter import murmur3
    assert murmur3("foo") == -156908512 and murmur3("foo", 42) == -1322301282
    assert [murmur3("key1", s) for s in range(4)] == [-1684602587, 1833321129, 386463789, 201916224]
    for case in load_golden("mmh3_vectors.json")["cases"][:40]:  # seeds 0..15 per key
        key = bytes.fromhex(case["key_hex"])
        assert [murmur3(key, s) for s in (0, 1, 7, 15)] == [case["h"][s] for s in (0, 1, 7, 15)], case["key_hex"]


def test_bits_outside_the_bitmap_are_dropped_like_to_bytes():
    """BloomFilter(nb, k, bits=...) with bits wider than 8*nb or negative: the reference keeps the
    int (bloom_filter.py:31), compares it whole in __eq__ (:36) and only ever reads its low
    8*nb_bytes bits (to_bytes, _is_bit_set) — same bytes, same equality here."""
    wide = (1 << 70) | 0b101
    bf = BloomFilter(8, 3, bits=wide)
    assert bf.to_bytes() == (5).to_bytes(8, "little") + b"\x03"
    assert bf.bits == wide
    assert bf != BloomFilter(8, 3, bits=5) and bf == BloomFilter(8, 3, bits=wide)
    assert BloomFilter(16, 3, bits=wide) == bf  # __eq__ ignores nb_bytes: 2^70 is in 16 B's bitmap
    bf.add("key1")  # the set bit joins the low part, the high part stays
    assert bf.bits >> 64 == 1 << 6 and bf.bits & ((1 << 64) - 1) != 5
    neg = BloomFilter(4, 2, bits=-1)
    assert neg.to_bytes() == b"\xff\xff\xff\xff\x02"
    assert neg.may_contain("anything") and neg.may_contain("")
    assert neg.bits == -1 and neg != BloomFilter(4, 2, bits=0xFFFFFFFF)
