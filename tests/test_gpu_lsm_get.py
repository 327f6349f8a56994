"""Batched LsmStorage.get filter stage (src/lsm_storage.py:153-179) on
an MI355X (`-m gpu`): the device key-range pre-check against Python's own ``str`` comparison,
and the full candidate order against a restatement of the reference loop
(oracle/lsm_get_oracle.py) on a fixture with overlapping and disjoint level ranges."""
import ctypes
import random

import numpy as np
import pytest

from pebbledb_amd import BloomFilter, PackedKeys
from pebbledb_amd import _native
from pebbledb_amd.lsm_get import LevelTable, candidate_lists, candidate_masks, candidates_one, key_range_masks
from conftest import load_golden

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ALPH = "ab\x7f\u0080é￿\U0001f511z0"


def _rand_keys(rng, n, lo=0, hi=12):
    return ["".join(rng.choice(ALPH) for _ in range(rng.randint(lo, hi))) for _ in range(n)]


def _want_ranges(keys, bounds):
    return np.array([[f <= k <= l for k in keys] for f, l in bounds])


def test_range_mask_equals_python_str_order():
    """Code points spanning 1..4 UTF-8 bytes, prefixes, empty keys and bounds, first > last
    (an empty range) and equal bounds: bytewise compare of UTF-8 == Python str order."""
    rng = random.Random(7)
    keys = _rand_keys(rng, 3001) + ["", "a", "ab", "abz", "é", "\U0001f511"]
    bounds = [("", "\U0010ffff"), ("a", "ab"), ("ab", "ab"), ("b", "a"), ("", ""), ("é", "￿"),
              ("\x7f", "\u0080"), ("a\U0001f511", "z")]
    bounds += [tuple(sorted(_rand_keys(rng, 2, 0, 6))) for _ in range(40)]
    got = key_range_masks(keys, bounds)
    want = _want_ranges(keys, bounds)
    bits = np.unpackbits(got, axis=1, bitorder="little")[:, :len(keys)].astype(bool)
    assert np.array_equal(bits, want)
    # fixed-width keys take the key_len path
    fx = ["%08d" % i for i in range(0, 90000, 7)]
    bfx = [("00001000", "00002000"), ("0000500", "00005001"), ("00089999", "99")]
    got = np.unpackbits(key_range_masks(PackedKeys.from_strs(fx), bfx), axis=1, bitorder="little")[:, :len(fx)]
    assert np.array_equal(got.astype(bool), _want_ranges(fx, bfx))


def test_range_mask_device_resident_and_many_tables():
    """Device pointers (on_device = 1, asynchronous on a stream) and enough long bounds that the
    tables are split over several LDS-sized launches."""
    rng = random.Random(9)
    keys = sorted(_rand_keys(rng, 20000, 1, 40))
    bounds = []
    for _ in range(700):
        a, b = sorted(_rand_keys(rng, 2, 60, 200))
        bounds.append((a, b))
    pk = PackedKeys.from_strs(keys)
    want = _want_ranges(keys, bounds)
    host = np.unpackbits(key_range_masks(pk, bounds), axis=1, bitorder="little")[:, :len(keys)].astype(bool)
    assert np.array_equal(host, want)
    enc = [s.encode() for p in bounds for s in p]
    bo = np.zeros(len(enc) + 1, np.uint64)
    np.cumsum([len(e) for e in enc], out=bo[1:])
    d = {name: torch.from_numpy((a.view(np.int64) if a.dtype == np.uint64 else a).copy()).cuda()
         for name, a in (("k", pk.data), ("ko", pk.offsets), ("b", np.frombuffer(b"".join(enc), np.uint8).copy()),
                         ("bo", bo))}
    out = torch.zeros(len(bounds) * ((len(keys) + 7) // 8), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    s = torch.cuda.current_stream().cuda_stream
    vp = ctypes.c_void_p
    _native.check(_native.lib().pbf_key_range_mask(0, vp(s), vp(d["k"].data_ptr()), vp(d["ko"].data_ptr()), 0,
                                                   len(keys), vp(d["b"].data_ptr()), vp(d["bo"].data_ptr()),
                                                   len(bounds), vp(out.data_ptr()), 1), "range")
    torch.cuda.synchronize()
    dev = np.unpackbits(out.cpu().numpy().reshape(len(bounds), -1), axis=1, bitorder="little")[:, :len(keys)]
    assert np.array_equal(dev.astype(bool), want)


def test_candidate_order_equals_reference_get_loop(oracle):
    """L0 (3 filters of different sizes, overlapping key sets, newest first) + L1 (4 disjoint
    ranges) + L2 (overlapping ranges, a one-key table and a table no probe key reaches): for
    every probe key the SSTables the reference's get would read, in its order."""
    from oracle.lsm_get_oracle import reference_candidates
    rng = random.Random(3)
    universe = sorted(set("k%06d" % i for i in range(60000)) | set(_rand_keys(rng, 3000, 1, 10)))
    sample = lambda a, b, step: universe[a:b:step]  # noqa: E731
    l0_sets = [sample(0, 30000, 3), sample(10000, 50000, 2), sample(20000, 63000, 5)]
    l0 = []
    l0_o = []
    for i, ks in enumerate(l0_sets):
        nb, k = [(4096, 5), (30011, 7), (2 ** 14, 6)][i]
        bf = BloomFilter(nb, k)
        bf.add_many(ks)
        l0.append(bf)
        l0_o.append((oracle.build(nb, k, PackedKeys.from_strs(ks)), k))
    levels, levels_o = [], []
    for spec in ([(0, 15000), (15000, 30000), (30000, 45000), (45000, len(universe))],
                 [(5000, 25000), (20000, 40000), (33333, 33334), (len(universe) - 5, len(universe))]):
        lvl, lvl_o = [], []
        for a, b in spec:
            ks = universe[a:b]
            bf = BloomFilter(2 ** 13, 6)
            bf.add_many(ks)
            lvl.append(LevelTable(ks[0], ks[-1], bf))
            lvl_o.append((ks[0], ks[-1], oracle.build(2 ** 13, 6, PackedKeys.from_strs(ks)), 6))
        levels.append(lvl)
        levels_o.append(lvl_o)
    # probe: members, non-members between them, keys beyond every range, unicode
    probes = universe[::11] + ["k%06d5" % i for i in range(0, 60000, 97)] + ["", "zzz", "\U0001f511", "a"]
    probes = [p for p in probes if p < universe[-5]]  # so the last L2 table is never reached
    masks = candidate_masks(probes, l0, levels)
    got = candidate_lists(masks, len(probes))
    want = reference_candidates(probes, l0_o, levels_o)
    assert got == want
    assert not masks[len(l0) + 7].any()  # the unreached L2 table
    assert any(len(c) > 3 for c in got)  # the fixture exercises several levels per key


def _golden_store():
    """The store of tests/golden/lsm_get_order.json (tools/gen_golden_lsm.py: the REAL
    reference's LsmStorage.get, src/lsm_storage.py:153-181, with every SSTable.get recorded):
    each table's filter built here with the product sizing (sstable.py:274) and checked against
    the reference's own bitmap."""
    import hashlib
    g = load_golden("lsm_get_order.json")
    U = g["universe"]
    l0, levels = [], [[], []]
    for t in g["tables"]:
        keys = U[t["start"]:t["stop"]:t["step"]]
        bf = BloomFilter.build_from_keys_and_fp_rate(keys, g["fp_rate"])
        assert (bf.nb_bytes, bf.nb_hash_functions) == (t["nb_bytes"], t["k"])
        bm = bf.bitmap()
        assert hashlib.sha256(bm).hexdigest() == t["sha256"] and sum(bin(b).count("1") for b in bm) == t["popcount"]
        assert (keys[0], keys[-1]) == (t["first_key"], t["last_key"])
        if t["level"] == 0:
            l0.append(bf)
        else:
            levels[t["level"] - 1].append(LevelTable(t["first_key"], t["last_key"], bf))
    return g, l0, levels


def test_candidate_order_equals_reference_lsm_get_golden():
    """Batched filter stage (candidate_masks: mixed-size L0 filters through the fused multi-filter
    probe, level ranges on the device) == the SSTable reads the real reference's get made."""
    g, l0, levels = _golden_store()
    masks = candidate_masks(g["probes"], l0, levels)
    assert candidate_lists(masks, len(g["probes"])) == g["order"]
    assert l0[0].last_probe_detail & _native.PBF_DETAIL_SET  # mixed sizes: one fused launch


def test_per_key_get_one_launch_equals_reference_lsm_get_golden():
    """The per-key form (candidates_one: host range check + ONE pbf_may_contain_set launch over
    the L0 and in-range level filters, all of different sizes) == the reference's get, key by key."""
    g, l0, levels = _golden_store()
    for key, want in zip(g["probes"], g["order"]):
        assert candidates_one(key, l0, levels) == want, key
    assert l0[0].last_probe_detail == (_native.PBF_DETAIL_ONE_KEY | _native.PBF_DETAIL_SET
                                       | _native.PBF_DETAIL_RESIDENT)
