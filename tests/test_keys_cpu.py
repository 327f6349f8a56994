"""Host key packing (PackedKeys.from_strs): the boundary layout of bloom_filter.py:43's
`key.encode("utf-8")` for a batch, on the fast joined path (all ASCII) and the per-key path."""
import numpy as np
import pytest

from pebbledb_amd.keys import PackedKeys, splitmix_hex_keys, splitmix_hex_keys_str


def _naive(keys):
    enc = [k.encode("utf-8") for k in keys]
    return b"".join(enc), [len(e) for e in enc]


@pytest.mark.parametrize("keys", [
    ["key1", "key2", "key3"],                      # fixed width
    ["a", "", "bcd", "efgh" * 20],                 # ragged, with an empty key
    ["héllo", "wörld", "ascii", "日本語", ""],      # multi-byte: per-key path
    ["ß" * 3, "abc"],                              # same char count, different byte counts
    [""] * 5,                                      # all empty
])
def test_from_strs_matches_per_key_encoding(keys):
    pk = PackedKeys.from_strs(keys)
    data, lens = _naive(keys)
    assert pk.n == len(keys)
    assert pk.data.tobytes() == data
    for i in range(len(keys)):
        assert pk.key(i) == keys[i].encode("utf-8")
    if pk.key_len == 0:
        assert list(np.diff(pk.offsets.astype(np.int64))) == lens


def test_from_strs_fixed_hex_equals_numpy_generator():
    pk = PackedKeys.from_strs(splitmix_hex_keys_str(7, 100, 5000))
    assert pk.key_len == 16
    assert np.array_equal(pk.data.reshape(-1, 16), splitmix_hex_keys(7, 100, 5000))


def test_from_strs_accepts_iterables():
    pk = PackedKeys.from_strs(k for k in ["x", "yy"])
    assert pk.n == 2 and pk.key(1) == b"yy"
