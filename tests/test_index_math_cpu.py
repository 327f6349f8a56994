"""The device's floor-mod (murmur_device.hpp py_index: Python's `h % bits_size` of the SIGNED
hash, bloom_filter.py:46-47) restated in numpy from the parameters the library computes on the
host (pbf_index_params), checked against Python's own `%` — exhaustively over the edges of every
quotient step and on random hashes, for m of every mode: powers of two, m < 2^30 (the 32-bit
reciprocal, Granlund-Montgomery with N = 31), 2^30 < m < 2^31 (one conditional subtract) and
m >= 2^31.  No GPU: the same arithmetic runs in the kernels."""
import ctypes

import numpy as np
import pytest

from pebbledb_amd import _native


def params(nb_bytes):
    mode, magic, shift = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_uint32()
    _native.check(_native.lib().pbf_index_params(nb_bytes, ctypes.byref(mode), ctypes.byref(magic), ctypes.byref(shift)))
    return mode.value, magic.value, shift.value


def device_index(h: np.ndarray, nb_bytes: int) -> np.ndarray:
    """py_index restated with numpy u32/u64 arithmetic (wrapping as the device's)."""
    m = 8 * nb_bytes
    mode, magic, shift = params(nb_bytes)
    hu = h.astype(np.uint32)
    if mode == 0:
        return (hu & np.uint32(m - 1)).astype(np.uint64)
    if mode == 2:
        return np.where(h >= 0, hu.astype(np.int64), h.astype(np.int64) + m).astype(np.uint64)
    a = np.where(h >= 0, hu, ~hu).astype(np.uint32)
    if mode == 3:
        r = np.where(a >= np.uint32(m), a - np.uint32(m), a).astype(np.uint32)
    else:
        assert mode == 1 and magic < 2 ** 32
        q = ((a.astype(np.uint64) * np.uint64(magic)) >> np.uint64(32)).astype(np.uint32) >> np.uint32(shift)
        r = (a - q * np.uint32(m)).astype(np.uint32)
    return np.where(h >= 0, r.astype(np.uint64), np.uint64(m - 1) - r.astype(np.uint64))


def python_index(h: np.ndarray, m: int) -> np.ndarray:
    return (h.astype(np.int64) % m).astype(np.uint64)  # numpy % on int64 = Python floor-mod


# every mode, edge sizes of each: tiny, SSTable product sizes (fp 0.001), C4's 224,649,806 B,
# just under / over 2^27 B and 2^28 B (m = 2^30, 2^31), non-multiples of 4, C3's 2^30 B
NB = [3, 5, 7, 13, 127, 1023, 1025, 1798, 17_971_985, 224_649_806, 2 ** 27 - 1, 2 ** 27 + 1, 2 ** 27 + 12345,
      2 ** 28 - 3, 2 ** 28 + 7, 2 ** 29 + 3, 2 ** 30, 2 ** 30 + 5, 1024, 2 ** 27, 2 ** 25, 3 << 20, 200_000_001]


@pytest.mark.parametrize("nb", NB)
def test_index_params_match_python_floor_mod(nb):
    m = 8 * nb
    mode, magic, shift = params(nb)
    pow2 = (m & (m - 1)) == 0
    assert mode == (0 if pow2 and m <= 2 ** 32 else 1 if m < 2 ** 30 else 3 if m < 2 ** 31 else 2)
    rng = np.random.default_rng(nb)
    h = [rng.integers(-2 ** 31, 2 ** 31, 400_000, dtype=np.int64)]
    # the edges of every quotient step a = q*m - 1, q*m, q*m + 1 for a < 2^31 (sampled q when
    # there are many), as +a and as the negative hash ~a
    qmax = (2 ** 31 - 1) // m
    qs = np.unique(np.concatenate([np.arange(0, min(qmax, 4096) + 1),
                                   rng.integers(0, qmax + 1, 4096), [qmax]]))
    edges = (qs[:, None] * m + np.array([-1, 0, 1])[None, :]).reshape(-1)
    edges = edges[(edges >= 0) & (edges < 2 ** 31)]
    h.append(edges)
    h.append(~edges)
    h.append(np.array([0, -1, 2 ** 31 - 1, -2 ** 31, 1, -2], dtype=np.int64))
    h = np.concatenate(h).astype(np.int32)
    assert np.array_equal(device_index(h, nb), python_index(h, m))
