"""SSTable bloom-section layout (src/sstable.py:57-62, 80-100), host logic only (no GPU)."""
import struct

import pytest

from conftest import load_golden
from pebbledb_amd.sstable_bloom import TRAILER, assemble, bloom_section_bounds, sstable_size


def test_assemble_matches_reference_file_bytes():
    g = load_golden("sstable_section.json")
    data, meta = bytes.fromhex(g["data_hex"]), bytes.fromhex(g["meta_hex"])
    bloom = bytes.fromhex(g["bloom_hex"])
    nb, k = len(bloom) - 1, bloom[-1]

    def write(view):
        view[:] = bloom[:nb]

    out = assemble(data, meta, nb, k, write)
    assert bytes(out) == bytes.fromhex(g["sstable_hex"])
    assert len(out) == sstable_size(len(data), len(meta), nb)
    mo, bo, end = bloom_section_bounds(out)
    assert (mo, bo) == (len(data), len(data) + len(meta))
    assert bytes(out[bo:end]) == bloom


def test_reference_decode_test_file():
    # test_sstable.py:80-97: a file whose bloom section is b'9\x02' and trailer 64/96
    encoded_data = bytes(64)
    meta = bytes(32)
    f = encoded_data + meta + b"9\x02" + b"@\x00\x00\x00" + b"`\x00\x00\x00"
    mo, bo, end = bloom_section_bounds(f)
    assert (mo, bo) == (64, 96) and f[bo:end] == b"9\x02"


def test_bad_trailers_and_k_range():
    with pytest.raises(ValueError):
        bloom_section_bounds(b"\x00" * 4)
    with pytest.raises(ValueError):
        bloom_section_bounds(struct.pack("ii", 5, 2))
    with pytest.raises(struct.error):
        assemble(b"", b"", 1, 256, lambda v: None)
    out = assemble(b"", b"", 0, 3, lambda v: None)
    assert bytes(out) == b"\x03" + struct.pack("ii", 0, 0) and len(out) == 1 + TRAILER
