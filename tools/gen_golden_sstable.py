"""Golden SSTable files from the REAL reference's SSTableBuilder (build container only):

    python tools/gen_golden_sstable.py

Writes tests/golden/sstable_build.json: for a few record sets (inputs: keys, values, block
size) the bytes the reference's ``SSTableBuilder.add`` / ``build`` write to disk
(src/sstable.py:209-288 → blocks.py:68-99 DataBlockBuilder, :9-44 DataBlock.to_bytes,
:102-137 MetaBlock, record.py:51-72 Record.to_bytes, sstable.py:80-86 SSTableEncoding), with the
block boundaries.  Small files are stored whole (hex); larger ones as sha256 + length + the
data/meta section sizes.  The reference's mmh3 dependency is the stand-in of tools/mmh3_shim
(see tools/gen_golden.py).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden", "sstable_build.json")
sys.path.insert(0, os.path.join(HERE, "mmh3_shim"))
sys.path.insert(1, "/root/reference")

from src.sstable import SSTableBuilder  # noqa: E402  (the reference)


def value_of(i: int, n: int) -> bytes:
    # deterministic bytes of length n, all byte values represented
    return bytes(((i * 131 + j * 29) & 0xFF) for j in range(n))


def case_records(name: str):
    if name == "small_blocks_unicode":
        keys, vals = [], []
        for i in range(300):
            if i % 50 == 7:
                k = f"clé-{i:04d}"          # 2-byte UTF-8: key_size counts characters (record.py:24)
            elif i % 50 == 31:
                k = f"ключ{i:04d}"          # Cyrillic: every letter 2 bytes
            elif i % 97 == 5:
                k = ""                        # empty key
            else:
                k = f"key{i:05d}"
            keys.append(k)
            vals.append(value_of(i, (i * 7) % 41))  # includes empty values
        return keys, vals, 256
    if name == "default_blocks":
        keys = [f"{i:016x}" for i in range(2500)]
        vals = [value_of(i, 40 + (i % 90)) for i in range(2500)]
        return keys, vals, 65_536
    if name == "exact_fit":
        # records of 64 bytes into 256-byte blocks: each block ends exactly at block_size
        keys = [f"k{i:07d}" for i in range(40)]   # 8 bytes
        vals = [value_of(i, 48) for i in range(40)]  # 4 + 8 + 4 + 48 = 64
        return keys, vals, 256
    raise KeyError(name)


def build(keys, vals, block_size) -> tuple[bytes, list]:
    b = SSTableBuilder(sstable_size=4 << 20, block_size=block_size)
    for k, v in zip(keys, vals):
        b.add(k, v)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "t.sst")
        sst = b.build(path)
        with open(path, "rb") as f:
            data = f.read()
    metas = [{"first_key": m.first_key, "last_key": m.last_key, "offset": m.offset} for m in sst.meta_blocks]
    return data, metas, sst.meta_block_offset


def main() -> None:
    cases = []
    for name in ("small_blocks_unicode", "default_blocks", "exact_fit"):
        keys, vals, bs = case_records(name)
        data, metas, meta_off = build(keys, vals, bs)
        c = {"name": name, "block_size": bs,
             "file_len": len(data), "file_sha256": hashlib.sha256(data).hexdigest(),
             "meta_blocks": metas, "meta_block_offset": meta_off}
        if len(data) <= 64 * 1024:
            c["file_hex"] = data.hex()
            c["keys"] = keys
            c["values_hex"] = [v.hex() for v in vals]
        else:  # inputs by rule (tests/test_sstable_data_cpu.py regenerates them)
            c["keys_rule"] = "f'{i:016x}' for i in range(2500)"
            c["values_rule"] = "bytes(((i * 131 + j * 29) & 0xFF) for j in range(40 + i % 90))"
        cases.append(c)
        print(name, len(data), "bytes,", len(metas), "blocks")
    with open(OUT, "w") as f:
        json.dump({"generator": "tools/gen_golden_sstable.py (reference SSTableBuilder)", "cases": cases}, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
