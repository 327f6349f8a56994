"""Generate the committed golden fixtures under tests/golden/ from the REAL reference.

Runs only in the build container (``/root/reference`` does not exist on the GPU box):

    python tools/gen_golden.py

It imports the reference's own ``src.bloom_filter.BloomFilter`` (and ``src.sstable`` for the
bloom section of an SSTable file) from /root/reference.  The reference's one third-party
dependency, ``mmh3==4.1.0`` (reference requirements.txt:12), is not installed; the stand-in in
``tools/mmh3_shim`` maps ``mmh3.hash`` onto scikit-learn's compiled MurmurHash3_x86_32.  The
stand-in is pinned by mmh3's documented values (written to mmh3_documented.json and checked in
tests/test_oracle_golden.py) and by the reference's own known-answer bytes.

Every fixture is data: inputs (keys, nb_bytes, k) and the outputs the reference computed.
Large bitmaps are stored as sha256 + popcount + a short prefix; small ones in full (hex).
"""
from __future__ import annotations

import hashlib
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(HERE, "mmh3_shim"))
sys.path.insert(1, "/root/reference")
sys.path.insert(2, REPO)

import mmh3  # noqa: E402  (the stand-in)
from src.bloom_filter import BloomFilter  # noqa: E402  (the reference, bloom_filter.py:8)

from pebbledb_amd.keys import splitmix_hex_keys_str, varlen_keys_str  # noqa: E402


def bitmap_bytes(bf) -> bytes:
    # == bf.to_bytes()[:-1] (bloom_filter.py:76-81) without the quadratic loop; equality is
    # asserted below on every filter small enough to run to_bytes() itself.
    return bf.bits.to_bytes(bf.nb_bytes, "little")


def describe(bf, full_limit=4096) -> dict:
    bm = bitmap_bytes(bf)
    d = {
        "nb_bytes": bf.nb_bytes,
        "nb_hash_functions": bf.nb_hash_functions,
        "popcount": bin(bf.bits).count("1"),
        "sha256": hashlib.sha256(bm).hexdigest(),
        "prefix_hex": bm[:32].hex(),
    }
    if bf.nb_bytes <= full_limit:
        tb = bf.to_bytes()
        assert tb[:-1] == bm and tb[-1] == bf.nb_hash_functions
        d["to_bytes_hex"] = tb.hex()
    return d


def hitmask(bf, keys) -> str:
    out = bytearray((len(keys) + 7) // 8)
    for i, k in enumerate(keys):
        if bf.may_contain(k):
            out[i >> 3] |= 1 << (i & 7)
    return bytes(out).hex()


def build(nb_bytes, k, keys):
    bf = BloomFilter(nb_bytes=nb_bytes, nb_hash_functions=k)
    for key in keys:
        bf.add(key)
    return bf


def dump(name, obj):
    os.makedirs(OUT, exist_ok=True)
    print("writing", name, flush=True)
    with open(os.path.join(OUT, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", name)


def main():
    if "--tail" in sys.argv:
        return tail()
    # 1. mmh3 documented values (mmh3 README) through the stand-in, plus a hash table over
    #    lengths 0..72 (every tail case), unicode, and seeds 0..15.
    dump("mmh3_documented.json", {
        "cases": [
            {"key": "foo", "seed": 0, "signed": -156908512},
            {"key": "foo", "seed": 42, "signed": -1322301282},
            {"key": "foo", "seed": 0, "unsigned": 4138058784},
        ],
        "stand_in_values": [mmh3.hash("foo"), mmh3.hash("foo", 42), mmh3.hash("foo", signed=False)],
    })
    hash_cases = []
    base = "The quick brown fox jumps over the lazy dog 0123456789 abcdefghijklmnopqrstuvwxyz"
    for L in range(0, 73):
        key = base[:L]
        hash_cases.append({"key_hex": key.encode().hex(), "h": [mmh3.hash(key.encode(), s) for s in range(16)]})
    for key in ["clé", "日本語のキー", "emoji-\U0001F600", "\x00\x01\x02\xff", "key1", "key2", "key3"]:
        enc = key.encode("utf-8")
        hash_cases.append({"key_hex": enc.hex(), "h": [mmh3.hash(enc, s) for s in range(16)]})
    # large seeds (k up to 255 → seeds up to 254)
    for s in (100, 200, 254):
        hash_cases.append({"key_hex": b"seed-test-key".hex(), "seed": s, "h1": mmh3.hash(b"seed-test-key", s)})
    dump("mmh3_vectors.json", {"cases": hash_cases})

    # 2. The reference's own known-answer tests (src/__tests__/test_bloom_filter.py,
    #    test_lsm_storage.py:287-317, src/__fixtures__/bloom_filter.py:6-22), recomputed.
    kats = []
    for (nb, k, keys, probes) in [
        (4, 3, ["foo", "bar", "baz"], ["foo", "bar", "baz", "not_in_bloom_filter", "missing"]),
        (1, 2, ["key1", "key2", "key3"], ["key1", "key4"]),
        (3, 2, ["key1", "key2", "key3"], ["key1", "key4"]),
        (2, 3, ["foo", "bar"], ["foo", "bar", "baz"]),
        (10, 3, ["key1", "key2", "key3", "key5", "key9"], ["key1", "key4", "key6"]),
        (10, 3, ["key1", "key2", "key3"], ["key1", "key5"]),
        (8, 3, ["key1", "key2", "key3"], ["key1"]),
        (8, 4, ["key1", "key2", "key3"], ["key1"]),
    ]:
        bf = build(nb, k, keys)
        kats.append({"nb_bytes": nb, "k": k, "keys": keys, "to_bytes_hex": bf.to_bytes().hex(),
                     "bits": str(bf.bits), "probes": probes,
                     "probe_results": [bf.may_contain(p) for p in probes]})
    dump("reference_kats.json", {"cases": kats})

    # 3. Index math (bloom_filter.py:38-49): the reference's own _hash() for many bits_size
    #    values: powers of two, odd / non-power-of-two m, m >= 2^31 (64-bit indices).
    idx_cases = []
    keys = ["key1", "foo", "0000000000000042", "a" * 40, "日本", ""] + [f"{i:016d}" for i in range(0, 50, 7)]
    for nb in [1, 3, 6, 7, 1024, 1798, 123457, 2 ** 27, 17971985, 2 ** 28 - 1, 2 ** 28, 2 ** 28 + 3,
               224649806, 2 ** 30, 2 ** 30 + 5, 3 * 2 ** 30]:
        bf = BloomFilter(nb_bytes=nb, nb_hash_functions=8)
        idx_cases.append({"nb_bytes": nb, "k": 8, "keys": keys, "indices": [bf._hash(kk) for kk in keys]})
    dump("index_math.json", {"cases": idx_cases})

    # 4. Sizing (bloom_filter.py:92-114) — nb_bytes and k for many (n, p) through the
    #    reference's classmethod itself (keys are irrelevant to sizing).
    sizing = []
    for n in [1, 2, 3, 5, 10, 100, 999, 1000, 1001, 2000]:
        for p in [0.5, 0.1, 0.01, 0.001, 0.0001, 1e-6]:
            bf = BloomFilter.build_from_keys_and_fp_rate([f"k{i}" for i in range(n)], p)
            sizing.append({"n": n, "p": p, "nb_bytes": bf.nb_bytes, "k": bf.nb_hash_functions})
    dump("sizing.json", {"cases": sizing})

    # 5. Config-1 (BASELINE.json configs[0]): 1000 keys f"{i:016d}", nb_bytes=1024, k=4,
    #    full bytes + probe hit mask of keys 0..10999 (1000 members, 10000 non-members).
    c1_keys = [f"{i:016d}" for i in range(1000)]
    bf = build(1024, 4, c1_keys)
    c1 = describe(bf)
    c1["probe_hitmask_hex"] = hitmask(bf, [f"{i:016d}" for i in range(11000)])
    c1["keys"] = "f'{i:016d}' for i in range(1000)"
    # product path at p=0.001 on the same keys (sstable.py:274)
    bfp = BloomFilter.build_from_keys_and_fp_rate(c1_keys, 0.001)
    c1_prod = describe(bfp)
    c1_prod["fp_rate"] = 0.001
    dump("config1.json", {"config1": c1, "product_p0001": c1_prod})

    # 6. The bench's synthetic key stream (pebbledb_amd/keys.py): 16-char lowercase hex of
    #    splitmix64(seed + i); 20000 members into nb_bytes=8192 (m=65536), k=6, + probes.
    sm = splitmix_hex_keys_str(0x5EEDB100, 0, 20000)
    sm_probe = splitmix_hex_keys_str(0x5EEDB100, 20000, 4000)
    bf = build(8192, 6, sm)
    d = describe(bf)
    d["keys_first"] = sm[:4]
    d["hitmask_members_first2048_hex"] = hitmask(bf, sm[:2048])
    d["hitmask_nonmembers_hex"] = hitmask(bf, sm_probe)
    # non-power-of-two m (nb_bytes=6007 → m=48056) and odd nb_bytes (tail byte), k=7
    bf2 = build(6007, 7, sm[:5000])
    d2 = describe(bf2, full_limit=0)
    d2["hitmask_nonmembers_hex"] = hitmask(bf2, sm_probe)
    dump("splitmix16.json", {"seed": 0x5EEDB100, "pow2": d, "odd": d2,
                             "members": 20000, "nonmember_start": 20000, "nonmembers": 4000})

    # 7. Variable-length keys (8..64 bytes, config-3 alphabet), m=8192*8, k=8; plus the
    #    survey's (f"{i:08d}"*8)[:8+i%57] family, m=8192, k=8.
    vk = varlen_keys_str(0xC3, 0, 3000)
    vprobe = varlen_keys_str(0xC3, 3000, 2000)
    bf = build(8192, 8, vk)
    dv = describe(bf, full_limit=0)
    dv["hitmask_nonmembers_hex"] = hitmask(bf, vprobe)
    dv["keys_first"] = vk[:3]
    sk = [(f"{i:08d}" * 8)[:8 + i % 57] for i in range(1000)]
    bfs = build(1024, 8, sk)
    dump("varlen.json", {"seed": 0xC3, "members": 3000, "nonmember_start": 3000, "nonmembers": 2000,
                         "varlen": dv, "survey_family": describe(bfs)})

    # 8. Unicode keys (UTF-8 encoding, bloom_filter.py:43) with a non-power-of-two m.
    uk = [f"clé-{i}-日本-{'é' * (i % 9)}" for i in range(500)]
    bf = build(999, 5, uk)
    du = describe(bf)
    du["keys"] = uk
    du["hitmask_hex"] = hitmask(bf, uk + [f"absent-{i}" for i in range(200)])
    dump("unicode.json", du)
    tail()


def tail():
    # 9. Large m (m >= 2^31): only [0,2^31) u [m-2^31, m) reachable.  Building these through
    #    the reference's add() materialises multi-GiB Python ints per bit (bloom_filter.py:53),
    #    so the set bits are taken as the union of the reference's own _hash() indices, which
    #    is exactly what add() ORs in (bloom_filter.py:60-65).
    big = []
    for nb in [2 ** 28, 2 ** 30, 3 * 2 ** 30]:
        bf = BloomFilter(nb_bytes=nb, nb_hash_functions=8)
        pos = sorted({b for i in range(64) for b in bf._hash(f"{i:016d}")})
        big.append({"nb_bytes": nb, "k": 8, "keys": "f'{i:016d}' for i in range(64)", "set_bits": pos})
    dump("large_m.json", {"cases": big})

    # 10. SSTable bloom section (sstable.py:57-62, 80-86): the bytes the reference writes
    #     between the meta blocks and the offset trailer, for a 3-key SSTable.
    from src.blocks import DataBlock, MetaBlock
    from src.sstable import SSTableEncoding
    data1 = b'\x04\x00\x00\x00key1\x06\x00\x00\x00value1\x04\x00\x00\x00key2\x06\x00\x00\x00value2'
    block1 = DataBlock(data=data1, offsets=[0, 18])
    data2 = b'\x04\x00\x00\x00key3\x06\x00\x00\x00value3'
    block2 = DataBlock(data=data2, offsets=[0])
    data = block1.to_bytes() + block2.to_bytes()
    mb = [MetaBlock(first_key="key1", last_key="key2", offset=0), MetaBlock(first_key="key3", last_key="key3", offset=42)]
    bf = BloomFilter.build_from_keys_and_fp_rate(["key1", "key2", "key3"], fp_rate=0.001)
    enc = SSTableEncoding(data=data, meta_blocks=mb, bloom_filter=bf).to_bytes()
    dump("sstable_section.json", {"keys": ["key1", "key2", "key3"], "fp_rate": 0.001,
                                  "data_hex": data.hex(),
                                  "meta_hex": b"".join(m.to_bytes() for m in mb).hex(),
                                  "sstable_hex": enc.hex(), "bloom_hex": bf.to_bytes().hex()})


if __name__ == "__main__":
    main()
