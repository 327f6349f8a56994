"""Offline stand-in for the third-party ``mmh3==4.1.0`` module (reference requirements.txt:12).

Used ONLY by ``tools/gen_golden.py`` in the build container to import the reference's
``src/bloom_filter.py`` (which does ``import mmh3`` at bloom_filter.py:5 and calls
``mmh3.hash(bytes, seed)`` at bloom_filter.py:46).  ``mmh3`` is not installed and there is no
network; scikit-learn ships an independent compiled MurmurHash3_x86_32, which is what
``mmh3.hash`` computes.  Equality with mmh3 4.1.0 is pinned by mmh3's documented values
(see tests/golden/mmh3_documented.json) and by the reference's own known-answer tests.
Never shipped to the GPU box, never imported by the product.
"""
from sklearn.utils.murmurhash import murmurhash3_32 as _mm


def hash(key, seed=0, signed=True):  # noqa: A001 - mirrors mmh3.hash's name
    if isinstance(key, str):
        key = key.encode("utf-8")
    return int(_mm(bytes(key), seed=seed, positive=not signed))
