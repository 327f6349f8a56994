"""pebbledb_amd — MI355X-native bloom-filter engine for pebbledb's per-SSTable filter path.

Drop-in for MaudGautier/pebbledb ``src/bloom_filter.py`` (``BloomFilter``), backed by
hand-written HIP kernels for gfx950 in ``libpebblebloom.so`` (C-ABI: include/pebblebloom.h).
"""
from .bloom_filter import BloomFilter, may_contain_multi, may_contain_set, probe_multi_device, set_default_device
from .keys import PackedKeys

__all__ = ["BloomFilter", "PackedKeys", "may_contain_multi", "may_contain_set", "probe_multi_device", "set_default_device"]
