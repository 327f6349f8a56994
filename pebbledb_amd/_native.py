"""ctypes binding of libpebblebloom.so (include/pebblebloom.h).

There is no fallback: if the library is missing or fails to load, every product call raises.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# PBF_LIB: an alternative build of the same library (A/B measurements of kernel variants)
LIB_PATH = os.environ.get("PBF_LIB") or os.path.join(_HERE, "libpebblebloom.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "pebblebloom.h")

PBF_OK = 0
PBF_ERR_INVALID = -1
PBF_ERR_HIP = -2
PBF_ERR_ZERO_SIZE = -3
PBF_BUILD_AUTO, PBF_BUILD_ATOMIC, PBF_BUILD_TILED = 0, 1, 2
PBF_PROBE_AUTO, PBF_PROBE_DIRECT, PBF_PROBE_TILED = 0, 1, 2
PBF_DETAIL_RING, PBF_DETAIL_SORT, PBF_DETAIL_ONE_KEY, PBF_DETAIL_SET, PBF_DETAIL_PACKED = 1, 2, 4, 8, 16
PBF_DETAIL_SHARED = 32
PBF_DETAIL_RESIDENT = 64
PBF_COPY_BOUNCE = 1

_u8p = ctypes.c_void_p
_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64
_u32 = ctypes.c_uint32
_int = ctypes.c_int

# name → (restype, argtypes); must cover every function declared in include/pebblebloom.h
SIGNATURES = {
    "pbf_version": (_int, []),
    "pbf_device_count": (_int, [ctypes.POINTER(_int)]),
    "pbf_create": (_int, [_int, _u64, _u32, ctypes.POINTER(_vp)]),
    "pbf_destroy": (_int, [_vp]),
    "pbf_clear": (_int, [_vp]),
    "pbf_add_fixed": (_int, [_vp, _u8p, _u32, _u64, _int]),
    "pbf_add": (_int, [_vp, _u8p, _vp, _u64, _int]),
    "pbf_build": (_int, [_vp, _u8p, _vp, _u64, _int]),
    "pbf_murmur3_x86_32": (_int, [_int, ctypes.c_char_p, _u64, _u32, ctypes.POINTER(ctypes.c_int32)]),
    "pbf_resident_launches": (_int, [_int, ctypes.POINTER(_u32)]),
    "pbf_resident_stats": (_int, [_int, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "pbf_resident_enable": (_int, [_int]),
    "pbf_probe_fixed": (_int, [_vp, _u8p, _u32, _u64, _u8p, _int]),
    "pbf_probe": (_int, [_vp, _u8p, _vp, _u64, _u8p, _int]),
    "pbf_probe_multi_fixed": (_int, [_vp, _u32, _u8p, _u32, _u64, _vp, _int]),
    "pbf_probe_multi": (_int, [_vp, _u32, _u8p, _vp, _u64, _vp, _int]),
    "pbf_probe_multi_placed": (_int, [_vp, _u32, _vp, _u8p, _vp, _u32, _u64, _vp]),
    "pbf_plan_groups": (_int, [_vp, _vp, _u32, _vp, _vp]),
    "pbf_hash_indices_fixed": (_int, [_vp, _u8p, _u32, _u64, _vp, _int]),
    "pbf_hash_indices": (_int, [_vp, _u8p, _vp, _u64, _vp, _int]),
    "pbf_get_bitmap": (_int, [_vp, _u8p, _u64]),
    "pbf_set_bitmap": (_int, [_vp, _u8p, _u64]),
    "pbf_popcount": (_int, [_vp, ctypes.POINTER(_u64)]),
    "pbf_set_bitmap_device": (_int, [_vp, _vp, _u64]),
    "pbf_get_bitmap_device": (_int, [_vp, _vp, _u64]),
    "pbf_copy_filter": (_int, [_vp, _int, _int, ctypes.POINTER(_vp)]),
    "pbf_sync": (_int, [_vp]),
    "pbf_stream": (_vp, [_vp]),
    "pbf_index_params": (_int, [_u64, ctypes.POINTER(_u32), ctypes.POINTER(_u64), ctypes.POINTER(_u32)]),
    "pbf_wait_stream": (_int, [_vp, _vp]),
    "pbf_signal_stream": (_int, [_vp, _vp]),
    "pbf_device_bitmap": (_vp, [_vp]),
    "pbf_set_build_mode": (_int, [_vp, _int]),
    "pbf_last_build_mode": (_int, [_vp]),
    "pbf_set_probe_mode": (_int, [_vp, _int]),
    "pbf_last_probe_mode": (_int, [_vp]),
    "pbf_last_probe_detail": (_u32, [_vp]),
    "pbf_last_build_detail": (_u32, [_vp]),
    "pbf_may_contain": (_int, [_vp, ctypes.c_char_p, _u64, ctypes.POINTER(_int)]),
    "pbf_may_contain_set": (_int, [_vp, _u32, ctypes.c_char_p, _u64, _u8p]),
    "pbf_trim": (_int, [_int]),
    "pbf_scratch_bytes": (_int, [_int, ctypes.POINTER(_u64)]),
    "pbf_encode_data_blocks": (_int, [_int, _u8p, _vp, _u8p, _vp, _u64, _vp, _vp, _u64, _u8p, _int]),
    "pbf_build_sstable": (_int, [_vp, _u8p, _vp, _u8p, _vp, _u64, _vp, _vp, _u64, _u8p, _u8p]),
    "pbf_build_sstables": (_int, [_vp, _u32, _u8p, _vp, _u8p, _vp, _u64, _vp, _vp, _u64, _vp, _vp, _vp]),
    "pbf_plan_compaction": (_int, [_vp, _vp, _u64, _u64, _u64, _vp, _vp, _vp, ctypes.POINTER(_u64), ctypes.POINTER(_u64),
                                   ctypes.POINTER(_u64)]),
    "pbf_plan_blocks": (_int, [_vp, _vp, _u64, _u64, _vp, _vp, ctypes.POINTER(_u64)]),
    "pbf_key_range_mask": (_int, [_int, _vp, _u8p, _vp, _u32, _u64, _u8p, _vp, _u32, _u8p, _int]),
    "pbf_gen_splitmix_hex": (_int, [_int, _vp, _u8p, _u64, _u64, _u64]),
    "pbf_gen_varlen": (_int, [_int, _vp, _u8p, _vp, _u64, _u64, _u64]),
    "pbf_last_error": (ctypes.c_char_p, []),
    "pbf_source_digest": (ctypes.c_char_p, []),
}

_lib = None


class NativeError(RuntimeError):
    pass


def header_functions() -> list[str]:
    """Every function name declared in include/pebblebloom.h."""
    with open(HEADER) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(pbf_\w+)\s*\(", text, re.M)))


def lib():
    """Load libpebblebloom.so (built by pebbledb_amd/build.py); raise loudly if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(there is no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    # a library compiled from other kernel sources than the tree's is never used (a prebuilt .so
    # travels to the GPU box with the tree): build() rebuilds it
    from . import build
    have, want = L.pbf_source_digest().decode(), build.source_digest()
    if have != want:
        raise NativeError(f"{LIB_PATH} is stale: compiled from sources {have[:16]}, the tree's are {want[:16]}; "
                          "run `python -c 'import __graft_entry__ as g; g.build()'`")
    _lib = L
    return L


def lib_path() -> str:
    """Path of the loaded libpebblebloom.so (PBF_LIB overrides, for A/B builds)."""
    return LIB_PATH


def check(rc: int, what: str = "") -> None:
    if rc == PBF_OK:
        return
    msg = lib().pbf_last_error().decode(errors="replace")
    if rc == PBF_ERR_ZERO_SIZE:
        raise ZeroDivisionError("integer modulo by zero")
    if rc == PBF_ERR_INVALID:
        raise ValueError(f"{what}: {msg}")
    raise NativeError(f"{what}: HIP failure: {msg}")


def device_count() -> int:
    n = _int(0)
    check(lib().pbf_device_count(ctypes.byref(n)), "pbf_device_count")
    return n.value
