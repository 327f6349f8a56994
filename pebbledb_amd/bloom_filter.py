"""``BloomFilter`` — drop-in for MaudGautier/pebbledb ``src/bloom_filter.py`` on MI355X.

Same constructor, attributes and methods as the reference class (bloom_filter.py:8-119):
``BloomFilter(nb_bytes, nb_hash_functions, bits=None)``, ``add``, ``may_contain``,
``to_bytes``, ``from_bytes``, ``build_from_keys_and_fp_rate``, ``__eq__`` and the attributes
``nb_bytes``, ``bits_size``, ``nb_hash_functions``, ``bits``.  Results are bit-identical to the
reference (tests/test_gpu_parity.py): MurmurHash3_x86_32 with seeds 0..k-1 over the key's
UTF-8 bytes, Python floor-mod of the signed hash by ``bits_size``.

The bitmap lives in HBM behind a ``pbf_filter_t`` handle (libpebblebloom.so, ctypes).  Per-key
``add()`` calls are buffered on the host and sent as one batch at the next read (probe,
serialisation, ``bits``), so an SSTableBuilder-style loop of ``add`` costs one kernel
pipeline, not one launch per key.  ``may_contain(key)`` — LsmStorage.get's per-key call — is
answered by the device's resident reader wave (the key posted into mapped pinned memory, no
launch per key; ``pbf_may_contain``, called through the ``_pebblefast`` C extension rather than
ctypes), or one launch where the resident reader does not apply.  ``lsm_get.candidates_one`` runs
a whole get's filter stage the same way.  Batch
entry points ``add_many`` / ``may_contain_many`` take ``list[str]``, ``PackedKeys`` or a
``KeyPacker`` directly.

Thread safety: the reference probes a filter from any reader thread without a lock
(lsm_storage.py:153-179).  Here builds, loads and batch probes hold the handle's lock
exclusively; one-key probes of a built filter hold it shared, so reader threads probe one filter
concurrently; the host-side ``add`` buffer has its own lock.
"""
from __future__ import annotations

import ctypes
import os
import struct
import threading
from math import ceil, log
from typing import Iterable, Optional

import numpy as np

from . import _native
from .keys import PackedKeys, PackedRecords

_PENDING_FLUSH = 1 << 16
_default_device = int(os.environ.get("PBF_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def set_default_device(device: int) -> None:
    global _default_device
    _default_device = int(device)


def _vp(a: np.ndarray | None):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


_FAST = None


def _fast():
    """csrc/fastcall.c (_pebblefast), bound to the loaded library's per-key entry points: the
    per-key calls go from a str to pbf_may_contain[_set] without ctypes."""
    global _FAST
    if _FAST is None:
        from . import _pebblefast
        L = _native.lib()
        _pebblefast.bind(ctypes.cast(L.pbf_may_contain, ctypes.c_void_p).value,
                         ctypes.cast(L.pbf_may_contain_set, ctypes.c_void_p).value)
        _FAST = _pebblefast
    return _FAST


class BloomFilter:
    """See module docstring; reference: src/bloom_filter.py:8."""

    def __init__(self, nb_bytes: int, nb_hash_functions: int, bits: Optional[int] = None,
                 device: Optional[int] = None):
        # bloom_filter.py:26-31
        self.nb_bytes = nb_bytes
        self.bits_size = 8 * nb_bytes
        self.nb_hash_functions = nb_hash_functions
        self.device = _default_device if device is None else int(device)
        self._pending: list[str] = []
        self._plock = threading.Lock()  # guards _pending (add / flush from several threads)
        self._h = None
        self._hv = 0  # the handle as an int
        self._fast = 0  # _hv while no add is buffered: the per-key calls' handle (_pebblefast)
        # the part of a `bits` int outside the bitmap (bits >= 8*nb_bytes, or a negative int's
        # sign extension): the reference keeps the whole int (bloom_filter.py:31) and compares it
        # in __eq__ (:36), while only the low 8*nb_bytes bits are ever read or serialised
        self._extra = 0
        if nb_bytes > 0:
            h = ctypes.c_void_p()
            _native.check(_native.lib().pbf_create(self.device, nb_bytes, nb_hash_functions, ctypes.byref(h)),
                          "pbf_create")
            self._h = h
            self._hv = self._fast = h.value
        if bits:
            self._upload_int(bits)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _native._lib is not None:
            _native._lib.pbf_destroy(h)
            self._h = None

    # ------------------------------------------------------------------ helpers
    def _require_modulus(self):
        """The reference computes `hash % bits_size` per hash function (bloom_filter.py:47)."""
        if self.nb_hash_functions <= 0:
            return False
        if self.nb_bytes == 0:
            raise ZeroDivisionError("integer modulo by zero")
        if self.nb_bytes < 0:
            raise ValueError("negative shift count")
        return True

    def _upload_int(self, bits: int) -> None:
        """The reference stores any int as ``bits`` and only ever reads its low 8*nb_bytes bits
        (``to_bytes`` bloom_filter.py:78 and ``_is_bit_set`` with indices < bits_size): those go to
        the device bitmap; the rest of the int (bits outside that range, a negative int's sign
        extension) is kept on the host for ``bits`` and ``__eq__``."""
        bits = int(bits)
        low = bits & ((1 << (8 * self.nb_bytes)) - 1) if self.nb_bytes > 0 else 0
        self._extra = bits - low
        if self.nb_bytes > 0:
            data = np.frombuffer(low.to_bytes(self.nb_bytes, "little"), dtype=np.uint8)
            _native.check(_native.lib().pbf_set_bitmap(self._h, _vp(data), self.nb_bytes), "pbf_set_bitmap")

    def _flush(self) -> None:
        if self._pending:
            with self._plock:
                pend, self._pending = self._pending, []
            if pend:
                self._add_packed(PackedKeys.from_strs(pend))
            with self._plock:
                if not self._pending:
                    self._fast = self._hv

    def _add_packed(self, pk: PackedKeys) -> None:
        if pk.n == 0 or not self._require_modulus():
            return
        L = _native.lib()
        if pk.key_len > 0:
            rc = L.pbf_add_fixed(self._h, _vp(pk.data), pk.key_len, pk.n, 0)
        else:
            rc = L.pbf_add(self._h, _vp(pk.data), _vp(pk.offsets), pk.n, 0)
        _native.check(rc, "pbf_add")

    def _probe_packed(self, pk: PackedKeys) -> np.ndarray:
        out = np.zeros((pk.n + 7) // 8, dtype=np.uint8)
        if pk.n == 0:
            return out
        if not self._require_modulus():  # k == 0: the AND over no bits is True
            out[:] = 0xFF
            if pk.n % 8:
                out[-1] = (1 << (pk.n % 8)) - 1
            return out
        self._flush()
        L = _native.lib()
        if pk.key_len > 0:
            rc = L.pbf_probe_fixed(self._h, _vp(pk.data), pk.key_len, pk.n, _vp(out), 0)
        else:
            rc = L.pbf_probe(self._h, _vp(pk.data), _vp(pk.offsets), pk.n, _vp(out), 0)
        _native.check(rc, "pbf_probe")
        return out

    def bitmap(self) -> bytes:
        """The nb_bytes-long little-endian bitmap (to_bytes() without the k byte)."""
        if self.nb_bytes <= 0:
            return b""
        self._flush()
        out = np.empty(self.nb_bytes, dtype=np.uint8)
        _native.check(_native.lib().pbf_get_bitmap(self._h, _vp(out), self.nb_bytes), "pbf_get_bitmap")
        return out.tobytes()

    # ------------------------------------------------------------------ reference surface
    @property
    def bits(self) -> int:
        """The filter as one Python int (bloom_filter.py:31), materialised on demand."""
        return int.from_bytes(self.bitmap(), "little") + self._extra

    @bits.setter
    def bits(self, value: int) -> None:
        with self._plock:
            self._pending = []
            self._fast = self._hv
        self._extra = 0
        if self.nb_bytes > 0:
            _native.check(_native.lib().pbf_clear(self._h), "pbf_clear")
        if value:
            self._upload_int(value)

    def __eq__(self, other):
        # bloom_filter.py:33-36 — compares bits and k only (not nb_bytes)
        if not isinstance(other, BloomFilter):
            return NotImplemented
        if self.nb_hash_functions != other.nb_hash_functions:
            return False
        if self._extra or other._extra:
            return self.bits == other.bits
        return self.bitmap().rstrip(b"\0") == other.bitmap().rstrip(b"\0")

    __hash__ = None

    def _hash(self, key: str) -> list[int]:
        """bloom_filter.py:38-49 — the k bit indices of `key`, computed on the GPU."""
        if not self._require_modulus():
            return []
        pk = PackedKeys.from_strs([key])
        k = self.nb_hash_functions
        out = np.zeros(k, dtype=np.uint64)
        L = _native.lib()
        if pk.key_len > 0:
            rc = L.pbf_hash_indices_fixed(self._h, _vp(pk.data), pk.key_len, 1, _vp(out), 0)
        else:
            rc = L.pbf_hash_indices(self._h, _vp(pk.data), _vp(pk.offsets), 1, _vp(out), 0)
        _native.check(rc, "pbf_hash_indices")
        return [int(x) for x in out]

    def add(self, key: str) -> None:
        """bloom_filter.py:60-65 (buffered; sent as one batch at the next read)."""
        if self.nb_hash_functions > 0:
            self._require_modulus()
        with self._plock:
            self._pending.append(key)
            self._fast = 0
            full = len(self._pending) >= _PENDING_FLUSH
        if full:
            self._flush()

    def may_contain(self, key: str) -> bool:
        """bloom_filter.py:67-74 for one key (pbf_may_contain: answered by the device's resident
        reader wave, or one launch), called from C (_pebblefast) with the str's UTF-8 bytes."""
        f = self._fast
        if not f and self._pending:
            self._flush()
            f = self._fast
        if f:
            r = (_FAST or _fast()).may_contain(f, key)
            if r is True or r is False:
                return r
            if r != -100:  # (-100: not a str; the reference's key.encode raises below)
                _native.check(r, "pbf_may_contain")
        enc = key.encode("utf-8")  # first, as bloom_filter.py:43 (AttributeError for a non-str)
        if not self._require_modulus():
            return True  # k == 0: the AND over no bits
        out = ctypes.c_int(0)
        rc = _native.lib().pbf_may_contain(self._h, enc, len(enc), ctypes.byref(out))
        if rc:
            _native.check(rc, "pbf_may_contain")
        return out.value != 0

    def to_bytes(self) -> bytes:
        """bloom_filter.py:76-81: little-endian bitmap + one byte of k (struct.error if k > 255)."""
        encoded_nb_hash_functions = struct.pack("B", self.nb_hash_functions)
        return self.bitmap() + encoded_nb_hash_functions

    @classmethod
    def from_bytes(cls, data, device: Optional[int] = None) -> "BloomFilter":
        """bloom_filter.py:83-90.  `data` may be bytes, bytearray or a memoryview slice of a
        file buffer (uploaded without an intermediate copy)."""
        nb_bytes = len(data) - 1
        nb_hash_functions = struct.unpack("B", bytes(data[nb_bytes:]))[0]
        bf = cls(nb_bytes=nb_bytes, nb_hash_functions=nb_hash_functions, device=device)
        if nb_bytes > 0:
            arr = np.frombuffer(data, dtype=np.uint8, count=nb_bytes)
            _native.check(_native.lib().pbf_set_bitmap(bf._h, _vp(arr), nb_bytes), "pbf_set_bitmap")
        return bf

    def replicate(self, device: Optional[int] = None, bounce: bool = False) -> "BloomFilter":
        """A copy of this filter on `device` (default: this filter's device): what
        ``from_bytes(self.to_bytes(), device)`` gives, device to device (pbf_copy_filter: peer
        copy over xGMI, or through pinned host memory with bounce=True).  The key-partitioned
        multi-GPU probe holds every SSTable's filter on every GPU this way: pebbledb builds a
        filter once per SSTable (src/sstable.py:274) and every get probes all of them
        (src/lsm_storage.py:164-179)."""
        dev = self.device if device is None else int(device)
        bf = object.__new__(type(self))
        bf.nb_bytes, bf.bits_size, bf.nb_hash_functions = self.nb_bytes, self.bits_size, self.nb_hash_functions
        bf.device = dev
        bf._pending = []
        bf._plock = threading.Lock()
        bf._h = None
        bf._hv = bf._fast = 0
        bf._extra = self._extra
        if self.nb_bytes > 0:
            self._flush()
            h = ctypes.c_void_p()
            _native.check(_native.lib().pbf_copy_filter(self._h, dev, _native.PBF_COPY_BOUNCE if bounce else 0,
                                                        ctypes.byref(h)), "pbf_copy_filter")
            bf._h = h
            bf._hv = bf._fast = h.value
        return bf

    @classmethod
    def from_device_bitmap(cls, ptr: int, nb_bytes: int, nb_hash_functions: int,
                           device: Optional[int] = None, stream: int = 0) -> "BloomFilter":
        """from_bytes() of a bitmap already in device memory on `device` (nb_bytes at `ptr`,
        e.g. a tensor an all-gather filled): no host copy.  `stream`: the producer's stream (its
        work is ordered before the load); the load is asynchronous on the filter's stream."""
        bf = cls(nb_bytes=nb_bytes, nb_hash_functions=nb_hash_functions, device=device)
        if nb_bytes > 0:
            bf.wait_stream(stream)
            _native.check(_native.lib().pbf_set_bitmap_device(bf._h, ctypes.c_void_p(ptr), nb_bytes),
                          "pbf_set_bitmap_device")
        return bf

    def bitmap_to_device(self, ptr: int) -> None:
        """to_bytes() without the k byte into device memory on this filter's device (nb_bytes at
        `ptr`); asynchronous on the filter's stream (sync() or signal_stream() before reading)."""
        if self.nb_bytes > 0:
            self._flush()
            _native.check(_native.lib().pbf_get_bitmap_device(self._h, ctypes.c_void_p(ptr), self.nb_bytes),
                          "pbf_get_bitmap_device")

    @classmethod
    def build_from_keys_and_fp_rate(cls, keys, fp_rate: float, device: Optional[int] = None) -> "BloomFilter":
        """bloom_filter.py:92-119 — same sizing expression order; one batched device build."""
        if isinstance(keys, PackedRecords):
            keys = keys.keys
        n = keys.n if isinstance(keys, PackedKeys) else len(keys)
        m = (-n * log(fp_rate)) / (log(2) ** 2)
        k = (m / n) * log(2)
        bloom_filter = cls(nb_bytes=ceil(m / 8), nb_hash_functions=round(k), device=device)
        bloom_filter.add_many(keys)
        return bloom_filter

    # ------------------------------------------------------------------ batch extensions
    def add_many(self, keys) -> None:
        """add() for every key of `keys` (list[str] / any iterable of str or records /
        PackedKeys / PackedRecords); iterables are packed as they are drained."""
        if isinstance(keys, PackedRecords):
            keys = keys.keys
        if isinstance(keys, PackedKeys):
            pk = keys
        elif isinstance(keys, list):
            pk = PackedKeys.from_strs(keys)
        else:
            pk = PackedKeys.from_iter(keys)
        self._add_packed(pk)

    def may_contain_many(self, keys, packed: bool = False) -> np.ndarray:
        """may_contain() for every key: bool array, or the LSB-first hit mask if packed=True."""
        pk = keys if isinstance(keys, PackedKeys) else PackedKeys.from_strs(list(keys))
        hm = self._probe_packed(pk)
        if packed:
            return hm
        return np.unpackbits(hm, bitorder="little")[:pk.n].astype(bool)

    # ------------------------------------------------------------------ device-resident batches
    # Pointers are device addresses on self.device (e.g. torch.Tensor.data_ptr()).  These calls
    # are asynchronous on the filter's stream: keep the buffers alive and call sync() (or wait
    # on an event recorded on `stream`) before reading results or freeing inputs.
    def clear(self) -> None:
        with self._plock:
            self._pending = []
            self._fast = self._hv
        if self._h is not None:
            _native.check(_native.lib().pbf_clear(self._h), "pbf_clear")

    def add_device_fixed(self, keys_ptr: int, key_len: int, n: int) -> None:
        if n and self._require_modulus():
            self._flush()
            _native.check(_native.lib().pbf_add_fixed(self._h, ctypes.c_void_p(keys_ptr), key_len, n, 1), "pbf_add_fixed")

    def add_device(self, keys_ptr: int, offsets_ptr: int, n: int) -> None:
        if n and self._require_modulus():
            self._flush()
            _native.check(_native.lib().pbf_add(self._h, ctypes.c_void_p(keys_ptr), ctypes.c_void_p(offsets_ptr), n, 1),
                          "pbf_add")

    def probe_device_fixed(self, keys_ptr: int, key_len: int, n: int, hitmask_ptr: int) -> None:
        if n:
            self._require_modulus()
            self._flush()
            _native.check(_native.lib().pbf_probe_fixed(self._h, ctypes.c_void_p(keys_ptr), key_len, n,
                                                        ctypes.c_void_p(hitmask_ptr), 1), "pbf_probe_fixed")

    def probe_device(self, keys_ptr: int, offsets_ptr: int, n: int, hitmask_ptr: int) -> None:
        if n:
            self._require_modulus()
            self._flush()
            _native.check(_native.lib().pbf_probe(self._h, ctypes.c_void_p(keys_ptr), ctypes.c_void_p(offsets_ptr), n,
                                                  ctypes.c_void_p(hitmask_ptr), 1), "pbf_probe")

    def sync(self) -> None:
        if self._h is not None:
            _native.check(_native.lib().pbf_sync(self._h), "pbf_sync")

    def wait_stream(self, stream: int) -> None:
        """Order this filter's next device work after everything queued on `stream` (an int
        hipStream_t, e.g. torch.cuda.current_stream().cuda_stream): a device key batch produced
        there needs no torch.cuda.synchronize() before add_device / probe_device."""
        if self._h is not None:
            _native.check(_native.lib().pbf_wait_stream(self._h, ctypes.c_void_p(stream or None)), "pbf_wait_stream")

    def signal_stream(self, stream: int) -> None:
        """Make `stream` wait for everything queued on this filter's stream (a consumer of a
        device hit mask or bitmap)."""
        if self._h is not None:
            _native.check(_native.lib().pbf_signal_stream(self._h, ctypes.c_void_p(stream or None)), "pbf_signal_stream")

    @property
    def stream(self) -> int:
        """The filter's hipStream_t as an int (torch.cuda.ExternalStream(stream))."""
        return 0 if self._h is None else int(_native.lib().pbf_stream(self._h) or 0)

    def popcount(self) -> int:
        if self.nb_bytes <= 0:
            return 0
        self._flush()
        out = ctypes.c_uint64()
        _native.check(_native.lib().pbf_popcount(self._h, ctypes.byref(out)), "pbf_popcount")
        return out.value

    def set_build_mode(self, mode: int) -> None:
        if self._h is not None:
            _native.check(_native.lib().pbf_set_build_mode(self._h, int(mode)), "pbf_set_build_mode")

    def set_probe_mode(self, mode: int) -> None:
        if self._h is not None:
            _native.check(_native.lib().pbf_set_probe_mode(self._h, int(mode)), "pbf_set_probe_mode")

    @property
    def last_probe_mode(self) -> int:
        return 0 if self._h is None else _native.lib().pbf_last_probe_mode(self._h)

    @property
    def last_probe_detail(self) -> int:
        """PBF_DETAIL_* flags of the last probe | (filters per fused gather << 8) | (tiled pipelines << 16)."""
        return 0 if self._h is None else int(_native.lib().pbf_last_probe_detail(self._h))

    @property
    def last_build_detail(self) -> int:
        """PBF_DETAIL_RING/SORT [| PBF_DETAIL_PACKED] | (keys per sub-chunk / 256) << 12."""
        return 0 if self._h is None else int(_native.lib().pbf_last_build_detail(self._h))

    @property
    def last_build_mode(self) -> int:
        return 0 if self._h is None else _native.lib().pbf_last_build_mode(self._h)

    @property
    def handle(self):
        return self._h

    def __repr__(self):
        return f"BloomFilter(nb_bytes={self.nb_bytes}, nb_hash_functions={self.nb_hash_functions}, device={self.device})"


def murmur3(key, seed: int = 0, device: Optional[int] = None) -> int:
    """mmh3.hash(key, seed) — MurmurHash3_x86_32 as the signed int32 bloom_filter.py:46 uses,
    computed on the device (pbf_murmur3_x86_32).  `key`: str (UTF-8 encoded) or bytes."""
    enc = key.encode("utf-8") if isinstance(key, str) else bytes(key)
    out = ctypes.c_int32(0)
    dev = _default_device if device is None else int(device)
    _native.check(_native.lib().pbf_murmur3_x86_32(dev, enc, len(enc), seed & 0xFFFFFFFF, ctypes.byref(out)),
                  "pbf_murmur3_x86_32")
    return out.value


# ---------------------------------------------------------------------- multi-filter probe
def _native_set(filters):
    """Split `filters` into the ones the native multi-probe takes (a device handle, k > 0) and
    the host-decided rest (k == 0: always True; nb_bytes == 0: ZeroDivisionError, as
    bloom_filter.py:47 raises)."""
    native = []
    for i, bf in enumerate(filters):
        if bf._require_modulus():
            bf._flush()
            native.append(i)
    return native


def may_contain_multi(filters, keys, groups=None) -> np.ndarray:
    """``may_contain`` of every key against every filter, the batched form of
    ``LsmStorage.get``'s filter checks (src/lsm_storage.py:164-175).  Returns a uint8 matrix
    [len(filters), ceil(n/8)] of LSB-first hit masks, row i = filters[i] (the get order).  Filters
    of one device that share (nb_bytes, k) are hashed and partitioned once (pbf_probe_multi);
    filters on several devices (or `groups`: a placement-group id per filter, filters of one group
    on one device) are probed by one host thread per group, each staging the batch to its own
    device (pbf_probe_multi_placed)."""
    filters = list(filters)
    pk = keys if isinstance(keys, PackedKeys) else PackedKeys.from_strs(list(keys))
    nbm = (pk.n + 7) // 8
    out = np.zeros((len(filters), nbm), dtype=np.uint8)
    if pk.n == 0 or not filters:
        return out
    native = _native_set(filters)
    for i in set(range(len(filters))) - set(native):
        out[i, :] = 0xFF
        if pk.n % 8:
            out[i, -1] = (1 << (pk.n % 8)) - 1
    if native:
        hs = (ctypes.c_void_p * len(native))(*[filters[i]._h.value for i in native])
        outs = (ctypes.c_void_p * len(native))(*[out[i].ctypes.data for i in native])
        L = _native.lib()
        if groups is not None:
            gs = np.ascontiguousarray([int(groups[i]) for i in native], dtype=np.uint32)
            rc = L.pbf_probe_multi_placed(hs, len(native), _vp(gs), _vp(pk.data),
                                          None if pk.key_len > 0 else _vp(pk.offsets), pk.key_len, pk.n, outs)
        elif pk.key_len > 0:
            rc = L.pbf_probe_multi_fixed(hs, len(native), _vp(pk.data), pk.key_len, pk.n, outs, 0)
        else:
            rc = L.pbf_probe_multi(hs, len(native), _vp(pk.data), _vp(pk.offsets), pk.n, outs, 0)
        _native.check(rc, "pbf_probe_multi")
    return out


def may_contain_set_bits(filters, key: str) -> int:
    """``may_contain_set`` as an int: bit i = ``filters[i].may_contain(key)``."""
    nf = len(filters)
    if not nf:
        return 0
    # the common shape (LsmStorage.get: built filters on one device, <= 64 of them): one C call
    # (_pebblefast), no ctypes or numpy; a buffered add (_fast == 0), a zero-size filter, filters
    # on several devices (PBF_ERR_INVALID) or a non-str key (-100) take the general path below
    if nf <= 64:
        hs = [bf._fast for bf in filters]
        if 0 not in hs:
            rc, bits = (_FAST or _fast()).may_contain_set(hs, key)
            if rc == 0:
                return bits
            if rc not in (-100, _native.PBF_ERR_INVALID):
                _native.check(rc, "pbf_may_contain_set")
    enc = key.encode("utf-8")
    native = _native_set(filters)
    bits = (1 << nf) - 1 - sum(1 << i for i in native)  # k == 0: the AND over no bits
    for dev in dict.fromkeys(filters[i].device for i in native):  # one call per device
        idx = [i for i in native if filters[i].device == dev]
        hs = (ctypes.c_void_p * len(idx))(*[filters[i]._h.value for i in idx])
        out = np.zeros((len(idx) + 7) // 8, dtype=np.uint8)
        _native.check(_native.lib().pbf_may_contain_set(hs, len(idx), enc, len(enc), _vp(out)),
                      "pbf_may_contain_set")
        got = np.unpackbits(out, bitorder="little")
        for j, i in enumerate(idx):
            bits |= int(got[j]) << i
    return bits


def may_contain_set(filters, key: str) -> list[bool]:
    """``filters[i].may_contain(key)`` for every filter, in ONE launch per k (pbf_may_contain_set):
    the per-key form of LsmStorage.get's bloom checks over its L0 and in-range level SSTables
    (src/lsm_storage.py:164-179).  Filters may have any sizes; filters on several devices take
    one launch per device."""
    filters = list(filters)
    bits = may_contain_set_bits(filters, key)
    return [(bits >> j) & 1 == 1 for j in range(len(filters))]


def probe_multi_device(filters, keys_ptr: int, n: int, hitmask_ptrs, key_len: int = 0, offsets_ptr: int = 0) -> None:
    """Device-resident multi-filter probe: keys (fixed key_len, or offsets) and the hit masks are
    device pointers on the filters' device; asynchronous on filters[0].stream (filters[0].sync())."""
    filters = list(filters)
    if n == 0 or not filters:
        return
    if len(hitmask_ptrs) != len(filters):
        raise ValueError("one hit mask per filter")
    for bf in filters:
        if not bf._require_modulus():
            raise ValueError("probe_multi_device: k == 0 filters are decided on the host (may_contain_multi)")
        bf._flush()
    hs = (ctypes.c_void_p * len(filters))(*[bf._h.value for bf in filters])
    outs = (ctypes.c_void_p * len(filters))(*[int(p) for p in hitmask_ptrs])
    L = _native.lib()
    if offsets_ptr:
        rc = L.pbf_probe_multi(hs, len(filters), ctypes.c_void_p(keys_ptr), ctypes.c_void_p(offsets_ptr), n, outs, 1)
    else:
        rc = L.pbf_probe_multi_fixed(hs, len(filters), ctypes.c_void_p(keys_ptr), key_len, n, outs, 1)
    _native.check(rc, "pbf_probe_multi")
