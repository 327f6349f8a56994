"""CPU-side checks of the C-ABI library: it loads and exports every symbol the header declares.

No compute calls here (there is no GPU in the build container)."""
import ctypes
import os
import subprocess

import pytest

from pebbledb_amd import _native


def test_header_declares_expected_functions():
    names = _native.header_functions()
    assert "pbf_create" in names and "pbf_probe" in names and "pbf_add" in names
    assert set(names) == set(_native.SIGNATURES), set(names) ^ set(_native.SIGNATURES)


def test_library_loads_and_exports_every_header_symbol():
    L = _native.lib()
    for name in _native.header_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(_native.header_functions()) <= exported


def test_library_targets_gfx950_only():
    data = open(_native.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"gfx942" not in data and b"gfx90a" not in data


def test_version_and_error_string_without_gpu():
    L = _native.lib()
    assert L.pbf_version() >= 100
    assert isinstance(L.pbf_last_error(), bytes)
    # argument validation happens before any device call
    h = ctypes.c_void_p()
    assert L.pbf_create(0, 0, 3, ctypes.byref(h)) == _native.PBF_ERR_ZERO_SIZE
    assert b"modulo by zero" in L.pbf_last_error()
    assert L.pbf_sync(None) == _native.PBF_ERR_INVALID


def test_product_package_never_imports_the_oracle():
    pkg = os.path.dirname(_native.__file__)
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".h", ".cpp")):
                text = open(os.path.join(root, f)).read()
                assert "oracle" not in text.replace("oracle/", "").lower() or f == "__init__.py", f


def test_build_deps_cover_every_included_header():
    """build.DEPS (staleness check + source_digest) must list every file the library's sources
    include, so an edit to any kernel header rebuilds the .so and changes the digest that gates
    roofline.traffic (round-3 verdict: set_kernels.hpp was missing)."""
    import re
    from pebbledb_amd import build
    csrc = os.path.join(os.path.dirname(_native.__file__), "csrc")
    deps = {os.path.normpath(d) for d in build.DEPS}
    for f in os.listdir(csrc):
        if not f.endswith((".hip", ".hpp")):
            continue
        for line in open(os.path.join(csrc, f), encoding="utf-8"):
            m = re.match(r'\s*#\s*include\s*"([^"]+)"', line)
            if m:
                inc = os.path.normpath(os.path.join(csrc, m.group(1)))
                assert inc in deps, f"{f} includes {m.group(1)}, missing from build.DEPS"
    # every kernel header in csrc/ is reachable from the library source
    for f in os.listdir(csrc):
        if f.endswith(".hpp"):
            assert os.path.join(csrc, f) in deps, f


def test_placement_groups_of_a_multi_device_probe_without_gpu():
    """pbf_plan_groups is the placement step of pbf_probe_multi_placed (and of a host-batch
    pbf_probe_multi over filters on several devices, grouped by device): the 8-GPU shape — 16
    SSTable filters spread over devices 0..7 — gives 8 groups in first-appearance order, each
    host thread's group on its own device; a group naming two devices is refused."""
    import numpy as np
    L = _native.lib()

    def plan(groups, devices):
        g = np.ascontiguousarray(groups, dtype=np.uint32)
        d = np.ascontiguousarray(devices, dtype=np.int32)
        slot = np.zeros(len(g), dtype=np.uint32)
        ng = ctypes.c_uint32(0)
        rc = L.pbf_plan_groups(g.ctypes.data, d.ctypes.data, len(g), slot.ctypes.data, ctypes.byref(ng))
        return rc, slot.tolist(), ng.value

    devices = [f % 8 for f in range(16)][::-1]  # filters on devices 7..0, 7..0
    rc, slot, ng = plan(devices, devices)  # by device, as pbf_probe_multi groups them
    assert rc == 0 and ng == 8
    assert slot == [0, 1, 2, 3, 4, 5, 6, 7] * 2  # device 7 first (first appearance), then 6, ...
    rc, slot, ng = plan([5, 5, 9, 5], [2, 2, 2, 2])  # two groups on one device are allowed
    assert rc == 0 and ng == 2 and slot == [0, 0, 1, 0]
    rc, _, _ = plan([1, 1], [0, 3])
    assert rc == _native.PBF_ERR_INVALID and b"share a device" in L.pbf_last_error()
    assert plan([], []) [0] == 0


def test_library_digest_is_the_trees_and_a_stale_library_is_refused(monkeypatch):
    """The library carries the source_digest() it was compiled from (build_lib passes it in);
    build.up_to_date() compares that, not file times, and _native.lib() refuses a library whose
    digest is not the tree's, so a stale prebuilt .so can never be tested or benchmarked."""
    from pebbledb_amd import build
    assert build.embedded_digest(_native.LIB_PATH) == build.source_digest()
    assert build.up_to_date()
    L = _native.lib()
    assert L.pbf_source_digest().decode() == build.source_digest()
    monkeypatch.setattr(build, "source_digest", lambda: "0" * 64)
    monkeypatch.setattr(_native, "_lib", None)
    assert not build.up_to_date()
    with pytest.raises(_native.NativeError, match="stale"):
        _native.lib()
    monkeypatch.undo()
    assert _native.lib() is not None
