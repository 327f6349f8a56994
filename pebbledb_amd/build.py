"""Build libpebblebloom.so in-tree (hipcc, gfx950) — called by __graft_entry__.build()."""
from __future__ import annotations

import os
import re
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libpebblebloom.so")
SOURCES = [os.path.join(CSRC, "pebblebloom.hip")]


def _local_includes(path: str, seen: set) -> None:
    """Every file a source pulls in by `#include "..."` (transitively), so an edit to any of them
    marks the library stale and changes source_digest()."""
    path = os.path.normpath(path)
    if path in seen:
        return
    seen.add(path)
    with open(path, encoding="utf-8") as fh:
        for line in fh:
            m = re.match(r'\s*#\s*include\s*"([^"]+)"', line)
            if m:
                _local_includes(os.path.join(os.path.dirname(path), m.group(1)), seen)


def _deps() -> list:
    seen: set = set()
    for src in SOURCES:
        _local_includes(src, seen)
    return sorted(seen)


DEPS = _deps()
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PBF_OFFLOAD_ARCH", "gfx950")


def source_digest() -> str:
    """sha256 over the library's sources and compile flags: identifies the kernels a measurement
    (e.g. the committed PMC traffic summary) was taken on, independent of rebuilds."""
    import hashlib
    h = hashlib.sha256()
    for d in sorted(DEPS):
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as fh:
            h.update(fh.read())
    h.update(ARCH.encode())
    return h.hexdigest()


DIGEST_MARKER = b"pbf-source-digest:"


def embedded_digest(path: str = LIB) -> str | None:
    """The source_digest() a library was compiled from (build_lib passes it as PBF_SOURCE_DIGEST
    and the library keeps it behind DIGEST_MARKER), read from the file without loading it; None
    for a library built without one."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as fh:
        data = fh.read()
    i = data.find(DIGEST_MARKER)
    if i < 0:
        return None
    d = data[i + len(DIGEST_MARKER):i + len(DIGEST_MARKER) + 64]
    return d.decode("ascii", "replace") if len(d) == 64 else None


def up_to_date() -> bool:
    """The library exists and was compiled from the sources in the tree (its embedded digest,
    not file times: a prebuilt .so travels to the GPU box with the tree)."""
    return embedded_digest(LIB) == source_digest()


def build_lib(force: bool = False, verbose: bool = True, out: str = LIB, defines=()) -> str:
    """Compile libpebblebloom.so (or, for A/B measurements, a variant with extra -D defines
    into `out`; select it at run time with PBF_LIB)."""
    if not force and out == LIB and not defines and up_to_date():
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-result", f'-DPBF_SOURCE_DIGEST="{source_digest()}"'] + \
        [f"-D{d}" for d in defines] + ["-o", out + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


INGEST_SRC = os.path.join(CSRC, "ingest.c")


def ingest_path() -> str:
    import sysconfig
    return os.path.join(PKG, "_pebbleingest" + sysconfig.get_config_var("EXT_SUFFIX"))


def _build_ext(src: str, out: str, force: bool, verbose: bool, openmp: bool) -> str:
    import sysconfig
    if not force and os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
        return out
    cmd = [os.environ.get("CC", "gcc"), "-O2", "-fPIC", "-shared"] + (["-fopenmp"] if openmp else []) + \
        ["-Wall", "-Wextra", "-Wno-missing-field-initializers", "-Wno-unused-parameter", "-Wno-cast-function-type",
         "-I", sysconfig.get_paths()["include"], "-o", out + ".tmp", src]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_ingest(force: bool = False, verbose: bool = True) -> str:
    """The host-side packed-ingestion extension (csrc/ingest.c, CPython C API, gcc)."""
    return _build_ext(INGEST_SRC, ingest_path(), force, verbose, openmp=True)


FAST_SRC = os.path.join(CSRC, "fastcall.c")


def fast_path() -> str:
    import sysconfig
    return os.path.join(PKG, "_pebblefast" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_fast(force: bool = False, verbose: bool = True) -> str:
    """The per-key call extension (csrc/fastcall.c: may_contain / may_contain_set without
    ctypes, CPython C API, gcc)."""
    return _build_ext(FAST_SRC, fast_path(), force, verbose, openmp=False)


if __name__ == "__main__":
    # python -m pebbledb_amd.build [--force] [--out PATH -DNAME ...]
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else LIB
    defs = [a[2:] for a in args if a.startswith("-D")]
    print(build_lib(force="--force" in args or out != LIB, out=out, defines=defs))
