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


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build_lib(force: bool = False, verbose: bool = True, out: str = LIB, defines=()) -> str:
    """Compile libpebblebloom.so (or, for A/B measurements, a variant with extra -D defines
    into `out`; select it at run time with PBF_LIB)."""
    if not force and out == LIB and not defines and up_to_date():
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-result"] + [f"-D{d}" for d in defines] + ["-o", out + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


INGEST_SRC = os.path.join(CSRC, "ingest.c")


def ingest_path() -> str:
    import sysconfig
    return os.path.join(PKG, "_pebbleingest" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_ingest(force: bool = False, verbose: bool = True) -> str:
    """The host-side packed-ingestion extension (csrc/ingest.c, CPython C API, gcc)."""
    import sysconfig
    out = ingest_path()
    if not force and os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(INGEST_SRC):
        return out
    cmd = [os.environ.get("CC", "gcc"), "-O2", "-fPIC", "-shared", "-fopenmp", "-Wall", "-Wextra",
           "-Wno-missing-field-initializers", "-Wno-unused-parameter", "-I", sysconfig.get_paths()["include"],
           "-o", out + ".tmp", INGEST_SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    # python -m pebbledb_amd.build [--force] [--out PATH -DNAME ...]
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else LIB
    defs = [a[2:] for a in args if a.startswith("-D")]
    print(build_lib(force="--force" in args or out != LIB, out=out, defines=defs))
