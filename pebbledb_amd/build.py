"""Build libpebblebloom.so in-tree (hipcc, gfx950) — called by __graft_entry__.build()."""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libpebblebloom.so")
SOURCES = [os.path.join(CSRC, "pebblebloom.hip")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("bloom_kernels.hpp", "murmur_device.hpp", "tiled_kernels.hpp", "ring_kernels.hpp")] + [
    os.path.join(REPO, "include", "pebblebloom.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PBF_OFFLOAD_ARCH", "gfx950")


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build_lib(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-result", "-o", LIB + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build_lib(force="--force" in sys.argv)
    print(LIB)
