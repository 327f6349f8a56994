"""HBM traffic per pass from rocprofv3 PMC passes (tools/gpu_session.sh step `traffic`).

    python tools/traffic_summary.py FETCH_DIR WRITE_DIR OUT.json [--config c2] [--probe-scale X]

FETCH_SIZE and WRITE_SIZE come from separate `--pmc` runs of the same short bench (one counter
group per run: FETCH_SIZE uses 3 of the 4 TCC slots, WRITE_SIZE 2).  Both are in KiB.  Per
MI355X_MICROARCH.md §HBM, on gfx950 FETCH_SIZE reports exactly half the bytes of a wide
(16 B/lane) streaming read, so fetched bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for
16-B-per-lane stores.

The factor is calibrated per access shape (tools/microbench/fetch_cal.hip, record
profiles/r05/ab/summary.md "FETCH_SIZE calibration"): a 1 GiB buffer read once with each load
shape the bloom kernels use — 16 B per lane non-temporal and temporal, 16 B per lane on every
other 64-B quad, 4 B per lane with 8 lanes per word, 4 B per lane contiguous — reported
FETCH_SIZE = 524,298-524,300 KiB each, i.e. a factor of 2.000 for every shape.  READ_FACTOR maps
each kernel to the shape of its HBM reads and that shape's measured factor.

Per kernel the median over dispatches of the full-size launches is taken; a pass's traffic is
the sum over its kernels.  A pass split into several pipelines (C3's probe: 200M keys in two
equal pipelines of 100M, each under the 2^30-position limit) is scaled from its full-size launch
by keys (--probe-scale = keys per pass / keys per full-size launch = 2.0 for C3).  bench.py reads OUT.json to
fill `roofline.traffic`.
"""
from __future__ import annotations

import collections
import csv
import json
import sys

# bytes / (FETCH_SIZE x 1024) measured per load shape (fetch_cal.hip, MI355X, round 5)
CALIBRATION = {
    "16B_lane_nt": 2.000,       # k_cal_read16
    "16B_lane": 2.000,          # k_cal_read16_t
    "16B_lane_half_lines": 2.000,  # k_cal_read16_q: the whole 128-B line is fetched
    "4B_lane_shared_word": 2.000,  # k_cal_read4_w
    "4B_lane": 2.000,           # k_cal_read4
}
# the shape of each kernel's dominant HBM reads
KERNEL_SHAPE = {
    "k_part_ring": "16B_lane_nt",      # 16-B key loads
    "k_part": "16B_lane_nt",
    "k_tile_build": "16B_lane_nt",     # region words, packed entries
    "k_ovf_build": "4B_lane",
    "k_tile_probe": "16B_lane_nt",     # region words (LDS-DMA or 16-B loads) + bitmap tile
    "k_tile_probe_set": "16B_lane",    # temporal: a set's workgroups share lines
    "k_gather_ring": "16B_lane_half_lines",  # failed quads' entries; result words 4 B / lane
    "k_gather": "16B_lane_half_lines",
    "k_hw_to_hitmask": "4B_lane",
}


def read_factor(kernel: str) -> tuple[str, float]:
    base = kernel.replace("pbf::", "").split("<")[0]
    shape = KERNEL_SHAPE.get(base, "16B_lane")
    return shape, CALIBRATION[shape]


PASSES = {
    "build": ("k_part_ring<", "false", "k_part<", "k_tile_build", "k_ovf_build"),
    "probe": ("k_part_ring<", "true", "k_part<", "k_tile_probe", "k_gather"),
}


def per_kernel(path: str, counter: str) -> dict[str, float]:
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{path}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        vals[name].append(float(r["Counter_Value"]))
    # full-size launches: the upper half of the dispatches by counter value
    out = {}
    for k, v in vals.items():
        v = sorted(v)
        out[k] = v[len(v) // 2] if len(v) < 3 else v[(3 * len(v)) // 4]
    return out


def pass_of(kernel: str) -> str | None:
    if not kernel.startswith("pbf::"):
        return None
    if kernel.startswith("pbf::k_part"):
        # k_part<KMAX, KM, PROBE> / k_part_ring<KMAX, KM, PROBE, POW2>
        args = kernel[kernel.index("<") + 1:].rstrip(">").split(",")
        return "probe" if args[2].strip() == "true" else "build"
    if kernel.split("<")[0] in ("pbf::k_tile_build", "pbf::k_ovf_build"):
        return "build"
    # templated kernels (k_gather_ring<NF>) match on the name before the argument list
    if kernel.split("<")[0] in ("pbf::k_tile_probe", "pbf::k_tile_probe_set", "pbf::k_gather", "pbf::k_gather_ring",
                                "pbf::k_hw_to_hitmask"):
        return "probe"
    return None


def main() -> None:
    fdir, wdir, out = sys.argv[1:4]
    config = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "c2"
    pscale = float(sys.argv[sys.argv.index("--probe-scale") + 1]) if "--probe-scale" in sys.argv else 1.0
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    res = {"config": config, "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE ({fdir}, {wdir})",
           "correction": "read bytes = factor(shape) x FETCH_SIZE x 1024 (gfx950 read halving, calibrated per load "
                         "shape), write bytes = WRITE_SIZE x 1024",
           "calibration": {"record": "profiles/r05/ab/summary.md (FETCH_SIZE calibration; tools/microbench/fetch_cal.hip)",
                           "factors": CALIBRATION},
           "kernels": {}, "passes": {}}
    for k in sorted(set(fetch) | set(write)):
        p = pass_of(k)
        if p is None:
            continue
        shape, factor = read_factor(k)
        rd = factor * fetch.get(k, 0.0) * 1024
        wr = write.get(k, 0.0) * 1024
        res["kernels"][k] = {"pass": p, "read_bytes": rd, "write_bytes": wr, "read_shape": shape, "read_factor": factor}
        agg = res["passes"].setdefault(p, {"read_bytes": 0.0, "write_bytes": 0.0})
        agg["read_bytes"] += rd
        agg["write_bytes"] += wr
    if pscale != 1.0 and "probe" in res["passes"]:
        res["probe_scale"] = pscale
        for key in ("read_bytes", "write_bytes"):
            res["passes"]["probe"][key] *= pscale
    for p in res["passes"].values():
        p["traffic_bytes"] = p["read_bytes"] + p["write_bytes"]
    # the kernels these counters were taken on (bench.py only uses a summary of its own sources)
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from pebbledb_amd.build import source_digest
    res["source_sha256"] = source_digest()
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(f"{k:45s} {v['pass']:6s} read {v['read_bytes'] / 1e6:9.1f} MB  write {v['write_bytes'] / 1e6:9.1f} MB")
    for p, v in res["passes"].items():
        print(f"pass {p}: {v['traffic_bytes'] / 1e6:.1f} MB")


if __name__ == "__main__":
    main()
