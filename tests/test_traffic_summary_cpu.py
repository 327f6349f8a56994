"""tools/traffic_summary.py assigns every kernel of the tiled build/probe passes to its pass, so
bench.py's roofline.traffic sums the whole pass (a templated name such as k_gather_ring<1> was
once dropped silently)."""
import csv
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

from traffic_summary import pass_of  # noqa: E402

# kernels that belong to no timed pass of the C2 step (key generation, direct paths, encoder)
NOT_IN_A_PASS = ("k_gen_", "k_popcount", "k_probe", "k_build_atomic", "k_encode_blocks", "k_hash")


def test_pass_of_names():
    assert pass_of("pbf::k_part_ring<8, 0, true, true>") == "probe"
    assert pass_of("pbf::k_part_ring<8, 0, false, true>") == "build"
    assert pass_of("pbf::k_part<8, 1, true>") == "probe"
    assert pass_of("pbf::k_tile_build") == "build"
    assert pass_of("pbf::k_ovf_build") == "build"
    assert pass_of("pbf::k_tile_probe") == "probe"
    assert pass_of("pbf::k_tile_probe_set<2>") == "probe"
    assert pass_of("pbf::k_gather_ring<1>") == "probe"
    assert pass_of("pbf::k_gather_ring<8>") == "probe"
    assert pass_of("pbf::k_hw_to_hitmask") == "probe"
    assert pass_of("__amd_rocclr_copyBuffer") is None


def test_every_profiled_pass_kernel_is_assigned():
    path = os.path.join(REPO, "profiles", "r01", "s12", "kernel_stats.csv")
    names = [r["Name"].split("(")[0].replace("void ", "").strip() for r in csv.DictReader(open(path))]
    pbf = [n for n in names if n.startswith("pbf::")]
    assert pbf
    for n in pbf:
        if any(n.split("::")[1].startswith(p) for p in NOT_IN_A_PASS):
            continue
        assert pass_of(n) in ("build", "probe"), n


def test_committed_traffic_matches_the_sources():
    """bench.py fills roofline.traffic only from a PMC summary taken on the current kernel sources
    (source digest); every committed config summary must be one (a kernel edit without new PMC
    passes would leave the driver's bench line with traffic null)."""
    import json

    from pebbledb_amd.build import source_digest
    for cfg in ("c2", "c3", "c4", "c5"):
        t = json.load(open(os.path.join(REPO, "profiles", f"traffic_{cfg}.json")))
        assert t["source_sha256"] == source_digest(), cfg
        assert t["passes"]["build"]["traffic_bytes"] > 0 and t["passes"]["probe"]["traffic_bytes"] > 0
    assert pass_of("pbf::k_tile_build<true>") == "build"


def test_every_pass_kernel_has_a_calibrated_read_shape():
    """Each kernel of a timed pass is mapped to the load shape its FETCH_SIZE factor was
    calibrated on (fetch_cal.hip, profiles/r05/ab/summary.md), not a default."""
    from traffic_summary import CALIBRATION, KERNEL_SHAPE, read_factor
    for name in ("pbf::k_part_ring<6, 0, true, true, true>", "pbf::k_part<8, 2, true>", "pbf::k_tile_build<true>",
                 "pbf::k_ovf_build", "pbf::k_tile_probe<2>", "pbf::k_tile_probe_set<2>", "pbf::k_gather_ring<1>",
                 "pbf::k_gather_ring<8>", "pbf::k_hw_to_hitmask"):
        base = name.replace("pbf::", "").split("<")[0]
        assert base in KERNEL_SHAPE, name
        shape, factor = read_factor(name)
        assert shape in CALIBRATION and factor == CALIBRATION[shape]
    assert all(abs(f - 2.0) < 0.01 for f in CALIBRATION.values())
