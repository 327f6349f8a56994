"""Issue-rate accounting of the C2 kernels from PMC counter passes (tools/pmc_passes.sh).

    python tools/issue_summary.py PMC_SUMMARY.txt KERNEL_STATS.csv

PMC_SUMMARY.txt is tools/pmc_summary.py's output (per kernel, mean counter values over
dispatches, summed over the 8 XCDs as rocprofv3 reports them); KERNEL_STATS.csv the rocprofv3
--stats table of the same sources (average duration per kernel).  Per kernel:
  clock      GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md, DVFS give-back)
  VALU       SQ_INSTS_VALU x 4 cycles / (duration x clock x 1024 SIMDs).  4 cycles per wave64
             32-bit integer op is measured, not the 2 of MI355X_MICROARCH.md's SIMD-32 (an FP32
             figure): the partition's hash alone (tools/microbench ring_time_hashonly: no appends,
             no barriers, no key loads) runs at ~4.3 SIMD cycles per VALU instruction
  SALU       SQ_INSTS_SALU / (duration x clock x 256 CUs), one scalar issue per CU per cycle
  LDS        SQ_INSTS_LDS (wave instructions) and the share of LDS-active cycles spent in bank
             conflicts (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE)
32-bit integer multiplies and the 64-bit ops take longer than 4 cycles, so VALU is a lower bound
of the VALU pipe's busy share.
"""
import csv
import sys

pmc, stats = sys.argv[1], sys.argv[2]
cnt, cur = {}, None
for line in open(pmc):
    if line.startswith("pbf"):
        cur = line.strip()
        cnt[cur] = {}
    elif cur and line.strip():
        k, v = line.split()
        cnt[cur][k] = float(v)
dur = {}
for r in csv.DictReader(open(stats)):
    name = r["Name"].split("(")[0].replace("void ", "").strip()
    dur[name] = float(r["AverageNs"]) * 1e-9
print(f"{'kernel':36s} {'us':>7s} {'GHz':>5s} {'VALU instr':>11s} {'VALU':>6s} {'SALU':>6s} {'LDS instr':>10s} {'LDS conflict':>12s}")
for k, c in sorted(cnt.items()):
    d = next((v for n, v in dur.items() if n.startswith(k)), None)
    if not d or "GRBM_GUI_ACTIVE" not in c:
        continue
    clk = c["GRBM_GUI_ACTIVE"] / 8 / d
    valu = c.get("SQ_INSTS_VALU", 0) * 4 / (d * clk * 1024)
    salu = c.get("SQ_INSTS_SALU", 0) / (d * clk * 256)
    lc = c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0))
    print(f"{k[:36]:36s} {d * 1e6:7.1f} {clk / 1e9:5.2f} {c.get('SQ_INSTS_VALU', 0):11.3g} {valu:6.1%} {salu:6.1%} "
          f"{c.get('SQ_INSTS_LDS', 0):10.3g} {lc:12.1%}")
