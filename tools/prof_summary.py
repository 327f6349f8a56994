"""Print the rocprofv3 --kernel-trace --stats summary (kernel_stats.csv) found under a directory.

Usage: python tools/prof_summary.py gpurun_out/prof
"""
import csv
import glob
import sys


def main(root):
    files = sorted(glob.glob(f"{root}/**/*kernel_stats.csv", recursive=True))
    if not files:
        print(f"no kernel_stats.csv under {root}")
        return 1
    for f in files:
        print(f"# {f}")
        rows = list(csv.DictReader(open(f)))
        print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} {'pct':>6s}")
        for r in rows:
            name = r["Name"].split("(")[0].replace("void ", "")
            print(f"{name[:60]:60s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:10.2f} "
                  f"{float(r['MinNs']) / 1e3:10.2f} {float(r['MaxNs']) / 1e3:10.2f} {float(r['Percentage']):6.2f}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"))
