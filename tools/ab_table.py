"""Summarise A/B bench logs under gpurun_out/ (one JSON line per log): build / probe / step."""
import glob, json, sys

pat = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab*.log"
for p in sorted(glob.glob(pat)):
    for line in open(p, errors="replace"):
        if line.startswith("{"):
            d = json.loads(line)
            print(f"{p.split('/')[-1]:32s} value {d['value']:10.1f}  ms/step {d['ms_per_step']:.4f}  "
                  f"build {d.get('build_ms', 0):.4f}  probe {d.get('probe_ms', 0):.4f}")
