#!/bin/bash
# Round 6 session 20: C5 with more partition workgroups per pipeline (PBF_PART_G): smaller
# per-workgroup key bitmaps let one pipeline hold more of the 100M-key batch, so the 8 bitmaps
# stream through the set tile test fewer times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for g in 256 512 768 1024; do
  PBF_PART_G=$g timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-host-c5 \
    > gpurun_out/s20_g$g.log 2>&1 || { tail -20 gpurun_out/s20_g$g.log; exit 1; }
  echo "G=$g $(grep -h '"metric"' gpurun_out/s20_g$g.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("check"), d.get("pipelines"))')"
done
