#!/bin/bash
# Round 6 session 21: C5 kernel times at PBF_PART_G=256 (3 pipelines) and 768 (1 pipeline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in 256 768; do
  PBF_PART_G=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s21_g$g -o run -- \
    python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-host-c5 --no-compare > gpurun_out/s21_g$g.log 2>&1 || { tail -20 gpurun_out/s21_g$g.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/s21_g$g > gpurun_out/s21_g${g}_summary.txt 2>&1 || true
  head -12 gpurun_out/s21_g${g}_summary.txt
done
