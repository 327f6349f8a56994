#!/bin/bash
# Round 6 session 22: C2 build pass with the ring partition (shipped) vs the counting sort with
# packed entries (PBF_PART=sort_build, PK3 for k = 6), alternated on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for i in 1 2; do
  for v in ring sort_build; do
    if [ $v = ring ]; then unset PBF_PART; else export PBF_PART=sort_build; fi
    timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-inclusive > gpurun_out/s22_${v}_$i.log 2>&1 || exit $?
    echo "$v $i $(grep -h '"metric"' gpurun_out/s22_${v}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["build_ms"], d["probe_ms"], d["build_mode"], d["check"]["members_all_hit"])')"
  done
done
unset PBF_PART
PBF_PART=sort_build timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s22_prof_sort -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive > gpurun_out/s22_prof.log 2>&1 || exit $?
python3 tools/prof_summary.py gpurun_out/s22_prof_sort | head -10
