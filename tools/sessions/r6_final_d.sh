#!/bin/bash
# Round 6 final records D (final sources): the driver's own C2 command (20 steps, 5 warmup) beside
# the default 100 / 20 run and a cold 200-step run, one box, to size the short-run effect on its
# line (gpu_ms_per_step_by_quarter: a step's GPU time over each quarter of the timed steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_$i.log 2>&1 || exit $?
done
timeout -k 10 240 python3 bench.py --gpus 1 --steps 100 --warmup 20 > gpurun_out/def_1.log 2>&1 || exit $?
timeout -k 10 240 python3 bench.py --gpus 1 --steps 200 --warmup 0 --no-cpu-baseline --no-host-inclusive \
  > gpurun_out/cold_1.log 2>&1 || exit $?
timeout -k 10 240 python3 bench.py --gpus 1 --steps 400 --warmup 0 --no-cpu-baseline --no-host-inclusive \
  > gpurun_out/cold_2.log 2>&1 || exit $?
grep -h '"metric"' gpurun_out/drv_*.log gpurun_out/def_*.log gpurun_out/cold_*.log \
  | python3 -c 'import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d["steps"], d["warmup"], d["ms_per_step"], d["build_ms"], d["probe_ms"], d["gpu_ms_per_step_by_quarter"])'
