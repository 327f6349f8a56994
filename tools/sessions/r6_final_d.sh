#!/bin/bash
# Round 6 final records D (final sources): the driver's own C2 command (20 steps, 5 warmup) three
# times beside the default 100 / 20 run, one box, to size the short-warmup effect on its line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
    > gpurun_out/drv_$i.log 2>&1 || exit $?
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 100 --warmup 20 \
    > gpurun_out/def_$i.log 2>&1 || exit $?
done
grep -h '"metric"' gpurun_out/drv_*.log gpurun_out/def_*.log | cut -c1-330
