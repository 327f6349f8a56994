#!/bin/bash
# Round 6 final records D2 (final sources): the driver's own C2 command twice, and the GPU suite
# once more on a fresh box (stability of the final sources).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_$i.log 2>&1 || exit $?
done
grep -h '"metric"' gpurun_out/drv_*.log | python3 -c 'import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d["steps"], d["warmup"], d["value"], d["ms_per_step"], d["build_ms"], d["probe_ms"], d["gpu_ms_per_step_by_quarter"])'
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest2.log 2>&1 || { tail -30 gpurun_out/pytest2.log; exit 1; }
tail -1 gpurun_out/pytest2.log
