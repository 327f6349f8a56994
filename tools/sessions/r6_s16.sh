#!/bin/bash
# Round 6 session 16: which path a get's filter stage takes, and its cost by layer, beside the
# C-level latencies on the same box; the descriptor-index reuse test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
: timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread -k "descriptor or one_key or threads" \
  > gpurun_out/s16_pytest.log 2>&1 || { tail -40 gpurun_out/s16_pytest.log; exit 1; }
: tail
timeout -k 10 120 tools/microbench/get_latency 20000 > gpurun_out/s16_getlat.log 2>&1 || { cat gpurun_out/s16_getlat.log; exit 1; }
cat gpurun_out/s16_getlat.log
timeout -k 10 300 python3 tools/diag/get_stage_check.py > gpurun_out/s16.log 2>&1 || { cat gpurun_out/s16.log; exit 1; }
cat gpurun_out/s16.log
