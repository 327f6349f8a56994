#!/bin/bash
# Round 6 session 26: the churn test inside the drop-in suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s26.log 2>&1 || { tail -40 gpurun_out/s26.log; exit 1; }
tail -2 gpurun_out/s26.log
