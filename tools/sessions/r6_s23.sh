#!/bin/bash
# Round 6 session 23: the RCCL branch at world 1 (tests/test_gpu_rccl.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 360 --timeout-method thread > gpurun_out/s23.log 2>&1 || { tail -60 gpurun_out/s23.log; exit 1; }
tail -3 gpurun_out/s23.log
