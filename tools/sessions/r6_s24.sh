#!/bin/bash
# Round 6 session 24: do a build pass and a probe pass on different streams overlap?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/diag/overlap_check.py > gpurun_out/s24.log 2>&1 || { cat gpurun_out/s24.log; exit 1; }
cat gpurun_out/s24.log
