#!/bin/bash
# Round 6 session 25: the resident reader under filter churn (tools/diag/reader_churn.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/diag/reader_churn.py 20 8 > gpurun_out/s25.log 2>&1 || { tail -20 gpurun_out/s25.log; exit 1; }
timeout -k 10 120 python3 -u tools/diag/reader_churn.py 20 32 >> gpurun_out/s25.log 2>&1 || { tail -20 gpurun_out/s25.log; exit 1; }
cat gpurun_out/s25.log
