#!/bin/bash
# Round 6 final records E (final sources): the whole GPU suite with the RCCL one-rank test, and smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_e.log 2>&1 || { tail -20 gpurun_out/smoke_e.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_e.log 2>&1 || { tail -40 gpurun_out/pytest_e.log; exit 1; }
tail -1 gpurun_out/smoke_e.log; tail -1 gpurun_out/pytest_e.log
