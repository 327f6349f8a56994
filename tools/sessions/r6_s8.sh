#!/bin/bash
# Round 6, session 8 (diagnostic): which stream kind can host the persistent reader wave.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 120 tools/microbench/cumask_block > gpurun_out/cumask_block2.log 2>&1; rc=$?; cat gpurun_out/cumask_block2.log; exit $rc
