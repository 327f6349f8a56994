#!/bin/bash
# Round 6 session 14: per-key latency by filter size and k, from C.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 120 tools/microbench/get_latency 20000 > gpurun_out/s14_getlat.log 2>&1 || { cat gpurun_out/s14_getlat.log; exit 1; }
cat gpurun_out/s14_getlat.log
