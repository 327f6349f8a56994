#!/bin/bash
# Round 6 session 12: a get's per-key time from C (tools/microbench/get_latency) vs Python.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 120 tools/microbench/get_latency 20000 > gpurun_out/s12_getlat.log 2>&1 || { cat gpurun_out/s12_getlat.log; exit 1; }
cat gpurun_out/s12_getlat.log
