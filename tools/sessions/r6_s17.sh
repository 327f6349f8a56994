#!/bin/bash
# Round 6 session 17: resident reader bitmap loads, device-scope atomic (shipped) vs plain
# L2-cacheable (variant), C-level latencies alternated on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for i in 1 2; do
  echo "== shipped $i"; timeout -k 10 120 tools/microbench/get_latency 20000 || exit 1
  echo "== plain $i"; LD_LIBRARY_PATH=$PWD/build/variants/svc_plain timeout -k 10 120 tools/microbench/get_latency 20000 || exit 1
done > gpurun_out/s17.log 2>&1
cat gpurun_out/s17.log
