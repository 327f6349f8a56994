#!/bin/bash
# Round 6 session 19: the resident wave with and without its clock reads (request stats), C level.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for i in 1 2; do
  echo "== shipped $i"; timeout -k 10 120 tools/microbench/get_latency 20000 || exit 1
  echo "== noclock $i"; LD_LIBRARY_PATH=$PWD/build/variants/svc_noclock timeout -k 10 120 tools/microbench/get_latency 20000 || exit 1
done > gpurun_out/s19.log 2>&1
grep -E "==|170k|over  1|over 16 filters:" gpurun_out/s19.log
