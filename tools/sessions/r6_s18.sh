#!/bin/bash
# Round 6 session 18: where the resident wave's 1.3 us per request goes: the ack's tick word
# reports the time to (1) the descriptors, (2) the hashes, (3) the bitmap tests, (0) the answer.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in svc_t1 svc_t2 svc_t3; do
  echo "== $v"; LD_LIBRARY_PATH=$PWD/build/variants/$v timeout -k 10 120 tools/microbench/get_latency 20000 || exit 1
done > gpurun_out/s18.log 2>&1
echo "== shipped" >> gpurun_out/s18.log
timeout -k 10 120 tools/microbench/get_latency 20000 >> gpurun_out/s18.log 2>&1 || exit 1
grep -E "==|over  1|over 16 filters:|resident" gpurun_out/s18.log
