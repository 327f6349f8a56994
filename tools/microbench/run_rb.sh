#!/bin/bash
# Run the ring_bench variant binaries (tools/microbench/rb_*) one after another on the GPU box.
# Usage: tools/microbench/run_rb.sh [names...]   (output: gpurun_out/rb.txt)
cd "$(dirname "$0")"
mkdir -p ../../gpurun_out
names=${*:-$(ls rb_* | grep -v '\.')}
for b in $names; do
  echo "== $b" | tee -a ../../gpurun_out/rb.txt
  timeout -k 5 90 ./$b 20 >> ../../gpurun_out/rb.txt 2>&1 || { echo "$b failed rc=$?" | tee -a ../../gpurun_out/rb.txt; exit 1; }
done
cat ../../gpurun_out/rb.txt
