#!/bin/bash
# Round 6 session 13: a get's filter stage in C (_pebblefast.candidates_one); the lsm_get and
# drop-in GPU tests, then the c1 legs twice and the C-level latencies.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsm_get.py tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/s13_pytest.log 2>&1 || { tail -30 gpurun_out/s13_pytest.log; exit 1; }
tail -2 gpurun_out/s13_pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config c1 > gpurun_out/s13_c1_$i.log 2>&1 || exit $?
  grep -h '"metric"' gpurun_out/s13_c1_$i.log | python3 -c 'import sys,json
d=json.loads(sys.stdin.read())["dropin_latency"]; print(d["pebbledb_amd"]["may_contain_us"], d["get_16_filters"]["one_call_us_per_get"], d["get_16_filters"]["one_launch_us_per_get"], d["get_16_filters"]["identical"], d.get("reader_threads"))'
done
timeout -k 10 120 tools/microbench/get_latency 20000 > gpurun_out/s13_getlat.log 2>&1 || exit $?
cat gpurun_out/s13_getlat.log
