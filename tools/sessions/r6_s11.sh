#!/bin/bash
# Round 6 session 11: per-key get path without repeated stream queries (pending cleared by a
# reader that found the stream drained) and without allocations; drop-in tests and the c1 legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
: timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/s11_pytest.log 2>&1 || { tail -30 gpurun_out/s11_pytest.log; exit 1; }
tail -2 gpurun_out/s11_pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config c1 > gpurun_out/s11_c1_$i.log 2>&1 || exit $?
  grep -h '"metric"' gpurun_out/s11_c1_$i.log | python3 -c 'import sys,json
d=json.loads(sys.stdin.read())["dropin_latency"]; print(d["pebbledb_amd"]["may_contain_us"], d["get_16_filters"], d.get("reader_threads"), d.get("batch_probe_with_gets"))'
done
