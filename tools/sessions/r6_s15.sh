#!/bin/bash
# Round 6 session 15: the resident reader with descriptor indexes (LDS-cached), (filter, seed)
# pairs over the lanes and single-round-trip polls: the whole GPU suite, the C-level latencies
# and the c1 legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 120 tools/microbench/get_latency 20000 > gpurun_out/s15_getlat.log 2>&1 || { cat gpurun_out/s15_getlat.log; exit 1; }
cat gpurun_out/s15_getlat.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/s15_pytest.log 2>&1 || { tail -40 gpurun_out/s15_pytest.log; exit 1; }
tail -2 gpurun_out/s15_pytest.log
timeout -k 10 300 python3 bench.py --config c1 > gpurun_out/s15_c1.log 2>&1 || exit $?
grep -h '"metric"' gpurun_out/s15_c1.log | python3 -c 'import sys,json
d=json.loads(sys.stdin.read())["dropin_latency"]; print(d["pebbledb_amd"]["may_contain_us"], d["pebbledb_amd"]["may_contain_launch_us"], d["identical"], d["get_16_filters"], d.get("reader_threads"), d.get("batch_probe_with_gets"))'
