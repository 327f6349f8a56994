#!/bin/bash
# Round 6 session 27: C5 in one pipeline (multi-filter probes plan 2-4 rounds of partition
# workgroups while the gather does not fit; the tile test's table in region chunks): parity of
# the multi-filter and tile-test suites, C5 A/B against PBF_PART_G=256 (the previous plan), profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/s27_pytest.log 2>&1 || { tail -40 gpurun_out/s27_pytest.log; exit 1; }
tail -1 gpurun_out/s27_pytest.log
for i in 1 2; do
  for v in auto g256; do
    if [ $v = auto ]; then unset PBF_PART_G; else export PBF_PART_G=256; fi
    timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-host-c5 > gpurun_out/s27_${v}_$i.log 2>&1 || { tail -20 gpurun_out/s27_${v}_$i.log; exit 1; }
    echo "$v $i $(grep -h '"metric"' gpurun_out/s27_${v}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["check"])')"
  done
done
unset PBF_PART_G
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s27_prof -o run -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-host-c5 --no-compare > gpurun_out/s27_prof.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/s27_prof > gpurun_out/s27_prof_summary.txt 2>&1
head -10 gpurun_out/s27_prof_summary.txt
