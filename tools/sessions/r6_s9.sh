#!/bin/bash
# Round 6, session 9: the reader on a high-priority non-blocking stream, pool-backed scratch
# (no device-wide syncs), XCD-aware partitions while a reader is live: GPU suite, the per-key and
# concurrent-gets legs, the probe-with-gets diagnostic under rocprofv3 (exit with a live reader),
# the C2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_session.sh pytest bench_c1 || exit $?
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -n 3 gpurun_out/$name.log; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step gets_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gets_prof -o run -- python tools/diag/probe_with_gets.py
PBF_SPARE_CU=0 step gets_nospare 300 python tools/diag/probe_with_gets.py
python tools/prof_summary.py gpurun_out/gets_prof > gpurun_out/gets_prof_summary.txt
bash tools/gpu_session.sh bench
