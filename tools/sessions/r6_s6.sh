#!/bin/bash
# Round 6, session 6 (diagnostic): a batched probe beside per-key gets, kernel traces with the
# XCD-aware planning on (default while a reader is live) and forced off, and the C2 step with the
# planning forced on and no reader.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
set -o pipefail
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -n 3 gpurun_out/$name.log; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step gets_spare 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gets_spare -o run -- python tools/diag/probe_with_gets.py
PBF_SPARE_CU=0 step gets_nospare 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gets_nospare -o run -- python tools/diag/probe_with_gets.py
PBF_SPARE_CU=1 step c2_spare 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive
python tools/prof_summary.py gpurun_out/gets_spare > gpurun_out/gets_spare_summary.txt
python tools/prof_summary.py gpurun_out/gets_nospare > gpurun_out/gets_nospare_summary.txt
