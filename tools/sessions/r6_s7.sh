#!/bin/bash
# Round 6, session 7 (diagnostic): does null-stream work / a device sync / hipFree wait for a
# kernel on a CU-masked stream (the resident reader's); the C2 step with the XCD-aware partition
# planning forced on (no reader).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -n 8 gpurun_out/$name.log; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step cumask_block 120 tools/microbench/cumask_block
PBF_SPARE_CU=1 step c2_spare 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive
PBF_SPARE_CU=0 step c2_nospare 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive
