#!/bin/bash
# One GPU-box session: each GPU step under its own time limit; stop at the first fault /
# abort / timeout (exit codes other than 0 and 1).  Usage: tools/gpu_session.sh STEP...
# Steps: smoke, pytest, bench, prof, pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest 1200 python -m pytest tests -m gpu -q -rf ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5 ;;
    bench_atomic) run bench_atomic 600 python bench.py --steps 10 --warmup 3 --build-mode 1 --no-cpu-baseline ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
