#!/bin/bash
# One GPU-box session: each GPU step under its own time limit; stop at the first fault /
# abort / timeout (exit codes other than 0 and 1).  Usage: tools/gpu_session.sh STEP...
#   smoke pytest bench benchq prof profq traffic pmcall others bench_c1 bench_c3 bench_c4
#   bench_c5 bench_c5mixed bench_sst prof_c3 prof_c4 prof_c5 traffic_c3 pmc_c3 pmc_c4 ab ab_c3 ab_c4
#   ab_c5 ab_c5mixed abenv abenv_c5 selflaunch final
# A/B steps run the default library and every build/variants/*.so (PBF_LIB), alternating, with
# PBF_AB_ARGS appended to the bench command line.
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
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
prof() {  # name seconds bench-args...
  local name=$1 secs=$2; shift 2
  run $name $secs rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$name -o run -- python bench.py "$@"
  python tools/prof_summary.py gpurun_out/$name > gpurun_out/${name}_summary.txt 2>&1 || true
}
traffic() {  # tag bench-args...: FETCH_SIZE and WRITE_SIZE in separate passes, summed per pass
  local tag=$1; shift
  run pmc_fetch_$tag 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$tag -o run -- python bench.py --no-cpu-baseline --no-host-inclusive "$@"
  run pmc_write_$tag 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$tag -o run -- python bench.py --no-cpu-baseline --no-host-inclusive "$@"
  python tools/traffic_summary.py gpurun_out/pmc_fetch_$tag gpurun_out/pmc_write_$tag gpurun_out/traffic_$tag.json --config $tag ${TRAFFIC_ARGS:-} > gpurun_out/traffic_${tag}_summary.txt 2>&1 || true
}
abenv() {  # tag seconds rounds bench-args...: the default vs the environment in PBF_AB_ENV (VAR=value)
  local tag=$1 secs=$2 rounds=$3; shift 3
  for r in $(seq 1 $rounds); do
    run ${tag}_default_$r $secs python bench.py --no-cpu-baseline --no-host-inclusive "$@"
    run ${tag}_env_$r $secs env $PBF_AB_ENV python bench.py --no-cpu-baseline --no-host-inclusive "$@"
  done
}
ab() {  # tag seconds rounds bench-args...
  local tag=$1 secs=$2 rounds=$3; shift 3
  for r in $(seq 1 $rounds); do
    run ${tag}_default_$r $secs python bench.py --no-cpu-baseline --no-host-inclusive "$@" ${PBF_AB_ARGS:-}
    for v in build/variants/*.so; do
      [ -e "$v" ] || continue
      nm=$(basename $v .so)
      PBF_LIB=$PWD/$v run ${tag}_${nm}_$r $secs python bench.py --no-cpu-baseline --no-host-inclusive "$@" ${PBF_AB_ARGS:-}
    done
  done
}
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 150 --timeout-method thread ;;
    pytest_new) run pytest_new 600 python -u -m pytest ${PBF_TESTS:-tests/test_gpu_multi.py} -m gpu -x -v -rf --timeout 150 --timeout-method thread ;;
    bench) run bench 600 python bench.py ;;
    benchq) for r in 1 2; do run benchq_$r 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-host-inclusive; done ;;
    prof) prof prof 600 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive ;;
    profq) prof profq 300 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive ;;
    traffic) traffic c2 --steps 5 --warmup 2 ;;
    traffic_c3) TRAFFIC_ARGS="--probe-scale 2.0" traffic c3 --config c3 --steps 2 --warmup 1 ;;  # two equal 100M-key pipelines per probe pass
    traffic_c4) traffic c4 --config c4 --steps 2 --warmup 1 ;;  # per-filter build pass (bench scales by the rank's filters)
    traffic_c5) TRAFFIC_ARGS="--probe-scale 1.0" traffic c5 --config c5 --steps 2 --warmup 1 --no-host-c5 --no-compare ;;  # one pipeline (the 100M-key batch)
    pmcall) run pmcall 2400 tools/pmc_passes.sh gpurun_out/pmcall ;;
    pmc_c3) run pmc_c3 2400 tools/pmc_passes.sh gpurun_out/pmc_c3 --config c3 ;;
    pmc_c4) run pmc_c4 2400 tools/pmc_passes.sh gpurun_out/pmc_c4 --config c4 ;;
    pmc_c4s) PBF_STREAMS=1 run pmc_c4s 2400 tools/pmc_passes.sh gpurun_out/pmc_c4s --config c4 ;;
    bench_c1) run bench_c1 300 python bench.py --config c1 --steps 50 --warmup 5 ;;
    bench_c3) run bench_c3 600 python bench.py --config c3 --steps 5 --warmup 2 ;;
    bench_c4) run bench_c4 600 python bench.py --config c4 --steps 3 --warmup 1 ;;
    bench_c5) run bench_c5 600 python bench.py --config c5 --steps 5 --warmup 2 ;;
    bench_c5mixed) run bench_c5mixed 600 python bench.py --config c5mixed --steps 5 --warmup 2 ;;
    bench_sst) run bench_sst 600 python bench.py --config sst --steps 20 --warmup 3 ;;
    others) run bench_c1 300 python bench.py --config c1 --steps 50 --warmup 5
            run bench_c3 600 python bench.py --config c3 --steps 5 --warmup 2
            run bench_c4 600 python bench.py --config c4 --steps 3 --warmup 1
            run bench_c5 600 python bench.py --config c5 --steps 5 --warmup 2
            run bench_c5mixed 600 python bench.py --config c5mixed --steps 5 --warmup 2
            run bench_sst 600 python bench.py --config sst --steps 20 --warmup 3 ;;
    prof_c3) prof prof_c3 600 --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive ;;
    prof_c4) prof prof_c4 600 --config c4 --steps 2 --warmup 1 --no-cpu-baseline ;;
    prof_c5) prof prof_c5 600 --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-host-c5 ;;
    ab) ab ab 300 2 --steps 50 --warmup 5 ;;
    ab1) ab ab 300 1 --steps 50 --warmup 5 ;;
    c5sim) for lay in keys filters; do
             run c5sim_${lay}_w8 600 python bench.py --config c5 --sim-world 8 --sim-rank 0 --c5-layout $lay --steps 5 --warmup 2 --no-host-c5 --no-cpu-baseline --no-compare
             run c5sim_${lay}_w2 600 python bench.py --config c5 --sim-world 2 --sim-rank 0 --c5-layout $lay --steps 5 --warmup 2 --no-host-c5 --no-cpu-baseline --no-compare
           done ;;
    c4sim) run c4sim_w8 600 python bench.py --config c4 --sim-world 8 --sim-rank 0 --steps 3 --warmup 1 --no-cpu-baseline ;;
    profab) prof profq_default 300 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive
            for v in build/variants/*.so; do
              nm=$(basename $v .so)
              PBF_LIB=$PWD/$v prof profq_$nm 300 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive
            done ;;
    unaligned) run unaligned 120 tools/microbench/unaligned_loads ;;
    parity_var) for v in build/variants/*.so; do
                  nm=$(basename $v .so)
                  PBF_LIB=$PWD/$v run parity_$nm 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_lsm_get.py tests/test_gpu_device_resident.py -m gpu -x -q -rf --timeout 150 --timeout-method thread -k "${PBF_PARITY_K:-not config4 and not config3}"
                done ;;
    abenv) abenv abenv 300 2 --steps 50 --warmup 5 ;;
    abenv_c5) abenv abenvc5 300 1 --config c5 --steps 5 --warmup 2 --no-host-c5 ;;
    abenv_c3) abenv abenvc3 300 2 --config c3 --steps 3 --warmup 1 ;;
    abenv_c4) abenv abenvc4 400 2 --config c4 --steps 3 --warmup 1 ;;
    prof_var_c3) for v in build/variants/*.so; do
                   nm=$(basename $v .so)
                   PBF_LIB=$PWD/$v prof profv_c3_$nm 300 --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive
                 done ;;
    abenv_c3_1) abenv abenvc3 300 1 --config c3 --steps 3 --warmup 1 ;;
    abenv_c4_1) abenv abenvc4 400 1 --config c4 --steps 3 --warmup 1 ;;
    bench_c1_excl) PBF_SHARED_READERS=0 run bench_c1_excl 300 python bench.py --config c1 --steps 50 --warmup 5 ;;
    prof_c4_serial) PBF_STREAMS=1 prof prof_c4_serial 600 --config c4 --steps 2 --warmup 1 --no-cpu-baseline ;;
    ab_c3) ab abc3 300 1 --config c3 --steps 3 --warmup 1 ;;
    ab_c3_2) ab abc3 300 2 --config c3 --steps 3 --warmup 1 ;;
    ab_c4) ab abc4 400 1 --config c4 --steps 3 --warmup 1 ;;
    ab_c5mixed) ab abc5m 300 1 --config c5mixed --steps 5 --warmup 2 ;;
    ab_c5) ab abc5 300 1 --config c5 --steps 5 --warmup 2 --no-host-c5 ;;
    selflaunch) export PBF_BENCH_DEVICE=0 PBF_BENCH_BACKEND=gloo
                run sl_c2_n2 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-host-inclusive
                run sl_c2_n4 300 python bench.py --gpus 4 --steps 10 --warmup 3 --no-host-inclusive
                run sl_c5_n2 300 python bench.py --gpus 2 --config c5 --steps 3 --warmup 1 --no-host-c5
                unset PBF_BENCH_DEVICE PBF_BENCH_BACKEND ;;
    final_a) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
             run pytest 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 150 --timeout-method thread
             run bench 600 python bench.py
             prof prof 600 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive
             traffic c2 --steps 5 --warmup 2 ;;
    final_b) TRAFFIC_ARGS="--probe-scale 2.0" traffic c3 --config c3 --steps 2 --warmup 1
             traffic c4 --config c4 --steps 2 --warmup 1
             TRAFFIC_ARGS="--probe-scale 3.0" traffic c5 --config c5 --steps 2 --warmup 1 --no-host-c5 --no-compare ;;
    traffic_c5b) TRAFFIC_ARGS="--probe-scale 3.0" traffic c5 --config c5 --steps 2 --warmup 1 --no-host-c5 --no-compare ;;
    traffic_all) traffic c2 --steps 5 --warmup 2
             TRAFFIC_ARGS="--probe-scale 2.0" traffic c3 --config c3 --steps 2 --warmup 1
             traffic c4 --config c4 --steps 2 --warmup 1
             TRAFFIC_ARGS="--probe-scale 3.0" traffic c5 --config c5 --steps 2 --warmup 1 --no-host-c5 --no-compare ;;
    final_1) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
             run pytest 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 150 --timeout-method thread
             run bench 600 python bench.py
             prof prof 600 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive
             run bench_c1 300 python bench.py --config c1 --steps 50 --warmup 5
             PBF_SHARED_READERS=0 run bench_c1_excl 300 python bench.py --config c1 --steps 50 --warmup 5 ;;
    final_2) run bench_c3 600 python bench.py --config c3 --steps 5 --warmup 2
             run bench_c4 600 python bench.py --config c4 --steps 3 --warmup 1
             run bench_c5 600 python bench.py --config c5 --steps 5 --warmup 2
             run bench_c5mixed 600 python bench.py --config c5mixed --steps 5 --warmup 2
             run bench_sst 600 python bench.py --config sst --steps 20 --warmup 3
             prof prof_c3 600 --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive
             PBF_STREAMS=1 prof prof_c4_serial 600 --config c4 --steps 2 --warmup 1 --no-cpu-baseline
             prof prof_c5 600 --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-host-c5
             export PBF_BENCH_DEVICE=0 PBF_BENCH_BACKEND=gloo
             run sl_c2_n2 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-host-inclusive
             run sl_c2_n4 300 python bench.py --gpus 4 --steps 10 --warmup 3 --no-host-inclusive
             unset PBF_BENCH_DEVICE PBF_BENCH_BACKEND ;;
    final_c) run bench_c1 300 python bench.py --config c1 --steps 50 --warmup 5
             PBF_SHARED_READERS=0 run bench_c1_excl 300 python bench.py --config c1 --steps 50 --warmup 5
             run bench_c3 600 python bench.py --config c3 --steps 5 --warmup 2
             run bench_c4 600 python bench.py --config c4 --steps 3 --warmup 1
             run bench_c5 600 python bench.py --config c5 --steps 5 --warmup 2
             run bench_c5mixed 600 python bench.py --config c5mixed --steps 5 --warmup 2
             run bench_sst 600 python bench.py --config sst --steps 20 --warmup 3 ;;
    final_d) prof prof_c3 600 --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive
             PBF_STREAMS=1 prof prof_c4_serial 600 --config c4 --steps 2 --warmup 1 --no-cpu-baseline
             prof prof_c5 600 --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-host-c5
             export PBF_BENCH_DEVICE=0 PBF_BENCH_BACKEND=gloo
             run sl_c2_n2 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-host-inclusive
             run sl_c2_n4 300 python bench.py --gpus 4 --steps 10 --warmup 3 --no-host-inclusive
             unset PBF_BENCH_DEVICE PBF_BENCH_BACKEND ;;
    final) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
           run pytest 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 150 --timeout-method thread
           run bench 600 python bench.py
           prof prof 600 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive
           traffic c2 --steps 5 --warmup 2 ;;
    pmc_c3_insts) for pc in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
                            "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
                    i=$((${i:-0}+1))
                    run pmc_c3_insts_$i 400 rocprofv3 --pmc $pc --kernel-trace --output-format csv -d gpurun_out/pmc_c3_insts_$i -o run -- python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive
                  done ;;
    c5sim8) run c5sim_keys_w8 600 python bench.py --config c5 --sim-world 8 --sim-rank 0 --c5-layout keys --steps 10 --warmup 3 --no-host-c5 --no-cpu-baseline --no-compare
            prof prof_c5sim_keys_w8 600 --config c5 --sim-world 8 --sim-rank 0 --c5-layout keys --steps 10 --warmup 3 --no-host-c5 --no-cpu-baseline --no-compare ;;
    sl_c5) export PBF_BENCH_DEVICE=0 PBF_BENCH_BACKEND=gloo
           run sl_c5_n2 300 python bench.py --gpus 2 --config c5 --steps 3 --warmup 1 --no-host-c5
           unset PBF_BENCH_DEVICE PBF_BENCH_BACKEND ;;
    diag_repl) run diag_repl 300 python tools/diag/replicate_check.py
               run diag_repl_pytest 300 python -u -m pytest tests/test_gpu_device_resident.py -m gpu -x -v -rf --timeout 150 --timeout-method thread -k "replicate" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
