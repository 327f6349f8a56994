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
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest_multi) run pytest_multi 600 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -v -rf --timeout 300 --timeout-method thread ;;
    pytest) run pytest 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 120 --timeout-method thread ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5 ;;
    bench_c3) run bench_c3 600 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline ;;
    bench_c4) run bench_c4 600 python bench.py --config c4 --steps 3 --warmup 1 ;;
    bench_c5) run bench_c5 600 python bench.py --config c5 --steps 5 --warmup 2 ;;
    prof_c34) run prof_c4 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- python bench.py --config c4 --steps 2 --warmup 1
              python tools/prof_summary.py gpurun_out/prof_c4 > gpurun_out/prof_c4_summary.txt 2>&1
              ;;
    prof_c3) run prof_c3 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline
              python tools/prof_summary.py gpurun_out/prof_c3 > gpurun_out/prof_c3_summary.txt 2>&1 ;;
    gsplit) for sp in ${PBF_SPLITS:-8 12 16}; do PBF_GATHER_SPLIT=$sp run gsplit_$sp 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive; done ;;
    screen) PBF_PROBE_ROUNDS=2 run screen_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_resident.py -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "strategies or config2 or device_resident_equals or splitmix or sweep or incremental or tails or golden"
            PBF_PROBE_ROUNDS=2 run screen_bench 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive
            run noscreen_bench 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive ;;
    prof_screen) PBF_PROBE_ROUNDS=2 run prof_screen 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_screen -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive
                 python tools/prof_summary.py gpurun_out/prof_screen > gpurun_out/prof_screen_summary.txt 2>&1 ;;
    pytest_both) PBF_LIB=$PWD/build/variants/both.so run pytest_both 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_resident.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "strategies or config2 or device_resident_equals or sweep or golden" ;;
    final) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
           run pytest 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread
           run bench 600 python bench.py --steps 20 --warmup 5
           run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
           python tools/prof_summary.py gpurun_out/prof > gpurun_out/prof_summary.txt 2>&1
           run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive
           run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive
           run bench_c3 600 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline
           run bench_c4 600 python bench.py --config c4 --steps 3 --warmup 1
           run bench_c5 600 python bench.py --config c5 --steps 5 --warmup 2 ;;
    rehearse) export PBF_BENCH_DEVICE=0 PBF_BENCH_BACKEND=gloo
              run rh_c2_n2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3
              run rh_c2_n4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 10 --warmup 3
              run rh_c5_n2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --config c5 --steps 3 --warmup 1
              run rh_c4_n2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --config c4 --steps 2 --warmup 1
              unset PBF_BENCH_DEVICE PBF_BENCH_BACKEND ;;
    pytest_sst) run pytest_sst 600 python -u -m pytest tests/test_gpu_sstable_data.py -m gpu -x -v -rf --timeout 300 --timeout-method thread ;;
    bench_sst) run bench_sst 600 python bench.py --config sst --steps 20 --warmup 3
               run prof_sst 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sst -o run -- python bench.py --config sst --steps 10 --warmup 2 --cpu-seconds 1
               python tools/prof_summary.py gpurun_out/prof_sst > gpurun_out/prof_sst_summary.txt 2>&1 ;;
    prof_c5) run prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python bench.py --config c5 --steps 3 --warmup 1
             python tools/prof_summary.py gpurun_out/prof_c5 > gpurun_out/prof_c5_summary.txt 2>&1 ;;
    bench_atomic) run bench_atomic 600 python bench.py --steps 10 --warmup 3 --build-mode 1 --no-cpu-baseline ;;
    bench_tt) run bench_tt 300 python bench.py --steps 20 --warmup 5 --build-mode 2 --probe-mode 2 --no-cpu-baseline --no-host-inclusive ;;
    bench_modes) for bm in 1 2; do for pm in 1 2; do run bench_b${bm}_p${pm} 300 python bench.py --steps 20 --warmup 5 --build-mode $bm --probe-mode $pm --no-cpu-baseline; done; done ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
          python tools/prof_summary.py gpurun_out/prof > gpurun_out/prof_summary.txt 2>&1 || true ;;
    probe_s1) for s1 in 1 2 3 6; do PBF_PROBE_S1=$s1 run probe_s1_$s1 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline; done ;;
    pmc) run counters 120 rocprofv3 -L
         run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
         run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
         run pmc_tcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/pmc_tcc -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    traffic) run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive ${PBF_BENCH_ARGS:-}
             run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive ${PBF_BENCH_ARGS:-} ;;
    micro) run micro 300 tools/microbench/lds_rates ;;
    variants2) for r in 1 2; do for v in build/variants/*.so; do nm=$(basename $v .so); PBF_LIB=$PWD/$v run var_${nm}_$r 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive; done; done ;;
    variants) for v in build/variants/*.so; do nm=$(basename $v .so); PBF_LIB=$PWD/$v run var_$nm 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive; done
              run var_default 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive ;;
    variants_c3) for r in 1 2; do for v in build/variants/*.so; do nm=$(basename $v .so); PBF_LIB=$PWD/$v run c3var_${nm}_$r 300 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive; done; done ;;
    final2) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
            run pytest 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 150 --timeout-method thread
            run bench 600 python bench.py
            run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive
            python tools/prof_summary.py gpurun_out/prof > gpurun_out/prof_summary.txt 2>&1 || true
            run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive
            run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive
            python tools/traffic_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/traffic_c2.json > gpurun_out/traffic_summary.txt 2>&1 || true ;;
    others) run bench_c1 300 python bench.py --config c1 --steps 50 --warmup 5
            run bench_c3 600 python bench.py --config c3 --steps 5 --warmup 2
            run bench_c4 600 python bench.py --config c4 --steps 3 --warmup 1
            run bench_c5 600 python bench.py --config c5 --steps 5 --warmup 2
            run bench_sst 600 python bench.py --config sst --steps 20 --warmup 3 ;;
    parity) run parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_resident.py -m gpu -x -q -rf --timeout 150 --timeout-method thread ;;
    profq) run profq 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profq -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive
           python tools/prof_summary.py gpurun_out/profq > gpurun_out/profq_summary.txt 2>&1 || true ;;
    benchq) for r in 1 2; do run benchq_$r 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-host-inclusive; done ;;
    rphases)run rphases 300 tools/microbench/ring_phases ;;
    rtime) for b in ring_time ring_time_synth ring_time_nostore ring_time_synth_nostore; do run $b 300 tools/microbench/$b; done ;;
    phases) run phases_t0 300 tools/microbench/part_phases 0
            run phases_t16 300 tools/microbench/part_phases 16 ;;
    gapdiag) run native0 120 tools/microbench/pipeline_bench 50 0
             run native1 120 tools/microbench/pipeline_bench 50 1
             run native2 120 tools/microbench/pipeline_bench 50 2
             run native0b 120 tools/microbench/pipeline_bench 200 0
             run py_ev 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive
             run py_noev 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-events ;;
    pmcall) run pmcall 2400 tools/pmc_passes.sh gpurun_out/pmcall ;;
    pmcdirect) run pmcdirect 2400 tools/pmc_passes.sh gpurun_out/pmcdirect --probe-mode 1 ;;
    diag) run diag_a 300 python bench.py --steps 20 --warmup 5 --build-mode 2 --probe-mode 1 --no-cpu-baseline
          run diag_b 300 python bench.py --steps 20 --warmup 5 --build-mode 2 --probe-mode 1 --no-cpu-baseline --no-events
          run diag_c 300 python bench.py --steps 20 --warmup 5 --build-mode 2 --probe-mode 1 --no-cpu-baseline --sync-each-step
          run diag_d 300 python bench.py --steps 20 --warmup 5 --build-mode 2 --probe-mode 1 --no-cpu-baseline --no-events --sync-each-step
          run diag_e 300 python bench.py --steps 100 --warmup 5 --build-mode 2 --probe-mode 1 --no-cpu-baseline ;;
    tdepth) for t in 0 8 16; do PBF_TDEPTH=$t run tdepth_$t 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive; done
            for t in 0 8 16; do PBF_TDEPTH=$t run tdepth_prof_$t 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tdprof_$t -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive
                              python tools/prof_summary.py gpurun_out/tdprof_$t > gpurun_out/tdprof_$t.txt 2>&1; done ;;
    rep) run rep_long 300 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-host-inclusive
         for r in 1 2 3; do run rep_$r 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive; done
         run rep_native 120 tools/microbench/pipeline_bench 50 0
         run rep_native_ev 120 tools/microbench/pipeline_bench 50 1 ;;
    wrreq) run counters 120 rocprofv3 -L
           for t in 0 16; do PBF_TDEPTH=$t run wrreq_$t 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/wrreq_$t -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive; done ;;
    chunks) for c in ${PBF_CHUNKS:-2000000 4000000 6000000 10000000}; do PBF_PROBE_CHUNK=$c run chunk_$c 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-inclusive; done
            run chunk_none 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-inclusive ;;
    pytest_new) run pytest_new 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_dropin.py tests/test_gpu_distributed.py tests/test_gpu_lsm_get.py -m gpu -x -v -rf --timeout 600 --timeout-method thread ;;
    bench_c1) run bench_c1 300 python bench.py --config c1 --steps 50 --warmup 5 ;;
    bench_sst2) run bench_sst 600 python bench.py --config sst --steps 20 --warmup 3 ;;
    prof_c34ab) for part in ring sort; do
                  PBF_PART=$part run prof_c3_$part 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_$part -o run -- python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive
                  python tools/prof_summary.py gpurun_out/prof_c3_$part > gpurun_out/prof_c3_${part}_summary.txt 2>&1
                  PBF_PART=$part run prof_c4_$part 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4_$part -o run -- python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline
                  python tools/prof_summary.py gpurun_out/prof_c4_$part > gpurun_out/prof_c4_${part}_summary.txt 2>&1
                done ;;
    gsweep) for sp in 4 8 16; do for qt in 0 1; do PBF_GATHER_SPLIT=$sp PBF_GATHER_QTAB=$qt run gs_${sp}_q$qt 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-host-inclusive; done; done ;;
    selflaunch) export PBF_BENCH_DEVICE=0 PBF_BENCH_BACKEND=gloo
                run sl_c2_n2 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-host-inclusive
                run sl_c2_n4 300 python bench.py --gpus 4 --steps 10 --warmup 3 --no-host-inclusive
                run sl_c5_n2 300 python bench.py --gpus 2 --config c5 --steps 3 --warmup 1 --no-host-c5
                unset PBF_BENCH_DEVICE PBF_BENCH_BACKEND ;;
    gsweepG) for G in ${PBF_GS:-256 512 1024}; do PBF_PART_G=$G run c3_G$G 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive; done
             for G in 256 512; do PBF_PART_G=$G run c2_G$G 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-inclusive; done ;;
    gpacked) for r in 1 2; do for pk in 0 1; do PBF_GATHER_PACKED=$pk run gp${pk}_c2_$r 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-host-inclusive; done; done
             for pk in 0 1; do PBF_GATHER_PACKED=$pk run gp${pk}_c5 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-host-c5; done ;;
    direct) for s1 in 1 2 6; do PBF_PROBE_S1=$s1 run direct_s1_$s1 300 python bench.py --steps 40 --warmup 5 --probe-mode 1 --no-cpu-baseline --no-host-inclusive; done
            run prof_direct 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_direct -o run -- python bench.py --steps 20 --warmup 5 --probe-mode 1 --no-cpu-baseline --no-host-inclusive
            python tools/prof_summary.py gpurun_out/prof_direct > gpurun_out/prof_direct_summary.txt 2>&1 || true ;;
    ab) # A/B: the default library against every build/variants/*.so, alternating, PBF_AB_ARGS for the bench
        for r in 1 2; do
          run ab_default_$r 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive ${PBF_AB_ARGS:-}
          for v in build/variants/*.so; do nm=$(basename $v .so); PBF_LIB=$PWD/$v run ab_${nm}_$r 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive ${PBF_AB_ARGS:-}; done
        done ;;
    ab_c5) run abc5_default 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-host-c5
           for v in build/variants/*.so; do nm=$(basename $v .so); PBF_LIB=$PWD/$v run abc5_${nm} 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-host-c5; done ;;
    ab_c3) run abc3_default 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive
           for v in build/variants/*.so; do nm=$(basename $v .so); PBF_LIB=$PWD/$v run abc3_${nm} 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive; done ;;
    overlap) for r in 1 2; do for c in 0 2 3 4; do PBF_PROBE_OVERLAP=$c run ov${c}_$r 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive; done; done ;;
    overlap_parity) PBF_PROBE_OVERLAP=3 run ov_parity 600 python -u -m pytest tests/test_gpu_device_resident.py tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 150 --timeout-method thread ;;
    parity_var) for v in build/variants/*.so; do nm=$(basename $v .so); PBF_LIB=$PWD/$v run parity_$nm 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_resident.py tests/test_gpu_multi.py -m gpu -x -q -rf --timeout 300 --timeout-method thread; done ;;
    halves) for r in 1 2; do for h in 2 1; do PBF_RING_HALVES=$h run hv${h}_$r 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-inclusive; done; done
            for h in 2 1; do PBF_RING_HALVES=$h run hvc5_$h 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-host-c5; done ;;
    rtime2) for b in ring_time ring_time_nostore ring_time_noappend ring_time_hashonly ring_time_synth_hashonly; do run $b 300 tools/microbench/$b; done ;;
    rtime3) for b in ring_time ring_time_noappend ring_time_hashonly; do run $b 300 tools/microbench/$b; done ;;
    c4ab) for r in 1 2; do for lg in 31 30; do PBF_BUILD_POSITIONS_LOG2=$lg run c4ab_${lg}_$r 400 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline; done; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
