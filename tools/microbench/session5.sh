set -u
# wait/issue counters of the ring partition with and without memory traffic, then the GPU tests,
# the per-key latency bench (resident reader), the headline bench and its profile
cd /root/repo/tools/microbench
export TMPDIR=/tmp
for nm in rb_wait rb_synthnost2; do
  out=../../gpurun_out/pmcw_$nm
  mkdir -p $out
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES --output-format csv -d $out -o run -- ./$nm 5 > $out.log 2>&1
  rc=$?; echo "$nm pmc rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out.log; exit $rc; }
done
cd /root/repo
bash tools/gpu_session.sh pytest bench_c1 bench prof
