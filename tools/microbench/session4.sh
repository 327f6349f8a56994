set -u
# A/B of the loop-entry wait fix (rb_new: before; rb_wait: after), the probe pass with it, the
# one-key latency probe, the instruction accounting of the ring partition, then the GPU tests
cd /root/repo
rm -f gpurun_out/rb.txt gpurun_out/pb4.txt
tools/microbench/run_rb.sh rb_new rb_wait rb_waitplain rb_synthnost2 rb_wait || exit 1
cd tools/microbench
for b in pb_wait pb_wait_hw0 pb_wait; do
  echo "== $b" >> ../../gpurun_out/pb4.txt
  timeout -k 5 120 ./$b 20 >> ../../gpurun_out/pb4.txt 2>&1 || { echo "$b rc=$?"; cat ../../gpurun_out/pb4.txt; exit 1; }
done
cat ../../gpurun_out/pb4.txt
timeout -k 5 60 ./pingpong > ../../gpurun_out/pingpong.txt 2>&1; rc=$?; cat ../../gpurun_out/pingpong.txt; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
for nm in rb_wait rb_noappend rb_synthnost2; do
  out=../../gpurun_out/pmci_$nm
  mkdir -p $out
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH --output-format csv -d $out -o run -- ./$nm 5 > $out.log 2>&1
  rc=$?; echo "$nm pmc rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out.log; exit $rc; }
done
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; exit $rc
