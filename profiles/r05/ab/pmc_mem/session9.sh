set -u
# memory-pipeline counters of the ring partition, shipped (rb_cur) vs keys made in registers and
# no region stores (rb_synthnost2): where the ~78 us of memory-induced time goes
cd /root/repo/tools/microbench
export TMPDIR=/tmp
passes=(
  "TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
  "TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
  "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum"
  "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES SQ_WAIT_ANY"
)
for nm in rb_cur rb_synthnost2; do
  i=0
  for p in "${passes[@]}"; do
    out=../../gpurun_out/pmcm_$nm/p$i
    mkdir -p $out
    timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $out -o run -- ./$nm 5 > $out.log 2>&1
    rc=$?
    echo "$nm pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 $out.log; fi
    i=$((i+1))
  done
done
exit 0
