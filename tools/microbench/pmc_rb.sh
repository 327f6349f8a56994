#!/bin/bash
# PMC passes (one rocprofv3 run each) over ring_bench variant binaries.
# Usage: tools/microbench/pmc_rb.sh NAME...   (output: gpurun_out/pmc_<name>/p<i>)
cd "$(dirname "$0")"
export TMPDIR=/tmp
passes=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL"
  "SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT SQ_LDS_ATOMIC_RETURN"
  "TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
)
for nm in "$@"; do
  i=0
  for p in "${passes[@]}"; do
    out=../../gpurun_out/pmc_$nm/p$i
    mkdir -p $out
    timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $out -o run -- ./$nm 5 > $out.log 2>&1
    rc=$?
    echo "$nm pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $out.log; exit $rc; fi
    i=$((i+1))
  done
done
