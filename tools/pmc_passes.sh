#!/bin/bash
# Collect PMC counter passes (one rocprofv3 run per pass) for a short bench run.
# Usage: tools/pmc_passes.sh OUTDIR [bench args...]
set -u
out=$1; shift
mkdir -p "$out"
passes=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum"
)
i=0
for p in "${passes[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $p --output-format csv -d "$out/p$i" -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive "$@" > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
