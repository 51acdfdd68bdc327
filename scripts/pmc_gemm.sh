#!/bin/bash
# PMC passes over the headline projection GEMM (7712 x 4800 x 800): counter list first, then one
# rocprofv3 --kernel-trace --pmc pass per counter set (each within the per-block limits).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_gemm
mkdir -p $out
timeout -s KILL 60 rocprofv3 --list-avail > $out/avail.txt 2>&1 || true
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i + 1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $set -d $out/p$i -o run -- python3 tools/g8_pmc_run.py $GEMM_ARGS > $out/p$i.log 2>&1 || { echo "pass $i failed: $set"; exit 1; }
done <<SETS
GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD
TCC_HIT_sum TCC_MISS_sum
TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
SETS
