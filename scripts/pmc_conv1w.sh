#!/bin/bash
# PMC passes over the conv front-end kernels alone (tools/bench_conv.py), conv1_wgrad focus.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_c1w
mkdir -p $out
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d $out/p$i -o run -- python3 tools/bench_conv.py --iters 3 > $out/p$i.log 2>&1 || { echo "pass $i failed: $set"; exit 1; }
done <<SETS
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_VALU
SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL
TCC_HIT_sum TCC_MISS_sum
SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_BRANCH
SETS
