#!/bin/bash
# Conv front-end kernels alone (tools/bench_conv.py, headline geometry): a kernel-trace summary,
# then PMC passes (kernel trace only, one counter set per run, within one block's limits)
set -o pipefail
export TMPDIR=/tmp
out=${1:-gpurun_out/pmc_conv}
mkdir -p $out
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 tools/bench_conv.py --iters 5 > $out/trace.log 2>&1 || exit 1
python3 tools/rocpd_summary.py $out/trace/run_results.db -o $out/kernels.md > /dev/null || exit 1
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d $out/p$i -o run -- python3 tools/bench_conv.py --iters 2 > $out/p$i.log 2>&1 || exit 1
done
python3 tools/rocpd_pmc.py $out/p*/run_results.db -o $out/pmc.md > /dev/null
