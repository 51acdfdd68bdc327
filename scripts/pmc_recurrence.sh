#!/bin/bash
# PMC counters of the headline recurrence kernels (rnne forward, rnnrs BPTT; BiGRU-800, N = 32,
# T = 241) via tools/bench_rnn.py, one pass per counter set, kernel trace only.
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_rec
mkdir -p $out
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_VALU -d $out/p1 -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rnn.py --cell gru --H 800 --kernels xcd --iters 2 > $out/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM TCC_HIT_sum TCC_MISS_sum -d $out/p2 -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rnn.py --cell gru --H 800 --kernels xcd --iters 2 > $out/p2.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 tools/rocpd_pmc.py --match rnn $(ls $out/p1/*.db | head -1) $(ls $out/p2/*.db | head -1) -o $out/pmc.md > $out/sum.log 2>&1 || exit 1
