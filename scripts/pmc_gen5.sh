#!/bin/bash
# PMC counters of the generation-4 vs generation-5 GRU forward (one process each, kernel trace
# only): vector-memory read instructions, LDS / MFMA / VALU instruction counts, L2 read requests
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc
mkdir -p $out
for k in 0 4194304; do
  DS2_RNNX_KNOBS=$k timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES TCP_TCC_READ_REQ_sum -d $out/k$k -o run -- python3 tools/bench_rnn.py --cell gru --H 800 --kernels xcd --knobs $k --iters 2 > $out/k$k.log 2>&1 || exit 1
done
