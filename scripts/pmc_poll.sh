#!/bin/bash
# PMC counters of the headline recurrence kernels with the poll timing of round 6 (defaults)
# against drained polls with no sleep (DS2_RNNX_KNOBS bit 23): vector-memory read instructions
# issued (each stale poll round re-issues its loads) and L2 hits / misses per dispatch.
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_poll
mkdir -p $out
cd /tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $out/def -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rnn.py --cell gru --H 800 --kernels xcd --iters 2 --knobs 0 > $out/def.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $out/nosleep -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rnn.py --cell gru --H 800 --kernels xcd --iters 2 --knobs 8388608 > $out/nosleep.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 tools/rocpd_pmc.py --match rnn $(ls $out/def/*.db | head -1) -o $out/pmc_default.md > $out/sum1.log 2>&1 || exit 1
python3 tools/rocpd_pmc.py --match rnn $(ls $out/nosleep/*.db | head -1) -o $out/pmc_nosleep.md > $out/sum2.log 2>&1
