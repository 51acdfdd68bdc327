#!/bin/bash
# BPTT prefetch-ring LDS stores vectorised (ab/_C_lds16) vs the in-tree build: recurrence
# per-step times (tools/bench_rnn.py) and the headline step, alternated.
set -o pipefail
out=gpurun_out/ab_lds16
mkdir -p $out
ext=$(python -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
for r in 1 2 3; do
  (unset DS2_EXT_SO; timeout -k 10 120 python tools/bench_rnn.py --cell gru --H 800 --kernels xcd --iters 10 > $out/base_$r.log 2>&1) || exit 1
  (export DS2_EXT_SO=ab/_C_lds16${ext}; timeout -k 10 120 python tools/bench_rnn.py --cell gru --H 800 --kernels xcd --iters 10 > $out/lds16_$r.log 2>&1) || exit 1
done
bash scripts/ab_so.sh 3 lds16 > $out/ab.log 2>&1 || exit 1
