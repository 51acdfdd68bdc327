#!/bin/bash
# Same-box A/B of compile-time variants on the recurrence kernels alone (headline layer shape:
# GRU H=800, N=32, T=241, bidirectional): the in-tree _C against each ab/_C_<NAME>.so built by
# `build.py --variant NAME -D ...`, ROUNDS times. Less noisy than scripts/ab_so.sh for changes
# inside the recurrence kernels.
#   bash scripts/rnn_ab.sh ROUNDS NAME [NAME...] > gpurun_out/rnnab.log
set -o pipefail
rounds=${1:-3}; shift
ext=$(python -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
for r in $(seq 1 "$rounds"); do
  for v in base "$@"; do
    if [ "$v" = base ]; then unset DS2_EXT_SO; else export DS2_EXT_SO=ab/_C_${v}${ext}; fi
    echo "== $v $r"
    timeout -k 10 120 python tools/bench_rnn.py --cell gru --H 800 --N 32 --T 241 --ndir 2 --iters 20 \
      --kernels xcd || exit 1
  done
done
