#!/bin/bash
# Same-box A/B of the config-5 recurrence kernels (tools/bench_rnn_fp8.py) between the in-tree
# _C and other builds (DS2_EXT_SO), alternating ROUNDS times: scripts/ab_rnn_fp8.sh 3 ab/_C_head*.so
set -o pipefail
rounds=${1:-3}; shift
for r in $(seq 1 "$rounds"); do
  echo "round $r in-tree"
  timeout -k 10 120 python3 tools/bench_rnn_fp8.py --iters 10 || exit 1
  for so in "$@"; do
    echo "round $r $so"
    DS2_EXT_SO=$so timeout -k 10 120 python3 tools/bench_rnn_fp8.py --iters 10 || exit 1
  done
done
