#!/bin/bash
# Same-box alternating A/B of DS2_BESIDE_GRID (-1: the BPTT's idle CUs, 0: whole chip) on the
# configurations whose weight gradients run beside the BPTT: config 5 bf16 / fp8, and the
# headline with the data-parallel machinery forced on.
set -o pipefail
rounds=${1:-2}
for r in $(seq 1 "$rounds"); do
  for cfg in "--num_hidden 1280 --num_rnn_layers 7" "--num_hidden 1280 --num_rnn_layers 7 --fp8" "--force_dp"; do
    for g in -1 0; do
      out=$(DS2_BESIDE_GRID=$g timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_walk --no_infer $cfg | tail -1) || exit 1
      echo "round $r [$cfg] DS2_BESIDE_GRID=$g $(echo "$out" | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
