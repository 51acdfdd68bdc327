#!/bin/bash
# config 5 (fp8): early optimizer range of the upper stack beside layer 0's BPTT (A/B)
set -o pipefail
for r in 1 2; do
  for v in "DS2_EARLY_UPPER=0" "DS2_EARLY_UPPER=1" "DS2_UPPER_GRID=192" "DS2_UPPER_GRID=512"; do
    out=$(env $v timeout -k 10 120 python bench.py --num_hidden 1280 --num_rnn_layers 7 --steps 15 --warmup 5 --fp8 | tail -1) || exit 1
    echo "$v $(echo "$out" | grep -o '"ms_per_step": [0-9.]*')"
  done
done
