#!/bin/bash
# Same-box alternating A/B of the data-parallel machinery's cost at world size 1 (VERDICT r4
# item 5, r5 item 5): plain bench.py against bench.py --force_dp.
#   bash scripts/ab_dp.sh ROUNDS [bench args...]
set -o pipefail
rounds=$1; shift 1
for r in $(seq 1 "$rounds"); do
  out=$(timeout -k 10 150 python bench.py --steps 30 --warmup 10 --no_walk --no_infer "$@" | tail -1) || exit 1
  echo "round $r plain $(echo "$out" | grep -o '"ms_per_step": [0-9.]*')"
  out=$(timeout -k 10 150 python bench.py --steps 30 --warmup 10 --no_walk --no_infer --force_dp "$@" | tail -1) || exit 1
  echo "round $r force_dp $(echo "$out" | grep -o '"ms_per_step": [0-9.]*')"
done
