#!/bin/bash
# Same-box alternating A/B of one environment switch on the headline bench:
#   bash scripts/ab_env2.sh ROUNDS VAR VALUE_A VALUE_B [bench args...]
set -o pipefail
rounds=$1; var=$2; va=$3; vb=$4; shift 4
for r in $(seq 1 "$rounds"); do
  for v in "$va" "$vb"; do
    out=$(env "$var=$v" timeout -k 10 120 python bench.py --steps 30 --warmup 10 "$@" | tail -1) || exit 1
    echo "$var=$v $(echo "$out" | grep -o '"ms_per_step": [0-9.]*')"
  done
done
