#!/bin/bash
# Same-box A/B of environment settings on the headline bench, alternating arms per round.
#   scripts/ab_env.sh <rounds> "<arm A env>" "<arm B env>" [...]
# e.g. scripts/ab_env.sh 3 "DS2_SPLIT_ADAM=1" "DS2_SPLIT_ADAM=0"
# Prints one line per run: the arm, the round and ms/step. Extra bench flags: $BENCH_ARGS.
set -o pipefail
rounds="$1"; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 "$rounds"); do
  a=0
  for arm in "$@"; do
    a=$((a + 1))
    log=gpurun_out/ab/arm${a}_r${r}.log
    env $arm timeout -k 10 150 python bench.py --steps ${STEPS:-30} --warmup 5 $BENCH_ARGS > "$log" 2>&1 || { tail -20 "$log"; exit 1; }
    echo "[$arm] round $r: $(tail -1 "$log" | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])') ms/step"
  done
done
