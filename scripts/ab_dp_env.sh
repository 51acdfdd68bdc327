#!/bin/bash
# Same-box A/B of environment arms on bench.py --force_dp (DP machinery at world 1).
#   out=gpurun_out/x ROUNDS=3 bash scripts/ab_dp_env.sh "A=1" "A=0"
set -o pipefail
out=${out:-gpurun_out/abdp}
mkdir -p $out
for r in $(seq 1 ${ROUNDS:-3}); do
  for arm in "$@"; do
    env $arm timeout -k 10 150 python bench.py --no_walk --no_infer --force_dp --steps ${STEPS:-30} --warmup 5 > $out/b.log 2>&1 || exit 1
    echo "$arm round $r: $(tail -1 $out/b.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $out/ab.txt
  done
done
