#!/bin/bash
# Same-box A/B of environment arms on the headline (bench.py --no_walk --no_infer), arms
# alternated each round; appends "arm round ms" lines to $out/ab.txt.
#   out=gpurun_out/x ROUNDS=5 bash scripts/ab_env3.sh "A=1" "A=0"
set -o pipefail
out=${out:-gpurun_out/ab3}
mkdir -p $out
for r in $(seq 1 ${ROUNDS:-5}); do
  for arm in "$@"; do
    env $arm timeout -k 10 150 python bench.py --no_walk --no_infer --steps ${STEPS:-40} --warmup 5 $BENCH_ARGS > $out/b.log 2>&1 || exit 1
    echo "$arm round $r: $(tail -1 $out/b.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $out/ab.txt
  done
done
