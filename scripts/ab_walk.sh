#!/bin/bash
# Same-box A/B of environment arms on the headline AND the SortaGrad epoch walk
# (bench.py --no_infer), arms alternated each round; appends "arm round: ms walk" lines.
#   out=gpurun_out/x ROUNDS=3 bash scripts/ab_walk.sh "A=1" "A=0"
set -o pipefail
out=${out:-gpurun_out/abw}
mkdir -p $out
for r in $(seq 1 ${ROUNDS:-3}); do
  for arm in "$@"; do
    env $arm timeout -k 10 240 python bench.py --no_infer --steps ${STEPS:-30} --warmup 5 $BENCH_ARGS > $out/b.log 2>&1 || exit 1
    echo "$arm round $r: $(tail -1 $out/b.log | python3 -c 'import sys,json; j=json.loads(sys.stdin.read()); w=j["epoch_walk"]; print(j["ms_per_step"], w["audio_s_per_s"], w["eager_audio_s_per_s"])')" >> $out/ab.txt
  done
done
