#!/bin/bash
# Upper optimizer range grid with the uncapped lowest dU, then a profile of the headline step.
set -o pipefail
out=gpurun_out/r5_tail2
mkdir -p $out
out=$out ROUNDS=3 STEPS=30 bash scripts/ab_env3.sh "DS2_UPPER_OPT_GRID=512" "DS2_UPPER_OPT_GRID=0" "DS2_UPPER_OPT_GRID=256" || exit 1
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 8 -- python3 bench.py --steps 5 --warmup 3 --no_infer --no_walk > $out/prof.log 2>&1 || exit 1
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 5 --phases > $out/timeline.txt 2>&1 || exit 1
