#!/bin/bash
# DP machinery at world 1 against the single-device path, and a profile of the --force_dp step.
set -o pipefail
out=gpurun_out/r5_dpprof
mkdir -p $out
bash scripts/ab_dp.sh 3 "-1" > $out/ab.txt 2>&1 || exit 1
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 8 -- python3 bench.py --steps 5 --warmup 3 --no_infer --no_walk --force_dp > $out/prof.log 2>&1 || exit 1
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 5 --phases > $out/timeline.txt 2>&1 || exit 1
