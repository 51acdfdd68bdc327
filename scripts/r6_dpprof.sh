#!/bin/bash
# Kernel trace of the --force_dp step with conv2's weight gradient on its own stream.
set -o pipefail
out=gpurun_out/r6_dpprof
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 8 -- python3 bench.py --force_dp --steps 5 --warmup 3 --no_infer --no_walk > $out/prof.log 2>&1 || exit 1
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 5 --phases > $out/timeline.txt 2>&1 || exit 1
grep "step period" $out/timeline.txt
