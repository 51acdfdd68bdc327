#!/bin/bash
# Kernel trace of the final round-6 headline step: timeline and per-step census.
set -o pipefail
out=gpurun_out/r6_prof_final
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 8 -- python3 bench.py --steps 5 --warmup 3 --no_infer --no_walk > $out/prof.log 2>&1 || exit 1
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 5 --phases > $out/timeline.txt 2>&1 || exit 1
python3 tools/step_kernels.py $db > $out/step_kernels.md 2>&1 || exit 1
grep "step period" $out/timeline.txt
