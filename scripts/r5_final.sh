#!/bin/bash
# Round-5 end numbers: headline bench twice (driver defaults), then a kernel-trace profile of the
# headline step and its timeline (tail after the last BPTT).
set -o pipefail
out=gpurun_out/r5_final
mkdir -p $out
for r in 1 2; do
  timeout -k 10 300 python bench.py > $out/bench_$r.log 2>&1 || exit 1
  tail -1 $out/bench_$r.log >> $out/bench.txt
done
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 8 -- python3 bench.py --steps 5 --warmup 3 --no_infer --no_walk > $out/prof.log 2>&1 || exit 1
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 5 --phases > $out/timeline.txt 2>&1 || exit 1
