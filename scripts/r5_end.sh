#!/bin/bash
# Round-5 end: full GPU suite, smoke, two driver-default bench runs.
set -o pipefail
out=gpurun_out/r5_end
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/suite.log 2>&1 || exit 1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_$r.log 2>&1 || exit 1
  tail -1 $out/bench_$r.log >> $out/bench.txt
done
