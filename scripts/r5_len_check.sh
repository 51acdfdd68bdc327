#!/bin/bash
# Length-dependent partial deferral: early-range tests, headline + epoch walk, per-length A/B.
set -o pipefail
out=gpurun_out/r5_len
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "early_optimizer_range" > $out/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py > $out/bench_$r.log 2>&1 || exit 1
  tail -1 $out/bench_$r.log >> $out/bench.txt
done
for r in 1 2; do
  for arm in "DS2_PARTIAL_MIN_T=160" "DS2_PARTIAL_MIN_T=0" "DS2_PARTIAL_MIN_T=100000"; do
    env $arm timeout -k 10 200 python tools/host_overhead.py --frames 600,700,800 --steps 20 > $out/ho.log 2>&1 || exit 1
    echo "$arm round $r" >> $out/ho.txt; cat $out/ho.log >> $out/ho.txt
  done
done
