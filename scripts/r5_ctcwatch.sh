#!/bin/bash
# Fused loss mean + divergence watch in the CTC gradient launch: tests, then A/B against the
# separate launches is not possible in one build, so the headline and 100-frame graph step are timed.
set -o pipefail
out=gpurun_out/r5_ctcwatch
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stats_gpu.py tests/test_step_graphs_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_convergence_gpu.py > $out/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --no_walk --no_infer --steps 30 --warmup 5 > $out/b.log 2>&1 || exit 1
  echo "headline round $r: $(tail -1 $out/b.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $out/ab.txt
  timeout -k 10 200 python tools/host_overhead.py --frames 100,200 --steps 30 --graph > $out/ho_$r.log 2>&1 || exit 1
done
