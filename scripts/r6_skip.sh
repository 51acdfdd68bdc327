#!/bin/bash
# Round 6: gemm8 dead-quadrant skipping (ragged tiles) + nt loads on the column GEMMs; GEMM /
# kernel / reduce tests, production-geometry trajectories, same-box A/B against the build
# without skipping, glue ops left in the step.
set -o pipefail
out=gpurun_out/r6_skip
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gemm_gpu.py \
  tests/test_reduce_gpu.py tests/test_trajectory_production_gpu.py -s > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
grep -E "windowed|passed|failed" $out/tests.log | tail -8
BENCH_ARGS="--no_infer --no_walk" timeout -k 10 400 bash scripts/ab_so.sh 3 noskip > $out/ab.log 2>&1 || exit 1
grep -o '"variant": "[a-z]*", "round": [0-9]*\|"ms_per_step": [0-9.]*' $out/ab.log | paste - - | tee $out/ab.txt
timeout -k 10 200 python tools/glue_ops.py > $out/glue.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/glue.txt | head -60
