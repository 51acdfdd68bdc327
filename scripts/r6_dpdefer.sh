#!/bin/bash
# DP short sequences on the single-device (grouped, deferred) weight-gradient schedule.
set -o pipefail
out=gpurun_out/r6_dpdefer
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dp_ready_gpu.py \
  tests/test_dp_gpu.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for fr in 100 200 400; do
  for a in "--step_graphs" "--force_dp" "--force_dp --step_graphs"; do
    o=$(timeout -k 10 200 python bench.py --frames $fr --steps 50 --warmup 10 --no_infer --no_walk $a | tail -1) || exit 1
    echo "[frames $fr] [${a:-eager}] $(echo "$o" | grep -o '"ms_per_step": [0-9.]*')" | tee -a $out/short.txt
  done
done
timeout -k 10 300 python -u -m pytest -x -s -q --timeout 250 --timeout-method thread "tests/test_engine_gpu.py::test_headline_geometry_matches_reference" 2>&1 | grep -E "passed|failed|over tolerance" | tee $out/tol.txt
