#!/bin/bash
# In-tree single-device beside grid 40 (schedule_for): trajectory / deferral / DP GPU tests and
# the driver bench twice. Logs: gpurun_out/r6_beside3/
set -o pipefail
out=gpurun_out/r6_beside3
mkdir -p $out
timeout -k 10 800 python -u -m pytest tests/test_trajectory_production_gpu.py tests/test_defer_update_gpu.py tests/test_dp_ready_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --no_infer > $out/bench$r.json 2> $out/bench$r.err || { tail -20 $out/bench$r.err; exit 1; }
  tail -1 $out/bench$r.json | cut -c1-200
done
