#!/bin/bash
# dU grid cap A/B, then the engine / DP / step-graph GPU tests.
set -o pipefail
out=gpurun_out/r5_du
mkdir -p $out
out=$out ROUNDS=3 STEPS=30 bash scripts/ab_env3.sh "DS2_DU_UNCAP=low" "DS2_DU_UNCAP=all" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_dp_ready_gpu.py tests/test_dp_gpu.py tests/test_step_graphs_gpu.py > $out/tests.log 2>&1 || exit 1
