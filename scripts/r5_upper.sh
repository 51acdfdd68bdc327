#!/bin/bash
# Upper optimizer range on its own stream: A/B, then the bitwise early-range tests with it on.
set -o pipefail
out=gpurun_out/r5_upper
mkdir -p $out
out=$out ROUNDS=3 STEPS=30 bash scripts/ab_env3.sh "DS2_UPPER_STREAM=0" "DS2_UPPER_STREAM=1" "DS2_UPPER_STREAM=1 DS2_UPPER_OPT_GRID=0" || exit 1
DS2_UPPER_STREAM=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "early_optimizer_range or bitwise or deterministic" > $out/tests.log 2>&1 || exit 1
