#!/bin/bash
# Adaptive pre-poll sleep (knob bit 27, ops/rnn.py) against the static defaults: headline and
# config 5 bf16, same box. Logs: gpurun_out/r6_pace/
set -o pipefail
out=gpurun_out/r6_pace
mkdir -p $out
A=134217728
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "birnn or bptt or wide or unirnn or fused_direction" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 3 "DS2_RNNX_KNOBS=0" "DS2_RNNX_KNOBS=$((A + (4 << 17) + (2 << 20)))" > $out/headline.txt 2>&1 || exit 1
BENCH_ARGS="--num_hidden 1280 --num_rnn_layers 7 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "DS2_RNNX_KNOBS=0" \
  "DS2_RNNX_KNOBS=$((A + (5 << 17)))" > $out/c5bf16.txt 2>&1
