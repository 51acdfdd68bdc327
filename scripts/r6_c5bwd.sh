#!/bin/bash
# Config 5 bf16 (R = 16 BPTT across XCDs): longer BPTT pre-gather sleeps (bit 29: units x4).
set -o pipefail
out=gpurun_out/r6_c5bwd
mkdir -p $out
X=8388608; F=$((5 << 17)); Q=$((1 << 29))
BENCH_ARGS="--num_hidden 1280 --num_rnn_layers 7 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "DS2_RNNX_KNOBS=0" \
  "DS2_RNNX_KNOBS=$((X + F + Q + (3 << 20)))" "DS2_RNNX_KNOBS=$((X + F + Q + (5 << 20)))" "DS2_RNNX_KNOBS=$((X + F + Q + (7 << 20)))" > $out/ab.txt 2>&1
