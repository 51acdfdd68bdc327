#!/bin/bash
# 7 x bi-RNN(ReLU)-1760 (rnnw kernels): BPTT sleep 4 (the default now) vs 2 vs 0, forward 4.
set -o pipefail
out=gpurun_out/r6_relu
mkdir -p $out
X=8388608; F=$((4 << 17))
BENCH_ARGS="--cell rnn_relu --num_hidden 1760 --num_rnn_layers 7 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "DS2_RNNX_KNOBS=0" \
  "DS2_RNNX_KNOBS=$((X + F + (2 << 20)))" "DS2_RNNX_KNOBS=$((X + F))" > $out/ab.txt 2>&1
