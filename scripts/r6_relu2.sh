#!/bin/bash
# 7 x bi-RNN(ReLU)-1760 (rnnw): forward sleep 2 / 3 vs 4 (default), BPTT 4.
set -o pipefail
out=gpurun_out/r6_relu2
mkdir -p $out
X=8388608; B=$((4 << 20))
BENCH_ARGS="--cell rnn_relu --num_hidden 1760 --num_rnn_layers 7 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 3 "DS2_RNNX_KNOBS=0" \
  "DS2_RNNX_KNOBS=$((X + B + (2 << 17)))" "DS2_RNNX_KNOBS=$((X + B + (3 << 17)))" > $out/ab.txt 2>&1
