#!/bin/bash
# The poll-timing changes on the other shipped configurations: production (ab/_C_nodrain,
# explicit no sleep) vs the in-tree defaults, config 5 bf16 (H = 1280: rnnq forward, R = 16
# BPTT) and the reference's 7 x bi-RNN(ReLU)-1760 (rnnw kernels). Logs: gpurun_out/r6_cfgcheck/
set -o pipefail
out=gpurun_out/r6_cfgcheck
mkdir -p $out
E="DS2_EXT_SO=ab/_C_nodrain.cpython-310-x86_64-linux-gnu.so DS2_RNNX_KNOBS=8388608"
BENCH_ARGS="--cell rnn_relu --num_hidden 1760 --num_rnn_layers 7 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "$E" "DS2_RNNX_KNOBS=0" \
  "DS2_RNNX_KNOBS=$((2 << 17))" > $out/relu1760.txt 2>&1 || exit 1
BENCH_ARGS="--num_hidden 1280 --num_rnn_layers 7 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "$E" "DS2_RNNX_KNOBS=0" \
  "DS2_RNNX_KNOBS=$((2 << 17))" > $out/c5bf16.txt 2>&1
