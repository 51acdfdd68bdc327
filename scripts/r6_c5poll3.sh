#!/bin/bash
# Config 5 bf16: rnnq pre-poll sleep in s_sleep 4 units (F = 4..7) and BPTT pre-gather sleeps
# (B, s_sleep 1 units) against production. Logs: gpurun_out/r6_c5poll3/
set -o pipefail
out=gpurun_out/r6_c5poll3
mkdir -p $out
X=8388608
E="DS2_EXT_SO=ab/_C_nodrain.cpython-310-x86_64-linux-gnu.so DS2_RNNX_KNOBS=$X"
BENCH_ARGS="--num_hidden 1280 --num_rnn_layers 7 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "$E" \
  "DS2_RNNX_KNOBS=$((X + (4 << 17)))" "DS2_RNNX_KNOBS=$((X + (5 << 17)))" "DS2_RNNX_KNOBS=$((X + (7 << 17)))" \
  "DS2_RNNX_KNOBS=$((X + (5 << 17) + (4 << 20)))" "DS2_RNNX_KNOBS=$((X + (5 << 17) + (7 << 20)))" > $out/ab.txt 2>&1
