#!/bin/bash
# ReLU poll default (forward 2, BPTT 4): wide-kernel tests and the ReLU-1760 bench.
set -o pipefail
out=gpurun_out/r6_relu3
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "birnn or bptt or wide or unirnn" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
BENCH_ARGS="--cell rnn_relu --num_hidden 1760 --num_rnn_layers 7 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "DS2_RNNX_KNOBS=0" \
  "DS2_RNNX_KNOBS=$((8388608 + (4 << 20) + (4 << 17)))" > $out/ab.txt 2>&1
