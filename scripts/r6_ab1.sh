#!/bin/bash
# Same box: production build (ab/_C_nodrain, no pre-poll sleep) vs drained poll exits + forward
# pre-poll sleep 4 (the new default), + conv2 weight gradient on its own stream, + BPTT
# pre-gather sleep 2; then phase stamps of both builds. Logs: gpurun_out/r6_ab1/
set -o pipefail
mkdir -p gpurun_out/r6_ab1
E="DS2_EXT_SO=ab/_C_nodrain.cpython-310-x86_64-linux-gnu.so DS2_RNNX_KNOBS=8388608"
F4=524288; B2=2097152
BENCH_ARGS='--no_infer --no_walk' bash scripts/ab_env.sh 4 "$E" "DS2_RNNX_KNOBS=0" "DS2_CONV_WSIDE=1" \
  "DS2_RNNX_KNOBS=$((F4 + B2))" > gpurun_out/r6_ab1/ab.txt 2>&1 || exit 1
env $E timeout -k 10 200 python tools/bench_rnn.py --kernels xcd --iters 5 --stamps > gpurun_out/r6_ab1/stamps_prod.txt 2>&1 || exit 1
timeout -k 10 200 python tools/bench_rnn.py --kernels xcd --iters 5 --stamps > gpurun_out/r6_ab1/stamps_f4.txt 2>&1
