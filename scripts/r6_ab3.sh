#!/bin/bash
# Headline, same box: production (ab/_C_nodrain, no sleeps, conv2 wgrad in line) vs the in-tree
# defaults (forward sleep 4, BPTT sleep 2, conv2 wgrad side stream) and two neighbours.
set -o pipefail
out=gpurun_out/r6_ab3
mkdir -p $out
X=8388608
E="DS2_EXT_SO=ab/_C_nodrain.cpython-310-x86_64-linux-gnu.so DS2_RNNX_KNOBS=$X DS2_CONV_WSIDE=0"
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 4 "$E" "DS2_RNNX_KNOBS=0" "DS2_RNNX_KNOBS=$((X + (4 << 17)))" \
  "DS2_RNNX_KNOBS=$((X + (5 << 17) + (2 << 20)))" > $out/ab.txt 2>&1
