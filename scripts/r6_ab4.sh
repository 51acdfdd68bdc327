#!/bin/bash
# Headline: BPTT pre-gather sleep 2 (default) vs 3 vs 4 (forward sleep 4). Logs: gpurun_out/r6_ab4/
set -o pipefail
out=gpurun_out/r6_ab4
mkdir -p $out
X=8388608; F=$((4 << 17))
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 4 "DS2_RNNX_KNOBS=0" "DS2_RNNX_KNOBS=$((X + F + (3 << 20)))" \
  "DS2_RNNX_KNOBS=$((X + F + (4 << 20)))" > $out/ab.txt 2>&1
