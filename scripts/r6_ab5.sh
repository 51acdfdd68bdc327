#!/bin/bash
# Headline: forward pre-poll sleep 3 / 4 (default) / 5 / 6 with the BPTT sleep 4. Logs: gpurun_out/r6_ab5/
set -o pipefail
out=gpurun_out/r6_ab5
mkdir -p $out
X=8388608; B=$((4 << 20))
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 3 "DS2_RNNX_KNOBS=$((X + B + (3 << 17)))" "DS2_RNNX_KNOBS=0" \
  "DS2_RNNX_KNOBS=$((X + B + (5 << 17)))" "DS2_RNNX_KNOBS=$((X + B + (6 << 17)))" > $out/ab.txt 2>&1
