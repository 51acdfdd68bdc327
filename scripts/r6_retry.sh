#!/bin/bash
# Retry back-off of the polls: forward nap 1 / 2 (knob bits 12-13), BPTT gather +1 / +2 s_sleep 1
# per retry (bits 29-30), with the default pre-poll sleeps. Logs: gpurun_out/r6_retry/
set -o pipefail
out=gpurun_out/r6_retry
mkdir -p $out
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 3 "DS2_RNNX_KNOBS=0" "DS2_RNNX_KNOBS=4096" "DS2_RNNX_KNOBS=8192" \
  "DS2_RNNX_KNOBS=$((1 << 29))" "DS2_RNNX_KNOBS=$((2 << 29))" > $out/ab.txt 2>&1
