#!/bin/bash
# BPTT pre-gather sleep (knob bits 20-22) and forward pre-poll sleep (bits 17-19) on the
# headline bench, same box, alternating. Logs: gpurun_out/r6_presleep2/
set -o pipefail
mkdir -p gpurun_out/r6_presleep2
F3=393216; F4=524288; F5=655360
B2=2097152; B4=4194304; B6=6291456
BENCH_ARGS='--no_infer --no_walk' bash scripts/ab_env.sh 3 "DS2_RNNX_KNOBS=$F4" "DS2_RNNX_KNOBS=$F3" "DS2_RNNX_KNOBS=$F5" \
  "DS2_RNNX_KNOBS=$((F4 + B2))" "DS2_RNNX_KNOBS=$((F4 + B4))" "DS2_RNNX_KNOBS=$((F4 + B6))" > gpurun_out/r6_presleep2/ab.txt 2>&1
