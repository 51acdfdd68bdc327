#!/bin/bash
# Block cap of the carried optimizer chunks / dU GEMMs beside the forward recurrences: 40 / 48 vs 56.
set -o pipefail
out=gpurun_out/r6_carry
mkdir -p $out
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 3 "DS2_CARRY_AB=0" "DS2_CARRY_AB=40" "DS2_CARRY_AB=48" > $out/ab.txt 2>&1
