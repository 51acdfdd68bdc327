#!/bin/bash
# --force_dp with the conv2 side stream switched off under a bucketer, and the single-device step.
set -o pipefail
out=gpurun_out/r6_dpcheck2
mkdir -p $out
BENCH_ARGS="--force_dp --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "DS2_CONV_WSIDE=1" > $out/dp.txt 2>&1 || exit 1
BENCH_ARGS="--no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "DS2_CONV_WSIDE=1" "DS2_CONV_WSIDE=0" > $out/single.txt 2>&1
