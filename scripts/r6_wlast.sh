#!/bin/bash
# conv2's weight gradient after the dgrad -> BN1 -> conv1-wgrad chain (same stream) vs before.
set -o pipefail
out=gpurun_out/r6_wlast
mkdir -p $out
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 4 "DS2_CONV_WLAST=0" "DS2_CONV_WLAST=1" > $out/ab.txt 2>&1 || exit 1
BENCH_ARGS="--force_dp --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 1 "DS2_CONV_WLAST=0" "DS2_CONV_WLAST=1" > $out/dp.txt 2>&1
