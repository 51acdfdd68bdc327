#!/bin/bash
# conv2 wgrad side stream with torch events: --force_dp (where the cached-event version ran
# 9.4 ms/step) and single device, same box. DS2_CONV_WSIDE=1 also needs the bucketer guard off
# for the DP arm: DS2_CONV_WSIDE_DP=1 (A/B only).
set -o pipefail
out=gpurun_out/r6_sidecheck
mkdir -p $out
BENCH_ARGS="--force_dp --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "DS2_CONV_WSIDE=0" "DS2_CONV_WSIDE=1 DS2_CONV_WSIDE_DP=1" > $out/dp.txt 2>&1 || exit 1
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 3 "DS2_CONV_WSIDE=0" "DS2_CONV_WSIDE=1" > $out/single.txt 2>&1
