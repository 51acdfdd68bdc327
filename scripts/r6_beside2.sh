#!/bin/bash
# Beside-BPTT GEMM grid 40 vs the default, headline (4 rounds) and the DP machinery (2 rounds).
set -o pipefail
out=gpurun_out/r6_beside2
mkdir -p $out
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 4 "DS2_BESIDE_AB=-1" "DS2_BESIDE_AB=40" "DS2_BESIDE_AB=32" > $out/ab.txt 2>&1 || exit 1
BENCH_ARGS="--force_dp --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "DS2_BESIDE_AB=-1" "DS2_BESIDE_AB=40" > $out/dp.txt 2>&1
