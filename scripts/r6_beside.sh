#!/bin/bash
# Grid of the weight-gradient GEMMs beside a BPTT (the 56 idle CUs by default): 40 / 48.
set -o pipefail
out=gpurun_out/r6_beside
mkdir -p $out
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 3 "DS2_BESIDE_AB=-1" "DS2_BESIDE_AB=48" "DS2_BESIDE_AB=40" > $out/ab.txt 2>&1
