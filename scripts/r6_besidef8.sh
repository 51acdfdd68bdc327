#!/bin/bash
# Config 5 fp8: weight-gradient GEMMs beside the fp8 BPTT on 64 / 80 of the 96 idle CUs vs all.
set -o pipefail
out=gpurun_out/r6_besidef8
mkdir -p $out
BENCH_ARGS="--num_hidden 1280 --num_rnn_layers 7 --fp8 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "DS2_BESIDE_F8_AB=0" \
  "DS2_BESIDE_F8_AB=80" "DS2_BESIDE_F8_AB=64" > $out/ab.txt 2>&1
