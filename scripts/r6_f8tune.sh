#!/bin/bash
# Config 5 fp8: beside grid 72 / 88 vs 80 (default), fp8 BPTT sleep 5 (variant) vs 3.
set -o pipefail
out=gpurun_out/r6_f8tune
mkdir -p $out
ext=$(python -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
BENCH_ARGS="--num_hidden 1280 --num_rnn_layers 7 --fp8 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "DS2_BESIDE_F8_AB=0" \
  "DS2_BESIDE_F8_AB=72" "DS2_BESIDE_F8_AB=88" "DS2_EXT_SO=ab/_C_f8b5$ext" > $out/ab.txt 2>&1
