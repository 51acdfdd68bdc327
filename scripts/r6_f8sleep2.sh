#!/bin/bash
# Config 5 fp8: BPTT pre-gather sleep 1 / 2 / 3 / 4 (compile-time variants) against none.
set -o pipefail
out=gpurun_out/r6_f8sleep2
mkdir -p $out
ext=$(python -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
BENCH_ARGS="--num_hidden 1280 --num_rnn_layers 7 --fp8 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 3 "DS2_RNNX_KNOBS=0" \
  "DS2_EXT_SO=ab/_C_f8b1$ext" "DS2_EXT_SO=ab/_C_f8b2$ext" "DS2_EXT_SO=ab/_C_f8b3$ext" "DS2_EXT_SO=ab/_C_f8b4$ext" > $out/ab.txt 2>&1
