#!/bin/bash
# Config 5 fp8 (7 x BiGRU-1280, fp8 recurrences): pre-poll sleeps of the fp8 forward / BPTT
# (compile-time variants, build.py --variant f8f2|f8f4|f8b2) against the in-tree build.
set -o pipefail
out=gpurun_out/r6_f8sleep
mkdir -p $out
ext=$(python -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
BENCH_ARGS="--num_hidden 1280 --num_rnn_layers 7 --fp8 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 3 "DS2_RNNX_KNOBS=0" \
  "DS2_EXT_SO=ab/_C_f8f2$ext" "DS2_EXT_SO=ab/_C_f8f4$ext" "DS2_EXT_SO=ab/_C_f8b2$ext" > $out/ab.txt 2>&1
# forward phase stamps of MFMA waves 0 (SIMD 0, beside the memory wave), 1 and 3
for w in 0 1 3; do
  DS2_RNNX_KNOBS=$((w << 24)) timeout -k 10 200 python tools/bench_rnn.py --kernels xcd --iters 3 --stamps > $out/stamps_w$w.txt 2>&1 || exit 1
done
