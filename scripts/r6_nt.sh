#!/bin/bash
# Round 6: nt vs default cache policy of the column GEMMs per configuration (same box, 2 rounds).
set -o pipefail
out=gpurun_out/r6_nt
mkdir -p $out
for cfg in "" "--cell rnn_relu --num_hidden 1760 --num_rnn_layers 7" "--num_hidden 1280 --num_rnn_layers 7 --fp8"; do
  BENCH_ARGS="--no_infer --no_walk --steps 20 --warmup 5 $cfg" timeout -k 10 600 bash scripts/ab_so.sh 2 dflt > $out/ab.log 2>&1 || exit 1
  grep -o '"variant": "[a-z]*", "round": [0-9]*\|"ms_per_step": [0-9.]*' $out/ab.log | paste - - | sed "s/^/[$cfg] /" | tee -a $out/ab.txt
done
