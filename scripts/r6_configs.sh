#!/bin/bash
# Round 6: the headline and the secondary configurations (BASELINE config 5 bf16 / fp8, the
# reference's 7 x bi-ReLU-1760) with the carried update + carried dU against without (same box,
# alternating, 2 rounds).
set -o pipefail
out=gpurun_out/r6_configs
mkdir -p $out
for cfg in "" "--num_hidden 1280 --num_rnn_layers 7" "--num_hidden 1280 --num_rnn_layers 7 --fp8" \
           "--cell rnn_relu --num_hidden 1760 --num_rnn_layers 7"; do
  for r in 1 2; do
    for a in "" "--no_carry_du" "--no_defer_update"; do
      o=$(timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_infer --no_walk $cfg $a | tail -1) || exit 1
      echo "[$cfg] [${a:-default}] $(echo "$o" | grep -o '"ms_per_step": [0-9.]*')" | tee -a $out/ab2.txt
    done
  done
done
