#!/bin/bash
# 100 / 200-frame steps through bench.py (RCCL world 1 for --force_dp): eager vs step graphs.
set -o pipefail
out=gpurun_out/r6_short
mkdir -p $out
for fr in 100 200; do
  for a in "" "--step_graphs" "--force_dp" "--force_dp --step_graphs"; do
    o=$(timeout -k 10 200 python bench.py --frames $fr --steps 50 --warmup 10 --no_infer --no_walk $a | tail -1) || exit 1
    echo "[frames $fr] [${a:-eager}] $(echo "$o" | grep -o '"ms_per_step": [0-9.]*')" | tee -a $out/short.txt
  done
done
