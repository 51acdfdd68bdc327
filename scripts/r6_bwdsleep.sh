#!/bin/bash
# BPTT pre-gather sleep (knob bits 20-22, explicit bit 23) in the recurrence microbenchmark,
# one process, 3 passes. Logs: gpurun_out/r6_bwdsleep/
set -o pipefail
out=gpurun_out/r6_bwdsleep
mkdir -p $out
X=8388608; F=$((4 << 17))
K="$((X + F)),$((X + F + (1 << 20))),$((X + F + (2 << 20))),$((X + F + (3 << 20))),$((X + F + (4 << 20))),$((X + F + (6 << 20)))"
for r in 1 2 3; do
  timeout -k 10 240 python tools/bench_rnn.py --kernels xcd --iters 40 --knobs $K >> $out/rnn.log 2>&1 || exit 1
done
