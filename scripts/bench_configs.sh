#!/bin/bash
# Secondary benchmark configurations + their rocprof summaries (README table), one GPU call:
#   bash scripts/bench_configs.sh gpurun_out/configs
# config 5 (7 x BiGRU-1280, bf16 and fp8 projections) and the reference's own headline
# (7 x bi-RNN clipped-ReLU-1760, src/train.sh:42). Every step has its own time limit and the
# chain stops at the first failure.
set -o pipefail
out=${1:-gpurun_out/configs}
mkdir -p "$out"
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 180 python bench.py "$@" --steps 20 --warmup 5 --no_infer > "$out/$name.log" 2>&1; }
run c5_bf16 --num_hidden 1280 --num_rnn_layers 7 &&
run c5_fp8 --num_hidden 1280 --num_rnn_layers 7 --fp8 &&
run ref1760 --cell rnn_relu --num_hidden 1760 --num_rnn_layers 7 &&
timeout -k 10 240 bash scripts/rocprof.sh "$out/prof_1760" 8 -- python3 bench.py --cell rnn_relu --num_hidden 1760 \
  --num_rnn_layers 7 --steps 5 --warmup 3 --no_infer --no_walk > "$out/prof_1760.log" 2>&1 &&
timeout -k 10 240 bash scripts/rocprof.sh "$out/prof_c5" 8 -- python3 bench.py --num_hidden 1280 --num_rnn_layers 7 \
  --steps 5 --warmup 3 --no_infer --no_walk > "$out/prof_c5.log" 2>&1 &&
timeout -k 10 240 bash scripts/rocprof.sh "$out/prof_c5f8" 8 -- python3 bench.py --num_hidden 1280 --num_rnn_layers 7 \
  --fp8 --steps 5 --warmup 3 --no_infer --no_walk > "$out/prof_c5f8.log" 2>&1
