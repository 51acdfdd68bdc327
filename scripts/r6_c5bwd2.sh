#!/bin/bash
# Wide-plan BPTT sleep default (12 units): recurrence tests, config 5 bf16 and headline benches.
set -o pipefail
out=gpurun_out/r6_c5bwd2
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "birnn or bptt or wide or unirnn or fused_direction" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
BENCH_ARGS="--num_hidden 1280 --num_rnn_layers 7 --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "DS2_RNNX_KNOBS=0" \
  "DS2_RNNX_KNOBS=$((8388608 + (5 << 17)))" > $out/ab.txt 2>&1 || exit 1
o=$(timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_infer --no_walk | tail -1) || exit 1
echo "[headline] $(echo "$o" | grep -o '"ms_per_step": [0-9.]*')" | tee -a $out/ab.txt
