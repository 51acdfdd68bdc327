#!/bin/bash
# Same-box A/B of the GEMM routing: DS2_GEMM=hip (every GEMM hand-written: gemm.hip TUNED
# projections + gemm8) vs DS2_GEMM=proj (round-2 routing: dx / weight gradients on hipBLASLt),
# alternating, for the headline, config 5 (bf16 and fp8) and the reference's 7 x bi-ReLU-1760.
#   scripts/ab_gemm8.sh [rounds]
set -o pipefail
out=gpurun_out/ab_gemm8; mkdir -p $out
rounds=${1:-2}
run() {  # name env args...
  local name=$1 env=$2; shift 2
  env $env timeout -k 10 240 python bench.py "$@" > $out/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $out/$name.log; exit 1; }
  echo "$name $(tail -1 $out/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for r in $(seq 1 $rounds); do
  run head_hip_$r DS2_GEMM=hip
  run head_proj_$r DS2_GEMM=proj
done
for r in $(seq 1 $rounds); do
  run c5fp8_hip_$r DS2_GEMM=hip --num_hidden 1280 --num_rnn_layers 7 --fp8
  run c5fp8_proj_$r DS2_GEMM=proj --num_hidden 1280 --num_rnn_layers 7 --fp8
  run c5_hip_$r DS2_GEMM=hip --num_hidden 1280 --num_rnn_layers 7
  run c5_proj_$r DS2_GEMM=proj --num_hidden 1280 --num_rnn_layers 7
  run relu_hip_$r DS2_GEMM=hip --num_hidden 1760 --num_rnn_layers 7 --cell rnn_relu
  run relu_proj_$r DS2_GEMM=proj --num_hidden 1760 --num_rnn_layers 7 --cell rnn_relu
done
