#!/bin/bash
# Beside-BPTT GEMMs leave 2 idle CUs per XCD on one device (headline and config 5 fp8): GPU tests
# and benches. Logs: gpurun_out/r6_beside4/
set -o pipefail
out=gpurun_out/r6_beside4
mkdir -p $out
timeout -k 10 800 python -u -m pytest tests/test_trajectory_production_gpu.py tests/test_engine_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for cfg in "" "--num_hidden 1280 --num_rnn_layers 7 --fp8"; do
  for r in 1 2; do
    o=$(timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_infer --no_walk $cfg | tail -1) || exit 1
    echo "[$cfg] $(echo "$o" | grep -o '"ms_per_step": [0-9.]*')" | tee -a $out/configs.txt
  done
done
