#!/bin/bash
# Projection grid capped to the CUs a carried dU GEMM leaves: same-box A/B on the headline and
# config 5 bf16, then a headline kernel trace.
set -o pipefail
out=gpurun_out/r6_projgrid
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_defer_update_gpu.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for cfg in "" "--num_hidden 1280 --num_rnn_layers 7"; do
  for r in 1 2 3; do
    for a in "" "--no_proj_beside"; do
      o=$(timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no_infer --no_walk $cfg $a | tail -1) || exit 1
      echo "[$cfg] [${a:-default}] $(echo "$o" | grep -o '"ms_per_step": [0-9.]*')" | tee -a $out/ab.txt
    done
  done
done
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 8 -- python3 bench.py --steps 5 --warmup 3 --no_infer --no_walk > $out/prof.log 2>&1 || exit 1
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 5 --phases > $out/timeline.txt 2>&1 || exit 1
grep "step period" $out/timeline.txt
