#!/bin/bash
# Round 6: the upper layers' dU GEMMs carried into the next forward. Bitwise tests, same-box A/B
# (carry_du / no carry_du / no carried update at all), profile + timeline + per-step census.
set -o pipefail
out=gpurun_out/r6_carrydu
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_defer_update_gpu.py tests/test_engine_gpu.py tests/test_dp_ready_gpu.py \
  tests/test_reduce_gpu.py tests/test_step_graphs_gpu.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for r in 1 2 3; do
  for a in "" "--carry_blocks 1" "--carry_blocks 2" "--no_carry_du"; do
    o=$(timeout -k 10 150 python bench.py --steps 30 --warmup 10 --no_infer --no_walk $a | tail -1) || exit 1
    echo "[${a:-default}] $(echo "$o" | grep -o '"ms_per_step": [0-9.]*')" | tee -a $out/ab.txt
  done
done
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 8 -- python3 bench.py --steps 5 --warmup 3 --no_infer --no_walk > $out/prof.log 2>&1 || exit 1
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 5 --phases > $out/timeline.txt 2>&1 || exit 1
python3 tools/step_kernels.py $db > $out/step_kernels.md 2>&1 || exit 1
grep "step period" $out/timeline.txt
timeout -k 10 200 python tools/glue_ops.py > $out/glue.txt 2>&1 || exit 1
