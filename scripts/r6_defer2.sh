#!/bin/bash
# Round 6: carried optimizer update spread one chunk per recurrence; torch-glue reductions in
# csrc/reduce.hip; GPU checkpoint tests with the TF-bundle format; A/B vs the in-step update;
# profile; torch glue left in the step; checkpoint cadence in the driver.
set -o pipefail
out=gpurun_out/r6_defer2
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_reduce_gpu.py \
  tests/test_defer_update_gpu.py tests/test_checkpoint_gpu.py tests/test_step_graphs_gpu.py \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -5 $out/tests.log
for r in 1 2 3; do
  for a in "" "--no_defer_update"; do
    o=$(timeout -k 10 150 python bench.py --steps 30 --warmup 10 --no_infer --no_walk $a | tail -1) || exit 1
    echo "defer${a:+ off} $(echo "$o" | grep -o '"ms_per_step": [0-9.]*')" | tee -a $out/ab.txt
  done
done
BENCH_ARGS="--no_infer --no_walk" timeout -k 10 400 bash scripts/ab_so.sh 3 nt > $out/ab_nt.log 2>&1 || exit 1
grep -o '"variant": "[a-z]*", "round": [0-9]*\|"ms_per_step": [0-9.]*' $out/ab_nt.log | paste - - | tee $out/ab_nt.txt
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 8 -- python3 bench.py --steps 5 --warmup 3 --no_infer --no_walk > $out/prof.log 2>&1 || exit 1
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 5 --phases > $out/timeline.txt 2>&1 || exit 1
head -24 $out/timeline.txt
grep "step period" $out/timeline.txt
timeout -k 10 200 python tools/glue_ops.py > $out/glue.txt 2>&1 || exit 1
head -60 $out/glue.txt
ROUNDS=1 STEPS=1020 OUT=$out/ckpt timeout -k 10 700 bash scripts/ckpt_timing.sh 2>&1 | tee $out/ckpt.txt
