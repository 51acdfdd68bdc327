#!/bin/bash
# GPU check of the recurrence family map and the fp8 direction-pair hand-over, then a same-box
# A/B of config 5 fp8 with and without the pairs (DS2_FP8_PAIRS), arms alternated.
set -o pipefail
out=gpurun_out/pairs
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -s \
  tests/test_kernels_gpu.py -k "quant2" > $out/quant.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -s \
  tests/test_engine_gpu.py -k "direction_pairs or fp8_recurrence_model or same_upstream" > $out/engine.log 2>&1 || exit 1
for r in 1 2; do
  for arm in 1 0; do
    DS2_FP8_PAIRS=$arm timeout -k 10 200 python -u bench.py --num_hidden 1280 --num_rnn_layers 7 --fp8 --no_walk \
      --no_infer --steps 20 --warmup 5 > $out/c5f8_${arm}_$r.log 2>&1 || exit 1
    echo "pairs=$arm round $r: $(tail -1 $out/c5f8_${arm}_$r.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])') ms/step" >> $out/ab.txt
  done
done
