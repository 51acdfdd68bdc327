#!/bin/bash
# Round-6 final (late session): GPU suite, smoke, the driver bench twice, secondary configs and
# the DP machinery at world 1, one box. Logs: gpurun_out/r6_final5/
set -o pipefail
out=gpurun_out/r6_final5
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
for r in 1 2; do
  timeout -k 10 300 python bench.py > $out/bench$r.json 2> $out/bench$r.err || { tail -20 $out/bench$r.err; exit 1; }
  tail -1 $out/bench$r.json | cut -c1-220
done
for cfg in "--num_hidden 1280 --num_rnn_layers 7" "--num_hidden 1280 --num_rnn_layers 7 --fp8" \
           "--cell rnn_relu --num_hidden 1760 --num_rnn_layers 7" "--force_dp"; do
  o=$(timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_infer --no_walk $cfg | tail -1) || exit 1
  echo "[$cfg] $(echo "$o" | grep -o '"ms_per_step": [0-9.]*')" | tee -a $out/configs.txt
done
