#!/bin/bash
# Round-6 end: the whole GPU suite, smoke, the driver bench twice, a headline kernel trace with
# its timeline and per-step census, and the secondary configurations (same box).
set -o pipefail
out=gpurun_out/r6_final
mkdir -p $out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
for r in 1 2; do
  timeout -k 10 300 python bench.py > $out/bench$r.json 2> $out/bench$r.err || { tail -20 $out/bench$r.err; exit 1; }
  tail -1 $out/bench$r.json
done
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 8 -- python3 bench.py --steps 5 --warmup 3 --no_infer --no_walk > $out/prof.log 2>&1 || exit 1
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 5 --phases > $out/timeline.txt 2>&1 || exit 1
python3 tools/step_kernels.py $db > $out/step_kernels.md 2>&1 || exit 1
grep "step period" $out/timeline.txt
for cfg in "--num_hidden 1280 --num_rnn_layers 7" "--num_hidden 1280 --num_rnn_layers 7 --fp8" \
           "--cell rnn_relu --num_hidden 1760 --num_rnn_layers 7" "--force_dp"; do
  for r in 1 2; do
    o=$(timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_infer --no_walk $cfg | tail -1) || exit 1
    echo "[$cfg] $(echo "$o" | grep -o '"ms_per_step": [0-9.]*')" | tee -a $out/configs.txt
  done
done
