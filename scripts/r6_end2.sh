#!/bin/bash
# Round-6 end, part 2: headline kernel trace (timeline, per-step census) and the secondary
# configurations (config 5 bf16 / fp8, ReLU-1760, DP machinery at world 1), same box.
set -o pipefail
out=gpurun_out/r6_end
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 8 -- python3 bench.py --steps 5 --warmup 3 --no_infer --no_walk > $out/prof.log 2>&1 || exit 1
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 5 --phases > $out/timeline.txt 2>&1 || exit 1
python3 tools/step_kernels.py $db > $out/step_kernels.md 2>&1 || exit 1
grep "step period" $out/timeline.txt
for cfg in "--num_hidden 1280 --num_rnn_layers 7" "--num_hidden 1280 --num_rnn_layers 7 --fp8" \
           "--cell rnn_relu --num_hidden 1760 --num_rnn_layers 7" "--force_dp" ""; do
  for r in 1 2; do
    o=$(timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_infer --no_walk $cfg | tail -1) || exit 1
    echo "[$cfg] $(echo "$o" | grep -o '"ms_per_step": [0-9.]*')" | tee -a $out/configs.txt
  done
done
