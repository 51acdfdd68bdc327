#!/bin/bash
# Round 6: checkpoint cadence with sharded TF bundles (reference driver, dummy epoch, headline
# model), and the data-parallel machinery's cost at world size 1 (plain vs --force_dp).
set -o pipefail
out=gpurun_out/r6_ckpt_dp
mkdir -p $out
bash scripts/ab_dp.sh 2 > $out/dp.txt 2>&1 || exit 1
cat $out/dp.txt
ROUNDS=1 STEPS=1020 OUT=$out/ckpt timeout -k 10 700 bash scripts/ckpt_timing.sh 2>&1 | tee $out/ckpt.txt
# the headline shape alone (fixed 1000-frame batches) with 10-step checkpoints vs none
for every in 10 0; do
  d=/tmp/ds2_ckpt_h${every}; rm -rf $d
  timeout -k 10 300 python3 -m deepspeech_amd.train --dummy True --batch_size 32 --num_rnn_layers 5 --num_hidden 800 \
    --cell gru --max_steps 300 --checkpoint_every $every --max_to_keep 3 --train_dir $d --dummy_frames 1000 \
    > $out/headline_every$every.log 2>&1 || { tail -20 $out/headline_every$every.log; exit 1; }
  echo "headline checkpoint_every=$every: $(grep -E 'audio-sec/sec' $out/headline_every$every.log | tail -n 1)"
  python3 -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if 'checkpoint_summary' in l]; print('  cadence:', r[-1] if r else 'none')" $d/metrics.jsonl
done
