#!/bin/bash
# Reference training driver at the headline model (5 x BiGRU-800, batch 32, --dummy True: one
# SortaGrad dummy epoch, src/deepSpeech_dummy.py) with and without 10-step checkpoints
# (src/deepSpeech_train.py:354-356), alternating, ROUNDS rounds each. Prints each run's final
# throughput line. Output dir: ${OUT:-gpurun_out/ckpt_timing}.
set -e
ROUNDS=${ROUNDS:-2}
STEPS=${STEPS:-1020}
OUT=${OUT:-gpurun_out/ckpt_timing}
mkdir -p "${OUT}"
for r in $(seq 1 "${ROUNDS}"); do
  for every in 10 0; do
    d=/tmp/ds2_ckpt_${every}
    rm -rf "${d}"
    timeout -k 10 300 python3 deepSpeech_train.py --dummy True --batch_size 32 --num_rnn_layers 5 \
      --num_hidden 800 --cell gru --max_steps "${STEPS}" --checkpoint_every "${every}" --max_to_keep 3 \
      --train_dir "${d}" ${EXTRA} > "${OUT}/every${every}_r${r}.log" 2>&1
    echo "checkpoint_every=${every} round ${r}: $(grep -E 'audio-sec/sec' "${OUT}/every${every}_r${r}.log" | tail -n 1)"
    echo "  files: $(ls ${d} | grep -c 'model.ckpt.*index') checkpoints kept; $(grep -c 'skipping saves' "${OUT}/every${every}_r${r}.log" || true) stretches of saves skipped while the writer was busy"
    python3 -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if 'checkpoint_summary' in l]; print('  cadence:', r[-1] if r else 'no checkpoint written')" "${d}/metrics.jsonl"
  done
done
