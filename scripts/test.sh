#!/bin/bash
# One-shot evaluation on the test partition with the EMA weights (reference: src/test.sh:39).
set -e
source "$(dirname "$0")/_common.sh"
echo "-----------------------------------"
echo "Start testing"
nchw=${nchw:-True}
engine=${engine:-hip}
check_config
python ${repo_root}/deepSpeech_test.py --eval_data 'test' --nchw ${nchw} --engine ${engine} --run_once True \
  --checkpoint_dir ${checkpoint_dir:-../models/librispeech/train} --data_dir ${data_dir:-../data/LibriSpeech/processed/} ${extra_args}
echo "Done"
