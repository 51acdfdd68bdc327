#!/bin/bash
# Continuous validation: re-evaluates the latest checkpoint every eval_interval_secs
# (reference: src/validation.sh:40, deepSpeech_test.py --eval_data val, loop forever).
set -e
source "$(dirname "$0")/_common.sh"
echo "-----------------------------------"
echo "Start validation"
nchw=${nchw:-True}
engine=${engine:-hip}
check_config
python ${repo_root}/deepSpeech_test.py --eval_data 'val' --nchw ${nchw} --engine ${engine} \
  --checkpoint_dir ${checkpoint_dir:-../models/librispeech/train} --data_dir ${data_dir:-../data/LibriSpeech/processed/} ${extra_args}
echo "Done"
