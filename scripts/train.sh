#!/bin/bash
# Headline training launch (reference: src/train.sh:42 — batch 32, no-shuffle first epoch,
# 40k steps, lr 1e-4, 32 conv filters). Set gpus=N for data parallel over N GPUs of this
# node (torchrun, one process per GPU, RCCL over xGMI). restarts=K makes the job elastic:
# torchrun relaunches all ranks up to K times after a failure and they resume from the
# latest checkpoint in train_dir (deepspeech_amd/train.py resume_dir); every attempt builds
# its process group under its own store prefix (deepspeech_amd/parallel/dist.py).
set -e
source "$(dirname "$0")/_common.sh"
echo "-----------------------------------"
echo "Start training"
dummy=${dummy:-False}     # True or False
nchw=${nchw:-True}        # True or False
debug=${debug:-False}     # True or False
engine=${engine:-hip}     # hip, ref (tf, mkl, cudnn_rnn, mkldnn_rnn are aliases)
cell=${cell:-gru}         # gru (north-star) or rnn_relu (reference cell)
layers=${layers:-7}
hidden=${hidden:-1760}
gpus=${gpus:-1}
check_config
filename=${train_dir:-../models/librispeech/train}
datadir=${data_dir:-../data/LibriSpeech/processed/}
args="--batch_size 32 --no-shuffle --max_steps 40000 --num_rnn_layers ${layers} --num_hidden ${hidden}
      --num_filters 32 --initial_lr 1e-4 --temporal_stride 4 --train_dir ${filename} --data_dir ${datadir}
      --debug ${debug} --nchw ${nchw} --engine ${engine} --dummy ${dummy} --cell ${cell} ${extra_args}"
if [ "${gpus}" -gt 1 ] && [ "${restarts:-0}" -gt 0 ]; then
  python -m torch.distributed.run --nnodes=1 --nproc-per-node ${gpus} --max-restarts ${restarts} \
    --rdzv-backend c10d --rdzv-endpoint 127.0.0.1:${port:-29511} ${repo_root}/deepSpeech_train.py ${args}
elif [ "${gpus}" -gt 1 ]; then
  python -m torch.distributed.run --nnodes=1 --nproc-per-node ${gpus} --master-addr 127.0.0.1 \
    --master-port ${port:-29511} ${repo_root}/deepSpeech_train.py ${args}
else
  python ${repo_root}/deepSpeech_train.py ${args}
fi
echo "Done"
