#!/bin/bash
# A/B of the fp8 GRU forward generations (DS2_RNNX_KNOBS bit 23 = generation 1) at config 5
K=8388608
bash scripts/gpu_job.sh "t:240:python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k fp8" \
  "f1:120:python bench.py --num_hidden 1280 --num_rnn_layers 7 --steps 15 --warmup 5 --fp8" \
  "f2:120:env DS2_RNNX_KNOBS=$K python bench.py --num_hidden 1280 --num_rnn_layers 7 --steps 15 --warmup 5 --fp8" \
  "f3:120:python bench.py --num_hidden 1280 --num_rnn_layers 7 --steps 15 --warmup 5 --fp8" \
  "f4:120:env DS2_RNNX_KNOBS=$K python bench.py --num_hidden 1280 --num_rnn_layers 7 --steps 15 --warmup 5 --fp8" \
  "p:200:bash scripts/rocprof.sh gpurun_out/prof_f8 8 -- python3 bench.py --num_hidden 1280 --num_rnn_layers 7 --steps 5 --warmup 3 --fp8"
