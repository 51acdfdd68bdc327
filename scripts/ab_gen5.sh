#!/bin/bash
# A/B of the generation-5 GRU forward (K-eighths) against generation 4 (DS2_RNNX_KNOBS bit 22)
K=4194304
bash scripts/gpu_job.sh "t:240:python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "ab:200:python tools/bench_rnn.py --cell gru --H 800 --kernels xcd --knobs 0,$K,0,$K --iters 10 --stamps" \
  "h1:120:python bench.py --steps 30 --warmup 5" "h2:120:env DS2_RNNX_KNOBS=$K python bench.py --steps 30 --warmup 5" \
  "h3:120:python bench.py --steps 30 --warmup 5" "h4:120:env DS2_RNNX_KNOBS=$K python bench.py --steps 30 --warmup 5"
