#!/bin/bash
# Forward polls of the MFMA tile's padding rows (rows >= R) as out-of-range (no memory request)
# loads (knob bit 28) vs re-reads of row R-1. Kernel tests with the knob first.
set -o pipefail
out=gpurun_out/r6_padl
mkdir -p $out
DS2_RNNX_KNOBS=268435456 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "birnn or bptt or unirnn or fused_direction" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 4 "DS2_RNNX_KNOBS=0" "DS2_RNNX_KNOBS=268435456" > $out/ab.txt 2>&1
