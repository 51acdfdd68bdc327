#!/bin/bash
# DP machinery at world 1 (--force_dp): which late round-6 change moved it (production binary,
# conv2 wgrad side stream on / off, explicit no poll sleep). Logs: gpurun_out/r6_dpcheck/
set -o pipefail
out=gpurun_out/r6_dpcheck
mkdir -p $out
X=8388608
E="DS2_EXT_SO=ab/_C_nodrain.cpython-310-x86_64-linux-gnu.so DS2_RNNX_KNOBS=$X DS2_CONV_WSIDE=0"
BENCH_ARGS="--force_dp --no_infer --no_walk" STEPS=20 bash scripts/ab_env.sh 2 "$E" "DS2_CONV_WSIDE=0" "DS2_RNNX_KNOBS=$X" "DS2_CONV_WSIDE=1" > $out/ab.txt 2>&1
