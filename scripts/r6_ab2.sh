#!/bin/bash
# Same box: production (ab/_C_nodrain, knobs explicit 0) vs the in-tree build (drained poll
# exits + pre-poll sleep 4, abort word read beside the partials, pairwise partial sums), and
# the in-tree build with conv2's weight gradient on its own stream. Kernel tests first, phase
# stamps of both builds last. Logs: gpurun_out/r6_ab2/
set -o pipefail
out=gpurun_out/r6_ab2
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "birnn or bptt or wide or unirnn or fused_direction" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
E="DS2_EXT_SO=ab/_C_nodrain.cpython-310-x86_64-linux-gnu.so DS2_RNNX_KNOBS=8388608"
BENCH_ARGS='--no_infer --no_walk' bash scripts/ab_env.sh 4 "$E" "DS2_RNNX_KNOBS=0" "DS2_CONV_WSIDE=1" > $out/ab.txt 2>&1 || exit 1
env $E timeout -k 10 200 python tools/bench_rnn.py --kernels xcd --iters 5 --stamps > $out/stamps_prod.txt 2>&1 || exit 1
timeout -k 10 200 python tools/bench_rnn.py --kernels xcd --iters 5 --stamps > $out/stamps_new.txt 2>&1
