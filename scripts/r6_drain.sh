#!/bin/bash
# Same-box A/B: explicit vmcnt(0) at the recurrence poll's exits (in-tree _C) against the
# compiler's own waits (ab/_C_nodrain: build.py --variant nodrain -D DS2_NO_DRAIN).
# Logs: gpurun_out/r6_drain/
set -o pipefail
out=gpurun_out/r6_drain
mkdir -p $out
ext=$(python -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { echo "kernel tests failed"; tail -30 $out/tests.log; exit 1; }
for r in 1 2 3; do
  (unset DS2_EXT_SO; timeout -k 10 120 python tools/bench_rnn.py --kernels xcd --iters 20 | sed "s/^/base $r /") >> $out/rnn.log 2>&1 || exit 1
  (export DS2_EXT_SO=ab/_C_nodrain${ext}; timeout -k 10 120 python tools/bench_rnn.py --kernels xcd --iters 20 | sed "s/^/nodrain $r /") >> $out/rnn.log 2>&1 || exit 1
done
bash scripts/ab_so.sh 3 nodrain > $out/ab.txt 2>&1 || exit 1
