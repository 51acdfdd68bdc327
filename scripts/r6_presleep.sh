#!/bin/bash
# Recurrence forward poll timing: drained poll exits + a pre-poll sleep (knob bits 17-19,
# units of s_sleep 1) against the production build (ab/_C_nodrain), plus the retry back-off
# (nap, knob bits 12-13). Logs: gpurun_out/r6_presleep/
set -o pipefail
out=gpurun_out/r6_presleep
mkdir -p $out
ext=$(python -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
for r in 1 2; do
  (unset DS2_EXT_SO; timeout -k 10 200 python tools/bench_rnn.py --kernels xcd --iters 20 --knobs 0,131072,262144,393216,524288,786432 | sed "s/^/drain $r /") >> $out/rnn.log 2>&1 || exit 1
  (export DS2_EXT_SO=ab/_C_nodrain${ext}; timeout -k 10 200 python tools/bench_rnn.py --kernels xcd --iters 20 --knobs 0,4096,8192 | sed "s/^/nodrain $r /") >> $out/rnn.log 2>&1 || exit 1
done
