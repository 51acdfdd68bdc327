#!/bin/bash
# Streaming inference RTF (5 x uni-GRU-800, 0.5 s chunks, greedy) under poll timings: default
# (forward sleep 4), explicit no sleep, forward sleep 2. Logs: gpurun_out/r6_infer_poll/
set -o pipefail
out=gpurun_out/r6_infer_poll
mkdir -p $out
for r in 1 2; do
  for k in 0 8388608 $((8388608 + (2 << 17))); do
    echo "knobs $k round $r" >> $out/rtf.txt
    DS2_RNNX_KNOBS=$k timeout -k 10 200 python tools/bench_infer.py --chunks 0.5 --decoders greedy --seconds 10 >> $out/rtf.txt 2>&1 || exit 1
  done
done
