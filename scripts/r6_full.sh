#!/bin/bash
# Round 6: the whole GPU suite, the torch ops left in a headline step, and the driver bench.
set -o pipefail
out=gpurun_out/r6_full
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 200 python tools/glue_ops.py > $out/glue.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/glue.txt | head -80
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || exit 1
tail -1 $out/bench.json
