#!/bin/bash
# conv front-end kernels: tests, per-tile phase timeline, kernel-trace summary of tools/bench_conv.py
set -o pipefail
export TMPDIR=/tmp
out=${1:-gpurun_out/conv}
mkdir -p $out
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 120 python3 tools/conv_timeline.py > $out/timeline.log 2>&1 || { tail $out/timeline.log; exit 1; }
grep kernel $out/timeline.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 tools/bench_conv.py --iters 5 > $out/trace.log 2>&1 || { tail $out/trace.log; exit 1; }
python3 tools/rocpd_summary.py $out/trace/run_results.db -o $out/kernels.md > /dev/null && head -16 $out/kernels.md
