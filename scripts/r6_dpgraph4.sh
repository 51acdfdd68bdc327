#!/bin/bash
# After: no residency gates under capture, DP carry only for >= 200 recurrence steps, one ready
# event per gradient report. DP tests, short-length host / wall times, world-1 DP overhead A/B.
set -o pipefail
out=gpurun_out/r6_dpgraph4
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dp_ready_gpu.py \
  tests/test_dp_gpu.py tests/test_step_graphs_gpu.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for v in "--graph" "--force_dp" "--force_dp --graph"; do
  echo "== $v" | tee -a $out/host.md
  timeout -k 10 240 python tools/host_overhead.py --steps 30 --frames 100,200,400,1000 $v 2>&1 | grep -v "amdgpu.ids\|socket.cpp\|version\|Hostname\|Librccl" | tee -a $out/host.md || exit 1
done
bash scripts/ab_dp.sh 2 2>&1 | grep -v "amdgpu.ids\|socket.cpp" | tee $out/dp.txt
