#!/bin/bash
# DP step graphs (blocking collectives under capture) bitwise test, GPU beam search tests, short
# lengths host / wall time (single device and --force_dp, eager and graph), kernel trace of the
# 100-frame DP step, streaming RTF with the GPU beam search.
set -o pipefail
out=gpurun_out/r6_dpgraph3
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_beam_gpu.py \
  tests/test_dp_ready_gpu.py -k "beam or graphs" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for v in "--force_dp" "--force_dp --graph"; do
  echo "== $v" | tee -a $out/host.md
  timeout -k 10 240 python tools/host_overhead.py --steps 30 --frames 100,200,400,1000 $v 2>&1 | grep -v "amdgpu.ids\|socket.cpp\|version\|Hostname\|Librccl" | tee -a $out/host.md || exit 1
done
timeout -k 10 200 python tools/host_overhead.py --steps 20 --frames 100 --force_dp --cprofile 30 > $out/cprofile.txt 2>&1 || exit 1
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 0 -- python3 tools/host_overhead.py --steps 10 --frames 100 --force_dp > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 8 --phases > $out/timeline.txt 2>&1 || exit 1
grep "step period" $out/timeline.txt
timeout -k 10 200 python tools/bench_infer.py > $out/infer.txt 2>&1 || { tail -20 $out/infer.txt; exit 1; }
grep -v amdgpu.ids $out/infer.txt | tail -12
