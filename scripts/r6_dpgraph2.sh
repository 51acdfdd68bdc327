#!/bin/bash
# RCCL capture probe variants, GPU beam search tests, and a kernel trace of the 100-frame DP step.
set -o pipefail
out=gpurun_out/r6_dpgraph2
mkdir -p $out
timeout -k 10 600 python tools/probe_rccl_graph.py > $out/probe.txt 2>&1; grep -v amdgpu.ids $out/probe.txt | grep "==\|ok\|captured\|Error\|error" 
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_beam_gpu.py > $out/beam_tests.log 2>&1 || { tail -40 $out/beam_tests.log; exit 1; }
tail -3 $out/beam_tests.log
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 0 -- python3 tools/host_overhead.py --steps 10 --frames 100 --force_dp > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 8 --phases > $out/timeline.txt 2>&1 || exit 1
python3 tools/step_kernels.py $db > $out/step_kernels.md 2>&1 || exit 1
grep "step period" $out/timeline.txt
timeout -k 10 200 python tools/bench_infer.py > $out/infer.txt 2>&1 || { tail -20 $out/infer.txt; exit 1; }
grep -v amdgpu.ids $out/infer.txt | tail -12
