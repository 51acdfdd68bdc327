#!/bin/bash
# RCCL capture probe (HIP graphs of all_reduce at world 1), then host / wall time per step at the
# short SortaGrad lengths: single device eager / graph, --force_dp eager.
set -o pipefail
out=gpurun_out/r6_dpgraph
mkdir -p $out
timeout -k 10 400 python tools/probe_rccl_graph.py > $out/probe.txt 2>&1; cat $out/probe.txt
for v in "" "--graph" "--force_dp"; do
  echo "== ${v:-eager}" | tee -a $out/host.md
  timeout -k 10 240 python tools/host_overhead.py --steps 30 --frames 100,200,400,1000 $v 2>&1 | grep -v "amdgpu.ids\|socket.cpp" | tee -a $out/host.md || exit 1
done
