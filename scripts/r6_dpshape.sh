#!/bin/bash
# Why the DP step at 1000 frames is slower after shorter shapes ran (host_overhead --force_dp:
# 10.2 ms vs bench.py --force_dp 7.7): kernel trace of 400- then 1000-frame steps.
set -o pipefail
out=gpurun_out/r6_dpshape
mkdir -p $out
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 0 -- python3 tools/host_overhead.py --steps 10 --frames 400,1000 --force_dp > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
grep "^|" $out/prof.log
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 27 --phases > $out/timeline.txt 2>&1 || exit 1
grep "step period" $out/timeline.txt
grep wait_resident $out/timeline.txt | head -20
