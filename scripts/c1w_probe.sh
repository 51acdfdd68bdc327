#!/bin/bash
# conv1 weight-gradient kernel alone (tools/bench_conv.py under rocprofv3 --stats) at 1 and 2
# workgroups per CU; then the headline step alternated over DS2_C1W_BPC and DS2_GROUP_BEFORE_DX.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/c1w
mkdir -p $out
for b in 1 2; do
  DS2_C1W_BPC=$b timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/p$b -o run -- python3 tools/bench_conv.py --iters 10 > $out/p$b.log 2>&1 || exit 1
  python3 tools/rocpd_summary.py $out/p$b/run_results.db -o $out/p$b.md > /dev/null 2>&1 || true
done
for r in 1 2 3; do
  for arm in "DS2_C1W_BPC=1" "DS2_C1W_BPC=2" "DS2_GROUP_BEFORE_DX=0"; do
    env $arm timeout -k 10 150 python bench.py --no_walk --no_infer --steps 30 --warmup 5 > $out/b.log 2>&1 || exit 1
    echo "$arm round $r: $(tail -1 $out/b.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $out/ab.txt
  done
done
