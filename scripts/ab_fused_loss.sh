#!/bin/bash
# Same-box A/B of the fused loss mean + watch: 100 / 200-frame graph steps and the headline.
set -o pipefail
out=gpurun_out/ab_floss
mkdir -p $out
for r in 1 2 3; do
  for arm in 1 0; do
    DS2_FUSED_LOSS=$arm timeout -k 10 200 python tools/host_overhead.py --frames 100,200 --steps 40 --graph > $out/ho.log 2>&1 || exit 1
    echo "DS2_FUSED_LOSS=$arm round $r: $(grep '^| [12]00 ' $out/ho.log | awk -F'|' '{printf "%s:%s ", $2, $4}')" >> $out/ab.txt
  done
done
out=$out ROUNDS=3 STEPS=30 bash scripts/ab_env3.sh "DS2_FUSED_LOSS=1" "DS2_FUSED_LOSS=0" || exit 1
