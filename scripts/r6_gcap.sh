#!/bin/bash
# Grid cap of the grouped tail weight-gradient launch, with the reordered conv backward.
set -o pipefail
out=gpurun_out/r6_gcap
mkdir -p $out
BENCH_ARGS="--no_infer --no_walk" bash scripts/ab_env.sh 3 "DS2_GROUP_CAP_AB=0" "DS2_GROUP_CAP_AB=160" "DS2_GROUP_CAP_AB=224" "DS2_GROUP_CAP_AB=256" > $out/ab.txt 2>&1
