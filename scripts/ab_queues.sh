#!/bin/bash
# A/B of HIP hardware queues per process (GPU_MAX_HW_QUEUES) for the plain and the forced
# data-parallel step: with the DP ordering / RCCL streams a process has more streams than 4
# queues, and a side stream sharing a queue with the main stream serialises the weight-
# gradient GEMMs behind the BPTT.
set -o pipefail
mkdir -p gpurun_out/abq
for q in ${queues:-4 8 16}; do
  for i in 1 2; do
    for mode in plain dp; do
      extra=""; [ "$mode" = dp ] && extra="--force_dp"
      DS2_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py $extra > gpurun_out/abq/q${q}_${mode}_$i.log 2>&1 || exit 1
      echo "q=$q $mode run$i $(tail -1 gpurun_out/abq/q${q}_${mode}_$i.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"
    done
  done
done
