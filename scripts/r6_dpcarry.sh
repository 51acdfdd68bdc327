#!/bin/bash
# DP carried bucket update: bitwise test + world-1 --force_dp A/B against plain.
set -o pipefail
mkdir -p gpurun_out/r6_dpcarry
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_dp_ready_gpu.py tests/test_defer_update_gpu.py tests/test_dp_gpu.py > gpurun_out/r6_dpcarry/tests.log 2>&1 || { tail -30 gpurun_out/r6_dpcarry/tests.log; exit 1; }
tail -3 gpurun_out/r6_dpcarry/tests.log
bash scripts/ab_dp.sh 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r6_dpcarry/dp.txt
out=gpurun_out/r6_dpcarry
timeout -k 10 300 bash scripts/rocprof.sh $out/prof 8 -- python3 bench.py --steps 5 --warmup 3 --no_infer --no_walk --force_dp > $out/prof.log 2>&1 || exit 1
db=$(ls $out/prof/*.db | head -1)
python3 tools/rocpd_timeline.py $db --index 5 --phases > $out/timeline.txt 2>&1 || exit 1
python3 tools/step_kernels.py $db > $out/step_kernels.md 2>&1 || exit 1
grep "step period" $out/timeline.txt
