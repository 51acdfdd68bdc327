#!/bin/bash
# DP step at 1000 frames alone vs after a shorter shape, and the single-device path the same way.
set -o pipefail
out=gpurun_out/r6_dpshape2
mkdir -p $out
for v in "--force_dp --frames 1000" "--force_dp --frames 1000,1000" "--force_dp --frames 400,1000" "--frames 400,1000" \
         "--force_dp --frames 100,1000"; do
  echo "== $v" | tee -a $out/host.md
  timeout -k 10 240 python tools/host_overhead.py --steps 30 $v 2>&1 | grep "^|" | tee -a $out/host.md || exit 1
done
timeout -k 10 300 python -u -m pytest -x -s -q --timeout 250 --timeout-method thread "tests/test_engine_gpu.py::test_headline_geometry_matches_reference" 2>&1 | grep -E "relative gradient|passed|failed" | tee gpurun_out/r6_dpshape2/tol.txt
bash scripts/r6_projgrid.sh
