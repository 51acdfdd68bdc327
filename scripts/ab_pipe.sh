#!/bin/bash
# gemm8 pipelined unit seam (DS2_G8_PIPE variant build): numerics of the variant, isolated
# projection GEMM times of both builds, then the headline step alternated.
set -o pipefail
out=gpurun_out/pipe
mkdir -p $out
so=ab/_C_pipe$(python -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
DS2_EXT_SO=$so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
for r in 1 2; do
  timeout -k 10 120 python -u tools/g8_epi_probe.py >> $out/probe.log 2>&1 || exit 1
  DS2_EXT_SO=$so timeout -k 10 120 python -u tools/g8_epi_probe.py >> $out/probe.log 2>&1 || exit 1
done
BENCH_ARGS="--no_walk --no_infer" timeout -k 10 900 bash scripts/ab_so.sh 3 pipe > $out/ab.log 2>&1
