#!/bin/bash
# conv1 weight-gradient de-interleave lane order: numerics, solo kernel time (both builds), headline A/B.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/c1w2
mkdir -p $out
so=ab/_C_c1wold$(python -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py > $out/tests.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/pn -o run -- python3 tools/bench_conv.py --iters 10 > $out/pn.log 2>&1 || exit 1
DS2_EXT_SO=$so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/po -o run -- python3 tools/bench_conv.py --iters 10 > $out/po.log 2>&1 || exit 1
python3 tools/rocpd_summary.py $out/pn/run_results.db -o $out/pn.md > /dev/null 2>&1
python3 tools/rocpd_summary.py $out/po/run_results.db -o $out/po.md > /dev/null 2>&1
BENCH_ARGS="--no_walk --no_infer" timeout -k 10 700 bash scripts/ab_so.sh 3 c1wold > $out/ab.log 2>&1
