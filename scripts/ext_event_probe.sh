#!/bin/bash
# hipExtLaunchKernel stop events vs recorded markers (tools/probe_ext_event.py), then the GEMM tests.
set -o pipefail
out=gpurun_out/extev
mkdir -p $out
timeout -k 10 120 python3 tools/probe_ext_event.py --reps 8 > $out/plain.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$out -o run -- python3 $GRAFT_REPO_ROOT/tools/probe_ext_event.py --reps 8 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 tools/probe_ext_event.py --analyze $(ls $out/*.db | head -1) > $out/gaps.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $out/gemm_tests.log 2>&1 || exit 1
