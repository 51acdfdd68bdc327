set -o pipefail
mkdir -p gpurun_out/sm
timeout -k 10 240 python -u tools/bench_gemm_small_m.py --cfg5 --M 672,1312,2432,3712 > gpurun_out/sm/bench.log 2>&1 &&
for arm in 1 0 1 0; do DS2_SMALL_M=$arm timeout -k 10 200 python -u tools/host_overhead.py --graph --frames 100,200,400 > gpurun_out/sm/ho_$arm.log 2>&1 && echo "arm $arm" >> gpurun_out/sm/ho_all.log && tail -8 gpurun_out/sm/ho_$arm.log >> gpurun_out/sm/ho_all.log || exit 1; done &&
DS2_SMALL_M=1 timeout -k 10 300 python -u bench.py > gpurun_out/sm/bench1.log 2>&1 &&
DS2_SMALL_M=0 timeout -k 10 300 python -u bench.py > gpurun_out/sm/bench0.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_step_graphs_gpu.py > gpurun_out/sm/tests.log 2>&1
