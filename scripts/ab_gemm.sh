set -o pipefail
mkdir -p gpurun_out/ab
for spec in "hip" "proj,dx" "proj" "torch" "hip:3" "proj,dx,wgrad:w5"; do
  name=$(echo "$spec" | tr ',:' '__')
  g=${spec%%:*}; c=""
  case "$spec" in *:3) c=3;; esac
  if [ -n "$c" ]; then export DS2_GEMM_CFG=$c; else unset DS2_GEMM_CFG; fi
  DS2_GEMM=$g timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab/$name.log 2>&1 || exit 1
  echo "$spec $(tail -1 gpurun_out/ab/$name.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
