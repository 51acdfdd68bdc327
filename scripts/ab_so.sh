#!/bin/bash
# Same-box A/B of compile-time variants (build.py --variant NAME -D ...): alternate the
# in-tree _C and each ab/_C_<NAME>.so through bench.py, ROUNDS times, one JSON line each.
#   [BENCH_ARGS="--cell rnn_relu ..."] bash scripts/ab_so.sh ROUNDS NAME [NAME...] > gpurun_out/ab.log
set -o pipefail
rounds=${1:-3}; shift
ext=$(python -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
run() {   # $1 = variant name, $2 = round; DS2_EXT_SO already exported (or not) by the caller
  local out
  out=$(timeout -k 10 120 python bench.py --steps 30 --warmup 10 ${BENCH_ARGS:-} | tail -1) || { echo "bench failed: $1" >&2; exit 1; }
  echo "{\"variant\": \"$1\", \"round\": $2, \"bench\": $out}"
}
for r in $(seq 1 "$rounds"); do
  (unset DS2_EXT_SO; run base "$r") || exit 1
  for v in "$@"; do
    (export DS2_EXT_SO=ab/_C_${v}${ext}; run "$v" "$r") || exit 1
  done
done
