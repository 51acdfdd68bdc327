#!/bin/bash
# Kernel-level profile of a command (the reference's VTune wrappers, src/vtune.sh /
# tools/vtune.sh, run `amplxe-cl -collect hotspots -- ./train.sh`). rocprofv3 writes a rocpd
# database; tools/rocpd_summary.py turns it into the per-kernel markdown table.
#   scripts/rocprof.sh <out_dir> <steps> -- python3 bench.py --steps 5
#   mode=pmc counters="SQ_INSTS_VALU SQ_INSTS_MFMA" scripts/rocprof.sh ...   (counter run)
set -e
out=${1:?out dir}; steps=${2:-0}; shift 2; [ "$1" = "--" ] && shift
mkdir -p "${out}"
export TMPDIR=${TMPDIR:-/tmp}
if [ "${mode:-trace}" = "pmc" ]; then
  # counters are collected in their own run, with kernel trace only (never with sys/runtime traces)
  rocprofv3 --kernel-trace --pmc ${counters:-SQ_WAVES} -d "${out}" -o run -- "$@"
else
  rocprofv3 --kernel-trace --stats -d "${out}" -o run -- "$@"
fi
db=$(ls -t "${out}"/*_results.db 2>/dev/null | head -n 1 || true)
if [ -n "${db}" ]; then
  python3 "$(dirname "$0")/../tools/rocpd_summary.py" "${db}" --steps "${steps}" -o "${out}/kernels.md"
fi
