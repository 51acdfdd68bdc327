#!/bin/bash
# GPU job runner used with gpurun: runs named steps, each under its own time limit, and
# stops at the first fault / abort / segfault / timeout (exit 124, 134, 137, 139 or >128).
# A plain test failure (exit 1) does not stop later steps.
#   scripts/gpu_job.sh "name:seconds:command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DS2_RNN_TIMEOUT_S=${DS2_RNN_TIMEOUT_S:-10}
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"
  secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s): $cmd" | tee -a gpurun_out/job.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/job.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then
    echo "=== stopping after [$name] (rc=$rc)" | tee -a gpurun_out/job.log
    exit $rc
  fi
done
exit 0
