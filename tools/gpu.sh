#!/bin/bash
# Submit one gpurun call; resubmit ONLY when the pool had no box / the box failed before
# the command started (gpurun exit 3 or a "transient" status: nothing ran, nothing
# charged). A command that ran and failed is never retried.
#   tools/gpu.sh <timeout_s> '<command>'
t="$1"; shift
for i in 1 2 3 4 5 6; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1); rc=$?
  echo "$out" | grep -v "^W2026" | tail -n 40
  if [ $rc -eq 3 ] || echo "$out" | grep -q "status=transient"; then
    echo "[gpu.sh] no box (attempt $i), retrying in 60s"; sleep 60; continue
  fi
  exit $rc
done
exit 3
