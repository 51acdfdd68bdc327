#!/bin/bash
# Same-box alternating A/B of the current tree against another full source tree built in place
# (e.g. an older commit: mkdir -p ab/r4 && git archive <commit> | tar -x -C ab/r4 &&
# (cd ab/r4 && python build.py)):  bash scripts/ab_tree.sh ROUNDS DIR [bench args...]
set -o pipefail
rounds=$1; other=$2; shift 2
here=$(pwd)
for r in $(seq 1 "$rounds"); do
  for tree in "$here" "$other"; do
    out=$(cd "$tree" && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_infer --no_walk "$@" 2>/dev/null | tail -1) || \
      out=$(cd "$tree" && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_infer "$@" | tail -1) || exit 1
    echo "round $r [$tree] $(echo "$out" | grep -o '"ms_per_step": [0-9.]*')"
  done
done
