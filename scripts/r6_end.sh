#!/bin/bash
# Round-6 end (late session): the whole GPU suite, smoke, the driver bench twice, a headline
# kernel trace with its timeline and per-step census, and the secondary configurations.
set -o pipefail
out=gpurun_out/r6_end
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
for r in 1 2; do
  timeout -k 10 300 python bench.py > $out/bench$r.json 2> $out/bench$r.err || { tail -20 $out/bench$r.err; exit 1; }
  tail -1 $out/bench$r.json | cut -c1-200
done
