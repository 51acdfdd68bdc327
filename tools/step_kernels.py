#!/usr/bin/env python3
"""Per-step kernel census of a rocprofv3 kernel trace (rocpd database): only the dispatches
that start inside steady-state training steps (a step runs from one conv1_fwd_kernel to the
next), so set-up work (arena copies, plan fills, first-use captures) does not pollute the
per-step counts the way a whole-run --stats summary divided by the step count does.

  python tools/step_kernels.py gpurun_out/x/prof/run_results.db [--skip 3] [--marker conv1_fwd_kernel]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--skip", type=int, default=3, help="leading steps to ignore (warm-up)")
    ap.add_argument("--marker", default="conv1_fwd_kernel")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = list(cur.execute("select name, start, end from kernels order by start"))
    starts = [r[1] for r in rows if a.marker in r[0]]
    windows = list(zip(starts[a.skip:-1], starts[a.skip + 1:]))
    if not windows:
        raise SystemExit("no complete steady-state step in the trace")
    calls, busy = collections.Counter(), collections.Counter()
    for s0, s1 in windows:
        for name, b, e in rows:
            if s0 <= b < s1:
                calls[name] += 1
                busy[name] += (e - b) / 1e3
    n = len(windows)
    period = sum(s1 - s0 for s0, s1 in windows) / n / 1e3
    print("%d steady-state steps, mean period %.1f us; per step:" % (n, period))
    print()
    print("| calls/step | kernel us/step | kernel |")
    print("|---|---|---|")
    for name, t in sorted(busy.items(), key=lambda kv: -kv[1]):
        short = name if len(name) <= 100 else name[:97] + "..."
        print("| %.1f | %.1f | `%s` |" % (calls[name] / n, t / n, short))
    torch_k = [k for k in calls if "at::" in k or "rocclr" in k]
    print()
    print("PyTorch / runtime-copy kernels inside the steps: %s" % (", ".join(torch_k) if torch_k else "none"))


if __name__ == "__main__":
    main()
