#!/usr/bin/env python3
"""Print the kernel timeline of one training step from a rocprofv3 rocpd database:
start offset, duration, overlap with the previous kernel and a short name per dispatch.
Useful to see stream overlap (e.g. weight-gradient GEMMs running beside the BPTT kernel).

  python tools/rocpd_timeline.py gpurun_out/prof/run_results.db --anchor adam_ema --index -2
"""
from __future__ import annotations

import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", default="adam_ema", help="kernel-name substring that ends a step")
    ap.add_argument("--index", type=int, default=-2, help="which anchor occurrence ends the step shown")
    ap.add_argument("--width", type=int, default=70)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = sorted(c.execute("select name, start, end from kernels"), key=lambda r: r[1])
    ends = [i for i, r in enumerate(rows) if a.anchor in r[0]]
    if len(ends) < 2:
        raise SystemExit("need two anchors")
    hi = ends[a.index]
    lo = ends[a.index - 1] + 1
    t0 = rows[lo][1]
    busy_end = t0
    total_busy = 0.0
    for name, s, e in rows[lo:hi + 1]:
        short = name.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
        ov = max(0, min(busy_end, e) - s)
        print("%9.1f us  %8.1f us  ovl %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, ov / 1e3, short[:a.width]))
        total_busy += (e - max(s, busy_end)) / 1e3 if e > busy_end else 0.0
        busy_end = max(busy_end, e)
    print("step span %.1f us, union of kernel time %.1f us" % ((busy_end - t0) / 1e3, total_busy))


if __name__ == "__main__":
    main()
