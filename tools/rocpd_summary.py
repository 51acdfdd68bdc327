#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite ``*_results.db``) as a markdown table.

  python tools/rocpd_summary.py gpurun_out/prof/run_results.db [--steps K] [--top 40]
         [--title "..."] [-o profiles/xyz.md]

rocprofv3 (ROCm 7.x) writes its ``--kernel-trace --stats`` output as a rocpd database by
default; this groups the dispatches by kernel name (total / calls / avg / share) and, with
``--steps``, divides the totals by the number of profiled steps so the table reads as
"GPU time per training step". Also reports busy time vs. the wall span of the trace.
"""
from __future__ import annotations

import argparse
import sqlite3
import sys


def summarise(db: str, steps: int = 0, top: int = 40, title: str = "") -> str:
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels"))
    if not rows:
        return "(no kernel dispatches in %s)\n" % db
    agg = {}
    t0 = min(r[1] for r in rows)
    t1 = max(r[2] for r in rows)
    for name, s, e in rows:
        a = agg.setdefault(name, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1000.0                       # ns -> us
    total = sum(v[1] for v in agg.values())
    out = []
    if title:
        out.append("# " + title)
        out.append("")
    out.append("Dispatches: %d, kernel time %.2f ms, trace span %.2f ms%s." % (
        len(rows), total / 1000.0, (t1 - t0) / 1e6,
        (", %d steps -> %.3f ms kernel time per step" % (steps, total / 1000.0 / steps)) if steps else ""))
    out.append("")
    hdr = "| total ms | % | calls | avg us |" + (" ms/step |" if steps else "") + " kernel |"
    out.append(hdr)
    out.append("|" + "---|" * (hdr.count("|") - 1))
    for name, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        short = name if len(name) <= 110 else name[:107] + "..."
        short = short.replace("|", "\\|")
        row = "| %.2f | %.2f | %d | %.1f |" % (us / 1000.0, 100.0 * us / total, n, us / n)
        if steps:
            row += " %.3f |" % (us / 1000.0 / steps)
        out.append(row + " `%s` |" % short)
    return "\n".join(out) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--title", type=str, default="")
    ap.add_argument("-o", "--output", type=str, default="")
    a = ap.parse_args(argv)
    txt = summarise(a.db, a.steps, a.top, a.title)
    if a.output:
        with open(a.output, "w") as f:
            f.write(txt)
    sys.stdout.write(txt)
    return 0


if __name__ == "__main__":
    sys.exit(main())
