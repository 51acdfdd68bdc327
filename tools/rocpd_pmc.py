#!/usr/bin/env python3
"""Per-kernel PMC table from a rocprofv3 `--pmc` run's rocpd database: for every kernel whose
name matches --match, the mean per-dispatch value of each collected counter and the mean
dispatch duration.

  python tools/rocpd_pmc.py gpurun_out/pmc_conv/p1/run_results.db [--match conv2_dgrad] [-o out.md]
"""
import argparse
import collections
import sqlite3
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:70]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db", nargs="+")
    ap.add_argument("--match", default="", help="substring of kernel names to keep")
    ap.add_argument("-o", "--out")
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> counter -> [v]
    durs = collections.defaultdict(dict)                                     # kernel -> dispatch -> ns
    for path in a.db:
        c = sqlite3.connect(path)
        q = ("select dispatch_id, kernel_name, counter_name, sum(value), max(\"end\") - min(start) "
             "from counters_collection group by dispatch_id, counter_name")
        for did, kname, cname, v, dur in c.execute(q):
            if a.match and a.match not in kname:
                continue
            k = short(kname)
            vals[k][cname].append(v)
            durs[k][(path, did)] = dur
    lines = []
    for k in sorted(vals):
        d = durs[k]
        lines.append("### %s  (%d dispatches, mean %.1f us)" % (k, len(d), sum(d.values()) / max(1, len(d)) / 1e3))
        lines.append("| counter | mean per dispatch |\n|---|---|")
        for cn in sorted(vals[k]):
            v = vals[k][cn]
            lines.append("| %s | %.4g |" % (cn, sum(v) / len(v)))
        lines.append("")
    text = "\n".join(lines)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
