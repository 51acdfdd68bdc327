#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy table of a HIP source compiled for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage), flagging spills and scratch use.

  python tools/kernel_resources.py deepspeech_amd/csrc/rnn_xcd.hip [--filter rnnrs] [--strict]

--strict exits non-zero if any kernel spills VGPRs or uses scratch (a spilled
persistent kernel runs an order of magnitude slower: check after every edit).
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def analyse(src: str):
    with tempfile.TemporaryDirectory() as d:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-c",
               src, "-o", os.path.join(d, "k.o"), "-I", os.path.join(ROOT, "deepspeech_amd", "csrc"),
               "-Rpass-analysis=kernel-resource-usage"]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise SystemExit(r.stdout)
    rows, cur = [], None
    for line in r.stdout.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s+(\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return rows


def demangle(names):
    try:
        out = subprocess.run(["/opt/rocm/llvm/bin/llvm-cxxfilt"], input="\n".join(names), text=True,
                             stdout=subprocess.PIPE).stdout.splitlines()
        return out if len(out) == len(names) else names
    except OSError:
        return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src", nargs="+")
    ap.add_argument("--filter", default="")
    ap.add_argument("--strict", action="store_true")
    a = ap.parse_args()
    bad = 0
    for src in a.src:
        rows = [r for r in analyse(src) if a.filter in r["name"]]
        names = demangle([r["name"] for r in rows])
        print("## %s" % os.path.relpath(src, ROOT))
        print("| kernel | VGPR | AGPR | spill | scratch B | waves/SIMD | LDS B |")
        print("|---|---|---|---|---|---|---|")
        for r, n in zip(rows, names):
            spill = r.get("VGPRs Spill", 0)          # SGPR spills go to VGPR lanes: cheap, not flagged
            scratch = r.get("ScratchSize [bytes/lane]", 0)
            flag = " **SPILL**" if spill or scratch else ""
            bad += bool(spill or scratch)
            short = n.split("(")[0].replace("(anonymous namespace)::", "")
            print("| %s%s | %s | %s | %s | %s | %s | %s |" % (short[:70], flag, r.get("VGPRs", "?"), r.get("AGPRs", "?"),
                                                       spill, scratch, r.get("Occupancy [waves/SIMD]", "?"),
                                                       r.get("LDS Size [bytes/block]", "?")))
    if a.strict and bad:
        sys.exit(1)


if __name__ == "__main__":
    main()
