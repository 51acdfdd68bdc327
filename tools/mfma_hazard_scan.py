#!/usr/bin/env python3
"""Scan the gfx950 ISA of a HIP source for reads of a block-scaled MFMA's accumulators by a
non-MFMA instruction sooner than N wait states after the MFMA issues.

Why: hipcc (ROCm 7.2) pads only 12 wait states between `v_mfma_scale_f32_16x16x128_f8f6f4`
and a VALU read of its result; in the fp8 BPTT (csrc/rnn_fp8.hip) that read returned partly
updated sums (found with tools/probe_mfma_layout.hip and tests/test_kernels_gpu.py::
test_fp8_bptt_matches_emulation; fixed with an operand-tied s_nop). This lists every such read
per kernel with its distance, counting s_nop N as N + 1 wait states and any other instruction as 1.

  python tools/mfma_hazard_scan.py deepspeech_amd/csrc/rnn_fp8.hip [--min 18] [--strict]
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MFMA = re.compile(r"^\s*(v_mfma_scale\S*)\s+v\[(\d+):(\d+)\]")
VRANGE = re.compile(r"v\[(\d+):(\d+)\]")
VREG = re.compile(r"\bv(\d+)\b")


def isa_of(src: str) -> str:
    d = tempfile.mkdtemp(prefix="ds2isa_")
    out = os.path.join(d, "k.o")
    src = os.path.abspath(src)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, "-o", out,
           "--save-temps", "-I", os.path.dirname(os.path.abspath(src))]
    subprocess.run(cmd, cwd=d, check=True, capture_output=True)
    base = os.path.splitext(os.path.basename(src))[0]
    with open(os.path.join(d, base + "-hip-amdgcn-amd-amdhsa-gfx950.s")) as f:
        return f.read()


def scan(asm: str, window: int = 120):
    """[(kernel, mfma line, reader, gap)] for the first non-MFMA reader of each MFMA's result."""
    out, kernel = [], "?"
    lines = asm.splitlines()
    for i, line in enumerate(lines):
        if re.match(r"^_\w+:", line):
            kernel = line.split(":")[0]
        m = MFMA.match(line)
        if not m:
            continue
        regs = set(range(int(m.group(2)), int(m.group(3)) + 1))
        gap = 0
        for j in range(i + 1, min(i + window, len(lines))):
            t = lines[j].strip()
            if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
                continue
            nop = re.match(r"s_nop (\d+)", t)
            if nop:
                gap += int(nop.group(1)) + 1
                continue
            op, _, args = t.partition(" ")
            srcs = args.split(",", 1)[1] if "," in args else ""
            used = set()
            for a, b in VRANGE.findall(srcs):
                used |= set(range(int(a), int(b) + 1))
            used |= {int(a) for a in VREG.findall(srcs)}
            if used & regs and not op.startswith("v_mfma"):
                out.append((kernel, m.group(1), t[:80], gap))
                break
            dst = VRANGE.match(args.split(",")[0].strip()) if args else None
            if dst and set(range(int(dst.group(1)), int(dst.group(2)) + 1)) & regs and op.startswith("v_mfma"):
                break                            # a later MFMA overwrote the result first
            gap += 1
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--min", type=int, default=18, help="flag reads closer than this many wait states")
    ap.add_argument("--strict", action="store_true", help="exit 1 if any read is flagged")
    a = ap.parse_args()
    rows = scan(isa_of(a.src))
    bad = [r for r in rows if r[3] < a.min]
    per = {}
    for k, _, _, g in rows:
        per[k] = min(per.get(k, 10 ** 9), g)
    print("| kernel | scaled-MFMA result reads | closest (wait states) |\n|---|---|---|")
    for k, g in sorted(per.items()):
        print("| %s | %d | %d%s |" % (k[:70], sum(1 for r in rows if r[0] == k), g, " **< %d**" % a.min if g < a.min else ""))
    for k, op, t, g in bad:
        print("  %s: %s read after %d wait states: %s" % (k[:60], op, g, t))
    return 1 if (a.strict and bad) else 0


if __name__ == "__main__":
    sys.exit(main())
