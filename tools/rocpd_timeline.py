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
    ap.add_argument("--phases", action="store_true", help="also print a per-phase table")
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
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        ov = max(0, min(busy_end, e) - s)
        print("%9.1f us  %8.1f us  ovl %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, ov / 1e3, short[:a.width]))
        total_busy += (e - max(s, busy_end)) / 1e3 if e > busy_end else 0.0
        busy_end = max(busy_end, e)
    print("step span %.1f us, union of kernel time %.1f us" % ((busy_end - t0) / 1e3, total_busy))
    if a.phases:
        # per-phase busy time (kernel time, overlapping kernels counted in each) and the
        # phase's share of the step span
        acc = {}
        for name, s, e in rows[lo:hi + 1]:
            ph = phase_of(name)
            acc[ph] = acc.get(ph, 0.0) + (e - s) / 1e3
        span = (busy_end - t0) / 1e3
        print("\n| phase | kernel us | % of step span |\n|---|---|---|")
        for ph, us in sorted(acc.items(), key=lambda kv: -kv[1]):
            print("| %s | %.0f | %.1f |" % (ph, us, 100 * us / span))


_PHASES = [
    ("recurrence fwd", ("rnne_fwd", "rnnw_fwd", "rnnf8", "rnnq_fwd", "rnnx_fwd", "rnn_fwd")),
    ("recurrence BPTT", ("rnnw_bwd", "rnnrs_bwd", "rnnx_bwd", "rnn_bwd")),
    ("weight-gradient GEMMs (gemm8 column mode)", ("gemm8_kernel<false, 1, 1>", "gemm8_kernel<false, 1, 0>")),
    ("projection / dx / FC GEMM (hand-written)", ("gemm_kernel", "gemm8_kernel", "transpose_bf16")),
    ("library GEMM (hipBLASLt) BBS = dx", ("_BBS_",)),
    ("library GEMM (hipBLASLt) BSS = weight grads", ("_BSS_",)),
    ("conv front-end fwd", ("conv1_fwd", "conv2_fwd", "bn_cl_apply", "bn_cl_finalize")),
    ("conv front-end bwd", ("conv1_wgrad", "conv2_wgrad", "conv2_dgrad", "bn_cl_bwd")),
    ("CTC + head", ("ctc_", "fc_lsm")),
    ("optimizer", ("adam_ema", "grad_norm", "wgrad_reduce")),
    ("fills / copies", ("multi_fill", "rocclr_fill", "rocclr_copy", "FillFunctor", "copy_kernel")),
]


def phase_of(name: str) -> str:
    for ph, keys in _PHASES:
        if any(k in name for k in keys):
            return ph
    return "other (torch elementwise / reductions)"


if __name__ == "__main__":
    main()
