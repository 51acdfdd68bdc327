#!/usr/bin/env python3
"""Print the kernel timeline of one training step from a rocprofv3 rocpd database:
start offset, duration, overlap with the previous kernel and a short name per dispatch.
Useful to see stream overlap (e.g. weight-gradient GEMMs running beside the BPTT kernel).

  python tools/rocpd_timeline.py gpurun_out/prof/run_results.db [--index -2] [--phases]

A step is windowed on a kernel that runs ONCE per step at its START (``--anchor``, default the
conv1 forward): from one occurrence up to (not including) the next. Round 3 ended a step at an
``adam_ema`` launch, but a step issues two or three optimizer ranges, so that window dropped the
end of the step. The summary line reports the step period (anchor to
anchor), the span of the step's own kernels, and the TAIL: from the end of the last recurrence
kernel (BPTT) to the end of the step's last kernel.
"""
from __future__ import annotations

import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", default="conv1_fwd", help="kernel-name substring that STARTS a step (once per step)")
    ap.add_argument("--index", type=int, default=-2,
                    help="which anchor occurrence starts the step shown (needs a following anchor)")
    ap.add_argument("--width", type=int, default=70)
    ap.add_argument("--phases", action="store_true", help="also print a per-phase table")
    ap.add_argument("--quiet", action="store_true", help="summary only (no per-kernel lines)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = sorted(c.execute("select name, start, end from kernels"), key=lambda r: r[1])
    starts = [i for i, r in enumerate(rows) if a.anchor in r[0]]
    if len(starts) < 2:
        raise SystemExit("need two anchors")
    idx = a.index if a.index >= 0 else len(starts) + a.index
    if idx + 1 >= len(starts):
        idx = len(starts) - 2
    lo, nxt = starts[idx], starts[idx + 1]
    step = rows[lo:nxt]
    t0 = rows[lo][1]
    period = (rows[nxt][1] - t0) / 1e3
    busy_end = t0
    total_busy = 0.0
    last_bptt_end = None
    for name, s, e in step:
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        ov = max(0, min(busy_end, e) - s)
        if not a.quiet:
            print("%9.1f us  %8.1f us  ovl %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, ov / 1e3, short[:a.width]))
        total_busy += (e - max(s, busy_end)) / 1e3 if e > busy_end else 0.0
        busy_end = max(busy_end, e)
        if phase_of(name) == "recurrence BPTT":
            last_bptt_end = e if last_bptt_end is None else max(last_bptt_end, e)
    span = (busy_end - t0) / 1e3
    line = "step period %.1f us, span of its kernels %.1f us, union of kernel time %.1f us" % (period, span, total_busy)
    if last_bptt_end is not None:
        line += "; last BPTT ends at %.1f us, tail %.1f us" % ((last_bptt_end - t0) / 1e3, (busy_end - last_bptt_end) / 1e3)
    print(line)
    if a.phases:
        # per-phase busy time (kernel time, overlapping kernels counted in each) and the
        # phase's share of the step period
        acc = {}
        for name, s, e in step:
            ph = phase_of(name)
            acc[ph] = acc.get(ph, 0.0) + (e - s) / 1e3
        print("\n| phase | kernel us | % of step period |\n|---|---|---|")
        for ph, us in sorted(acc.items(), key=lambda kv: -kv[1]):
            print("| %s | %.0f | %.1f |" % (ph, us, 100 * us / period))


_PHASES = [       # first match wins: BPTT before fwd (the fp8 kernels share the rnnf8 prefix)
    ("recurrence BPTT", ("rnnf8_bwd", "rnnw_bwd", "rnnrs_bwd", "rnnx_bwd", "rnn_bwd")),
    ("recurrence fwd", ("rnne_fwd", "rnnw_fwd", "rnnf8", "rnnq_fwd", "rnnx_fwd", "rnn_fwd")),
    ("fp8 quantisers", ("quant_pow2", "amax_")),
    ("weight-gradient GEMMs (gemm8 column mode)", ("gemm8_kernel<false, 1, 1>", "gemm8_kernel<false, 1, 0>")),
    ("projection / dx / FC GEMM (hand-written)", ("gemm_kernel", "gemm8_kernel", "transpose_bf16")),
    ("library GEMM (hipBLASLt) BBS = dx", ("_BBS_",)),
    ("library GEMM (hipBLASLt) BSS = weight grads", ("_BSS_",)),
    ("conv front-end fwd", ("conv1_fwd", "conv2_fwd", "bn_cl_apply", "bn_cl_finalize")),
    ("conv front-end bwd", ("conv1_wgrad", "conv2_wgrad", "conv2_dgrad", "bn_cl_bwd", "wgrad_reduce")),
    ("CTC + head", ("ctc_", "fc_lsm")),
    ("optimizer", ("adam_ema", "grad_norm")),
    ("fills / copies", ("multi_fill", "rocclr_fill", "rocclr_copy", "FillFunctor", "copy_kernel")),
]


def phase_of(name: str) -> str:
    for ph, keys in _PHASES:
        if any(k in name for k in keys):
            return ph
    return "other (torch elementwise / reductions)"


if __name__ == "__main__":
    main()
