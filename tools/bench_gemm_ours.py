#!/usr/bin/env python3
"""Hand-written MFMA GEMMs (csrc/gemm.hip) vs the hipBLASLt calls they replace, on the
GEMM shapes of one DS2 training step (HIP events, random data, interleaved rounds).

  python tools/bench_gemm_ours.py [--T2 241] [--N 32] [--H 800] [--D 2400] [--rounds 5]

Prints one JSON line per (gemm, implementation): best/median us and TFLOP/s.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeech_amd.ops import gemm as G  # noqa: E402

NCFG = 9


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T2", type=int, default=241)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--H", type=int, default=800)
    ap.add_argument("--D", type=int, default=2400)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", type=str, default="", help="substring filter on case names")
    a = ap.parse_args()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    M = a.T2 * a.N
    GH2 = 6 * a.H
    cases = {}
    for D in (a.D, a.H):
        x = torch.randn(M, D, device=dev, dtype=bf)
        W = torch.randn(GH2, D, device=dev, dtype=bf) * 0.05
        b = torch.randn(GH2, device=dev, dtype=bf)
        dgx = torch.randn(M, GH2, device=dev, dtype=bf)
        o16 = torch.empty(M, GH2, device=dev, dtype=bf)
        dx16 = torch.empty(M, D, device=dev, dtype=bf)
        dW = torch.empty(GH2, D, device=dev)
        fl_p = 2.0 * M * D * GH2
        cases["proj D=%d torch" % D] = (fl_p, lambda x=x, W=W, b=b: torch.addmm(b, x, W.t()))
        for cfg in range(NCFG):
            cases["proj D=%d ours cfg%d" % (D, cfg)] = (
                fl_p, lambda x=x, W=W, b=b, o=o16, cfg=cfg, D=D: G.gemm(x, W, o, M, GH2, D, False, False, 0, 1.0, b, cfg))
        cases["dx D=%d torch" % D] = (fl_p, lambda dgx=dgx, W=W: torch.mm(dgx, W))
        for cfg in range(NCFG):
            cases["dx D=%d ours cfg%d" % (D, cfg)] = (
                fl_p, lambda dgx=dgx, W=W, o=dx16, cfg=cfg, D=D: G.gemm(dgx, W, o, M, D, GH2, False, True, 0, 1.0, None, cfg))
        Wt = W.t().contiguous()
        for cfg in range(NCFG):
            cases["dx D=%d rowrow cfg%d" % (D, cfg)] = (
                fl_p, lambda dgx=dgx, Wt=Wt, o=dx16, cfg=cfg, D=D: G.gemm(dgx, Wt, o, M, D, GH2, False, False, 0, 1.0, None,
                                                                          cfg))
        cases["dW D=%d torch" % D] = (fl_p, lambda dgx=dgx, x=x, o=dW: torch.mm(dgx.t(), x, out_dtype=torch.float32, out=o))
        for cfg in range(NCFG):
            cases["dW D=%d ours cfg%d" % (D, cfg)] = (
                fl_p, lambda dgx=dgx, x=x, o=dW, cfg=cfg, D=D: G.gemm(dgx, x, o, GH2, D, M, True, True, 1, 1.0, None, cfg))
    dgh = torch.randn(2, M, 3 * a.H, device=dev, dtype=bf)
    h = torch.randn(2, M, a.H, device=dev, dtype=bf)
    dU = torch.empty(2, 3 * a.H, a.H, device=dev)
    fl_u = 2 * 2.0 * M * 3 * a.H * a.H
    cases["dU torch bmm"] = (fl_u, lambda: torch.bmm(dgh.transpose(1, 2), h, out_dtype=torch.float32, out=dU))
    for cfg in range(NCFG):
        cases["dU ours cfg%d" % cfg] = (fl_u, lambda cfg=cfg: G.gemm(dgh, h, dU, 3 * a.H, a.H, M, True, True, 1, 1.0,
                                                                      None, cfg))
    if a.only:
        cases = {k: v for k, v in cases.items() if any(o in k for o in a.only.split(","))}
    for _, (fl, f) in cases.items():       # warm-up / tuning lookups
        f()
        f()
    torch.cuda.synchronize()
    times = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, (fl, f) in cases.items():
            times[k].append(timeit(f))
    for k, (fl, f) in cases.items():
        t = times[k]
        print(json.dumps({"gemm": k, "best_us": round(min(t), 1), "median_us": round(statistics.median(t), 1),
                          "TFLOPs": round(fl / min(t) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
