#!/usr/bin/env python3
"""csrc/gemm8.hip (256^2 8-phase, bf16 / fp8) against csrc/gemm.hip's best configuration and
hipBLASLt on the row-row ("NT") GEMMs of the DS2 configurations: forward projections
x W^T and input gradients dgx (W^T)^T with a K-contiguous W^T (HIP events, random data,
interleaved rounds, best of).

  python tools/bench_gemm8.py [--rounds 5] [--only proj]

One JSON line per (case, implementation): best / median us and TFLOP/s.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeech_amd.ops import gemm as G  # noqa: E402
from deepspeech_amd.ops import _ext  # noqa: E402


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", type=str, default="")
    ap.add_argument("--M", type=int, default=241 * 32)
    a = ap.parse_args()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    M = a.M
    # (name, N, K): projections N = 2 directions x gates x H, K = layer input; dx: N = layer
    # input, K = 2 x gates x H
    shapes = [("proj gru800 L0", 4800, 2400), ("proj gru800 L1", 4800, 800),
              ("dx gru800 L0", 2400, 4800), ("dx gru800 L1", 800, 4800),
              ("proj gru1280 L0", 7680, 2400), ("proj gru1280 L1", 7680, 1280),
              ("dx gru1280 L1", 1280, 7680), ("proj relu1760 L0", 3520, 2400), ("proj relu1760 L1", 3520, 1760),
              ("dx relu1760 L1", 1760, 3520)]
    cases = {}
    for name, N, K in shapes:
        if a.only and a.only not in name:
            continue
        x = torch.randn(M, K, device=dev, dtype=bf)
        W = torch.randn(N, K, device=dev, dtype=bf) * 0.05
        b = torch.randn(N, device=dev, dtype=bf)
        o = torch.empty(M, N, device=dev, dtype=bf)
        fl = 2.0 * M * N * K
        cases[name + " | hipblaslt"] = (fl, lambda x=x, W=W, b=b: torch.addmm(b, x, W.t()))
        cases[name + " | gemm cfg7"] = (fl, lambda x=x, W=W, b=b, o=o, N=N, K=K: G.gemm(x, W, o, M, N, K, False, False,
                                                                                         0, 1.0, b, 7))
        cases[name + " | gemm cfg1"] = (fl, lambda x=x, W=W, b=b, o=o, N=N, K=K: G.gemm(x, W, o, M, N, K, False, False,
                                                                                         0, 1.0, b, 1))
        cases[name + " | gemm8 bf16"] = (fl, lambda x=x, W=W, b=b, o=o: G.gemm8(x, W, o, 0, 1.0, b))
        if name.startswith("proj"):
            cases[name + " | gemm8 fp8 (+quant)"] = (fl, lambda x=x, W=W, b=b: G.linear_fp8(x, W, b, 1.0))
            Kp = G.fp8_pad(K)
            x8 = torch.zeros(M, Kp, device=dev, dtype=torch.float8_e4m3fn)
            x8[:, :K] = (x.float() * 8).to(torch.float8_e4m3fn)
            w8 = torch.zeros(N, Kp, device=dev, dtype=torch.float8_e4m3fn)
            w8[:, :K] = (W.float() * 100).to(torch.float8_e4m3fn)
            cases[name + " | gemm8 fp8 (GEMM only)"] = (fl, lambda x8=x8, w8=w8, b=b, o=o: G.gemm8(x8, w8, o, 0, 1.0, b))
    # input gradients with W read as stored ([6H][D]: column-mode B) and weight gradients
    # (both operands column mode), headline shapes
    for D in (2400, 800):
        name = "dx colB D=%d" % D
        if not a.only or a.only in name:
            dgx = torch.randn(M, 4800, device=dev, dtype=bf)
            W = torch.randn(4800, D, device=dev, dtype=bf) * 0.05
            o = torch.empty(M, D, device=dev, dtype=bf)
            fl = 2.0 * M * 4800 * D
            cases[name + " | hipblaslt"] = (fl, lambda dgx=dgx, W=W: torch.mm(dgx, W))
            cases[name + " | gemm cfg8"] = (fl, lambda dgx=dgx, W=W, o=o, D=D: G.gemm(dgx, W, o, M, D, 4800, False, True,
                                                                                       0, 1.0, None, 8))
            for sp in (1, 2, 3):
                cases[name + " | gemm8 S%d" % sp] = (fl, lambda dgx=dgx, W=W, o=o, sp=sp: G.gemm8(dgx, W, o, 0, b_col=True,
                                                                                                  splits=sp))
        name = "dW D=%d" % D
        if not a.only or a.only in name:
            dgx = torch.randn(M, 4800, device=dev, dtype=bf)
            x = torch.randn(M, D, device=dev, dtype=bf)
            o = torch.empty(4800, D, device=dev)
            fl = 2.0 * M * 4800 * D
            cases[name + " | hipblaslt"] = (fl, lambda dgx=dgx, x=x, o=o: torch.mm(dgx.t(), x, out_dtype=torch.float32,
                                                                                   out=o))
            cases[name + " | gemm cfg2"] = (fl, lambda dgx=dgx, x=x, o=o, D=D: G.gemm(dgx, x, o, 4800, D, M, True, True, 1,
                                                                                       1.0, None, 2))
            for sp in (1, 2, 3, 4):
                cases[name + " | gemm8 S%d" % sp] = (fl, lambda dgx=dgx, x=x, o=o, sp=sp: G.gemm8(
                    dgx, x, o, 1, a_col=True, b_col=True, splits=sp))
    name = "dU gru800"
    if not a.only or a.only in name:
        dgh = torch.randn(2, M, 2400, device=dev, dtype=bf)
        h = torch.randn(2, M, 800, device=dev, dtype=bf)
        o = torch.empty(2, 2400, 800, device=dev)
        fl = 2 * 2.0 * M * 2400 * 800
        cases[name + " | hipblaslt"] = (fl, lambda: torch.bmm(dgh.transpose(1, 2), h, out_dtype=torch.float32, out=o))
        cases[name + " | gemm cfg3"] = (fl, lambda: G.gemm(dgh, h, o, 2400, 800, M, True, True, 1, 1.0, None, 3))
        for sp in (1, 2, 3, 4):
            cases[name + " | gemm8 S%d" % sp] = (fl, lambda sp=sp: G.gemm8(dgh, h, o, 1, a_col=True, b_col=True,
                                                                            splits=sp))
    # wide layers: weight gradients (column-column) of config 5 (H = 1280) and the reference's
    # clipped-ReLU H = 1760, and config 5's dx
    for tag, GH, H, D in (("gru1280", 3 * 1280, 1280, 1280), ("relu1760", 1760, 1760, 1760)):
        name = "dU " + tag
        if not a.only or a.only in name:
            dgh = torch.randn(2, M, GH, device=dev, dtype=bf)
            h = torch.randn(2, M, H, device=dev, dtype=bf)
            o = torch.empty(2, GH, H, device=dev)
            fl = 2 * 2.0 * M * GH * H
            cases[name + " | hipblaslt"] = (fl, lambda dgh=dgh, h=h, o=o: torch.bmm(dgh.transpose(1, 2), h,
                                                                                   out_dtype=torch.float32, out=o))
            for sp in (1, 2, 3):
                cases[name + " | gemm8 S%d" % sp] = (fl, lambda dgh=dgh, h=h, o=o, sp=sp: G.gemm8(
                    dgh, h, o, 1, a_col=True, b_col=True, splits=sp))
        name = "dW " + tag
        if not a.only or a.only in name:
            dgx = torch.randn(M, 2 * GH, device=dev, dtype=bf)
            x = torch.randn(M, D, device=dev, dtype=bf)
            o = torch.empty(2 * GH, D, device=dev)
            fl = 2.0 * M * 2 * GH * D
            cases[name + " | hipblaslt"] = (fl, lambda dgx=dgx, x=x, o=o: torch.mm(dgx.t(), x, out_dtype=torch.float32,
                                                                                   out=o))
            for sp in (1, 2, 3):
                cases[name + " | gemm8 S%d" % sp] = (fl, lambda dgx=dgx, x=x, o=o, sp=sp: G.gemm8(
                    dgx, x, o, 1, a_col=True, b_col=True, splits=sp))
    name = "dxT gru1280"
    if not a.only or a.only in name:
        dgx = torch.randn(M, 7680, device=dev, dtype=bf)
        Wt = torch.randn(1280, 7680, device=dev, dtype=bf) * 0.05
        W = Wt.t().contiguous()
        o = torch.empty(M, 1280, device=dev, dtype=bf)
        fl = 2.0 * M * 7680 * 1280
        cases[name + " | hipblaslt"] = (fl, lambda: torch.mm(dgx, W))
        for sp in (1, 2):
            cases[name + " | gemm8 rowrow S%d" % sp] = (fl, lambda sp=sp: G.gemm8(dgx, Wt, o, 0, splits=sp))
            cases[name + " | gemm8 colB S%d" % sp] = (fl, lambda sp=sp: G.gemm8(dgx, W, o, 0, b_col=True, splits=sp))
    # the whole deferred weight-gradient tail of a model (every layer's dW and both directions'
    # dU, distinct tensors per layer): one library call each vs one gemm8 call each vs ONE
    # grouped gemm8 launch (ops/rnn.py WgradScheduler.flush)
    for tag, GH, H, L in (("gru800", 2400, 800, 5), ("gru1280", 3840, 1280, 7), ("relu1760", 1760, 1760, 7)):
        name = "tail " + tag
        if a.only and a.only not in name:
            continue
        mem, fl = [], 0.0
        for li in range(L):
            D = 2400 if li == 0 else H if tag != "gru800" else 800
            dgh = torch.randn(2, M, GH, device=dev, dtype=bf)
            h = torch.randn(2, M, H, device=dev, dtype=bf)
            dgx = torch.randn(M, 2 * GH, device=dev, dtype=bf)
            x = torch.randn(M, D, device=dev, dtype=bf)
            mem += [(dgh[0], h[0], torch.empty(GH, H, device=dev)), (dgh[1], h[1], torch.empty(GH, H, device=dev)),
                    (dgx, x, torch.empty(2 * GH, D, device=dev))]
            fl += 2.0 * M * (2 * GH * H + 2 * GH * D)

        def lib(mem=mem):
            for A, B, o in mem:
                torch.mm(A.t(), B, out_dtype=torch.float32, out=o)

        def each(mem=mem):
            for A, B, o in mem:
                G.gemm8(A, B, o, 1, a_col=True, b_col=True)

        cases[name + " | hipblaslt"] = (fl, lib)
        cases[name + " | gemm8 each"] = (fl, each)
        cases[name + " | gemm8 group"] = (fl, lambda mem=mem: G.gemm8_group(mem))
        # the same group writing views of ONE gradient arena, then the optimizer over those
        # elements (separate streaming Adam + EMA launch) vs the fused optimizer epilogue
        n = sum(o.numel() for _, _, o in mem)
        ar = dict(g=torch.zeros(n, device=dev), p=torch.randn(n, device=dev), m=torch.zeros(n, device=dev),
                  v=torch.zeros(n, device=dev), e=torch.randn(n, device=dev),
                  p16=torch.zeros(n, device=dev, dtype=bf))
        amem, pos = [], 0
        for A, B, o in mem:
            amem.append((A, B, ar["g"][pos:pos + o.numel()].view_as(o)))
            pos += o.numel()
        Cx = _ext.ext()

        def sep(amem=amem, ar=ar):
            G.gemm8_group(amem)
            Cx.adam_ema(ar["p"], ar["g"], ar["m"], ar["v"], ar["e"], ar["p16"], 1e-4, 0.9, 0.999, 1e-8, 1.0, 0.999,
                        None, 0)
        opt = ([ar["p"], ar["m"], ar["v"], ar["e"], ar["p16"], ar["g"]], [1e-4, 0.9, 0.999, 1e-8, 1.0, 0.999], False)
        cases[name + " | gemm8 group + adam"] = (fl, sep)
        cases[name + " | gemm8 group fused adam"] = (fl, lambda amem=amem, opt=opt: G.gemm8_group(amem, opt=opt))
        cases[name + " | adam alone"] = (fl, lambda ar=ar: Cx.adam_ema(
            ar["p"], ar["g"], ar["m"], ar["v"], ar["e"], ar["p16"], 1e-4, 0.9, 0.999, 1e-8, 1.0, 0.999, None, 0))
    res = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, (fl, fn) in cases.items():
            res[k].append(timeit(fn))
    for k, (fl, _) in cases.items():
        best, med = min(res[k]), statistics.median(res[k])
        print(json.dumps({"case": k, "best_us": round(best, 1), "median_us": round(med, 1),
                          "tflops": round(fl / best / 1e6, 1)}))


if __name__ == "__main__":
    main()
