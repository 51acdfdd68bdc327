#!/usr/bin/env python3
"""Time the library GEMMs of one DS2 training step under alternative operand layouts.

  python tools/bench_gemm.py [--T2 241] [--N 32] [--H 800] [--D 2400]

For each GEMM (input projection, dx, dW, dU, head) every equivalent formulation
(operand transposes / swapped operands producing the transposed result) is timed with
HIP events, so the engine can pick the layout hipBLASLt runs fastest on MI355X.
"""
import argparse
import json

import torch


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T2", type=int, default=241)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--H", type=int, default=800)
    ap.add_argument("--D", type=int, default=2400)
    a = ap.parse_args()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    M = a.T2 * a.N
    GH2 = 2 * 3 * a.H
    res = []
    for D in (a.D, a.H):
        x = torch.randn(M, D, device=dev, dtype=bf)
        W = torch.randn(GH2, D, device=dev, dtype=bf)
        Wt = W.t().contiguous()
        b = torch.randn(GH2, device=dev, dtype=bf)
        dgx = torch.randn(M, GH2, device=dev, dtype=bf)
        dgxt = dgx.t().contiguous()
        xt = x.t().contiguous()
        fl = 2.0 * M * D * GH2
        cases = {
            "proj x@W^T (W [N,K])": lambda: torch.addmm(b, x, W.t()),
            "proj x@Wt (Wt [K,N])": lambda: torch.addmm(b, x, Wt),
            "proj (W@x^T)^T": lambda: torch.mm(W, x.t()),
            "dx dgx@W": lambda: torch.mm(dgx, W),
            "dx dgx@Wt^T": lambda: torch.mm(dgx, Wt.t()),
            "dx (W^T@dgx^T)^T": lambda: torch.mm(W.t(), dgx.t()),
            "dW dgx^T@x fp32out": lambda: torch.mm(dgx.t(), x, out_dtype=torch.float32),
            "dW (x^T@dgx)^T fp32out": lambda: torch.mm(x.t(), dgx, out_dtype=torch.float32),
            "dW dgxt@x fp32out (pre-transposed)": lambda: torch.mm(dgxt, x, out_dtype=torch.float32),
            "dW dgx^T@x bf16out": lambda: torch.mm(dgx.t(), x),
        }
        for k, f in cases.items():
            us = timeit(f)
            res.append({"K/D": D, "gemm": k, "us": round(us, 1), "TFLOPs": round(fl / us / 1e6, 1)})
    # dU per direction
    dgh = torch.randn(M, 3 * a.H, device=dev, dtype=bf)
    h = torch.randn(M, a.H, device=dev, dtype=bf)
    fl = 2.0 * M * 3 * a.H * a.H
    dgh2 = torch.randn(2, M, 3 * a.H, device=dev, dtype=bf)
    h2 = torch.randn(2, M, a.H, device=dev, dtype=bf)
    cases = {
        "dU dgh^T@h fp32out": lambda: torch.mm(dgh.t(), h, out_dtype=torch.float32),
        "dU (h^T@dgh)^T fp32out": lambda: torch.mm(h.t(), dgh, out_dtype=torch.float32),
        "dU dgh^T@h bf16out": lambda: torch.mm(dgh.t(), h),
        "dU both dirs bmm bf16out": lambda: torch.bmm(dgh2.transpose(1, 2), h2),
    }
    for k, f in cases.items():
        us = timeit(f)
        mult = 2 if "both" in k else 1
        res.append({"gemm": k, "us": round(us, 1), "TFLOPs": round(mult * fl / us / 1e6, 1)})
    # head
    hh = torch.randn(M, a.H, device=dev, dtype=bf)
    d = torch.randn(M, 29, device=dev, dtype=bf)
    res.append({"gemm": "head dW d^T@h fp32out", "us": round(timeit(lambda: torch.mm(d.t(), hh, out_dtype=torch.float32)), 1)})
    res.append({"gemm": "head dW (h^T@d)^T fp32out", "us": round(timeit(lambda: torch.mm(hh.t(), d, out_dtype=torch.float32)), 1)})
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
