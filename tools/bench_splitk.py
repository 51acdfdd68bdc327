#!/usr/bin/env python3
"""Split-K weight gradients: time dW = dgx^T x / dU = dgh^T h as one hipBLASLt GEMM against
S-way K-split strided-batched GEMMs (fp32 partials) + a sum over the split.

  python tools/bench_splitk.py [--T2 241] [--N 32] [--H 800]

The headline's weight-gradient outputs are small (4800 x 800) against a long K (T2 * N =
7712): 256x128 output tiles give 133 workgroups for 256 CUs, so the tail GEMMs that run after
the last BPTT (deferred dW of layers 1-4, dW_0, dU_0) leave half the chip idle. A K-split
multiplies the tile count by S at the cost of S fp32 partial planes through HBM.
"""
import argparse
import json

import torch


def timeit(fn, iters=30):
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
    a = ap.parse_args()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    K = a.T2 * a.N
    GH2 = 6 * a.H
    res = []
    for name, rows, cols, batch in (("dW D=H", GH2, a.H, 1), ("dW D=2400", GH2, 2400, 1),
                                    ("dU 2 dirs", 3 * a.H, a.H, 2)):
        g = torch.randn(batch, K, rows, device=dev, dtype=bf)
        x = torch.randn(batch, K, cols, device=dev, dtype=bf)
        out = torch.empty(batch, rows, cols, device=dev, dtype=torch.float32)
        ref = torch.bmm(g.float().transpose(1, 2), x.float())
        flops = 2.0 * batch * rows * cols * K
        for S in (1, 2, 3, 4, 8):
            if K % S:
                continue
            k = K // S
            # split index outermost so each split is a contiguous K range of every batch
            gs = g.view(batch, S, k, rows).transpose(0, 1).reshape(S * batch, k, rows) if batch > 1 \
                else g.view(S, k, rows)
            xs = x.view(batch, S, k, cols).transpose(0, 1).reshape(S * batch, k, cols) if batch > 1 \
                else x.view(S, k, cols)
            part = torch.empty(S, batch, rows, cols, device=dev, dtype=torch.float32)

            def run(S=S, gs=gs, xs=xs, part=part):
                if S == 1:
                    torch.bmm(g.transpose(1, 2), x, out_dtype=torch.float32, out=out)
                else:
                    torch.bmm(gs.transpose(1, 2), xs, out_dtype=torch.float32,
                              out=part.view(S * batch, rows, cols))
                    torch.sum(part, dim=0, out=out)
            us = timeit(run)
            err = float((out - ref).abs().max() / ref.abs().max())
            res.append({"gemm": name, "split": S, "us": round(us, 1),
                        "tflops": round(flops / us * 1e-6, 1), "rel_err": err})
            print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
