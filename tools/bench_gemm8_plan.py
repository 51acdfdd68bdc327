#!/usr/bin/env python3
"""gemm8 launch plans (ops/gemm.py gemm8_plan: parallel split-K reduction for few tiles) against
the plain split-K policy, on the row-row projection / input-gradient shapes of the DS2 configurations at the batch row counts of several
SortaGrad buckets (M = 32 x T2). HIP events, random bf16 data, interleaved rounds, best of;
every planned result is checked against an fp32 torch reference.

  python tools/bench_gemm8_plan.py [--rounds 5] [--M 672,3712,7712]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeech_amd.ops import gemm as G  # noqa: E402


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
    ap.add_argument("--M", type=str, default="672,1312,3712,5632,7712")
    a = ap.parse_args()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    shapes = [("proj800 L1", 4800, 800), ("proj800 L0", 4800, 2400), ("dx800 L1", 800, 4800),
              ("dx800 L0", 2400, 4800), ("proj1280 L1", 7680, 1280), ("dx1280 L1", 1280, 7680)]
    cus = G._dev_cus(torch.empty(1, device=dev))
    print("| shape | M | plan (S, ext_red) | plain us | planned us | plain TF/s | planned TF/s | max rel err |")
    print("|---|---|---|---|---|---|---|---|")
    for M in [int(x) for x in a.M.split(",")]:
        for name, N, K in shapes:
            plan = G.gemm8_plan(M, N, K, 1, cus)
            if plan is None:
                continue
            x = torch.randn(M, K, device=dev, dtype=bf)
            W = torch.randn(N, K, device=dev, dtype=bf) * 0.05
            b = torch.randn(N, device=dev, dtype=bf)
            o1 = torch.empty(M, N, device=dev, dtype=bf)
            o2 = torch.empty(M, N, device=dev, dtype=bf)
            plain = G.gemm8_splits(M, N, K, 1, cus)
            f1 = lambda: G.gemm8(x, W, o1, 0, 1.0, b, splits=plain)          # noqa: E731
            f2 = lambda: G.gemm8(x, W, o2, 0, 1.0, b)                        # noqa: E731
            f2()
            torch.cuda.synchronize()
            ref = (x.float() @ W.float().t() + b.float())
            err = float(((o2.float() - ref).abs().max() / ref.abs().max()))
            t1, t2 = [], []
            for _ in range(a.rounds):
                t1.append(timeit(f1))
                t2.append(timeit(f2))
            fl = 2.0 * M * N * K
            print("| %s | %d | %s | %.1f | %.1f | %.0f | %.0f | %.2e |" % (
                name, M, plan, min(t1), min(t2), fl / min(t1) / 1e6, fl / min(t2) / 1e6, err), flush=True)


if __name__ == "__main__":
    main()
