#!/usr/bin/env python3
"""Row-row projection / input-gradient GEMMs at the batch row counts of the SortaGrad buckets
(M = 32 x T2): every csrc/gemm.hip tile configuration against csrc/gemm8.hip with its launch
plan (ops/gemm.py gemm8_plan), HIP events, random bf16 data, best of 5 rounds.
  python tools/bench_gemm_small_m.py [--M 672,1312,2432,3712]
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
    ap.add_argument("--M", default="672,1312,2432,3712")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--cfg5", action="store_true", help="add the config-5 (H 1280) and FC-head shapes")
    a = ap.parse_args()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    shapes = [("proj L1", 4800, 800), ("proj L0", 4800, 2400), ("dx L1", 800, 4800), ("dx L0", 2400, 4800)]
    if a.cfg5:
        shapes += [("head", 32, 800), ("proj1280 L1", 7680, 1280), ("dx1280 L1", 1280, 7680)]
    cfgs = [0, 1, 2, 3, 4, 5, 6, 7, 8]
    print("| shape | M | routed us | gemm8 us | " + " | ".join("cfg%d" % c for c in cfgs) + " | best |")
    print("|---|---|---|---|" + "---|" * len(cfgs) + "---|")
    for M in [int(x) for x in a.M.split(",")]:
        for name, N, K in shapes:
            x = torch.randn(M, K, device=dev, dtype=bf)
            W = torch.randn(N, K, device=dev, dtype=bf) * 0.05
            b = torch.randn(N, device=dev, dtype=bf)
            o = torch.empty(M, N, device=dev, dtype=bf)
            fns = {"route": lambda: G.matmul(x, W.t(), o, bias=b), "g8": lambda: G.gemm8(x, W, o, 0, 1.0, b)}
            for c in cfgs:
                fns[c] = (lambda c=c: G.gemm(x, W, o, M, N, K, False, False, 0, 1.0, b, c))
            best = {k: 1e9 for k in fns}
            for _ in range(a.rounds):
                for k, f in fns.items():
                    best[k] = min(best[k], timeit(f))
            tr = best["route"]
            G.matmul(x, W.t(), o, bias=b)
            torch.cuda.synchronize()
            ref = x.float() @ W.float().t() + b.float()
            err = float((o.float() - ref).abs().max() / ref.abs().max())
            assert err < 2e-2, (name, M, err)
            del best["route"]
            win = min(best, key=best.get)
            print("| %s | %d | %.1f | %.1f | %s | %s |" % (name, M, tr, best["g8"],
                                                       " | ".join("%.1f" % best[c] for c in cfgs), win), flush=True)


if __name__ == "__main__":
    main()
