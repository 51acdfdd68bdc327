#!/usr/bin/env python3
"""gemm8 time against K at a fixed M x N (default the BiGRU-800 projection 7712 x 4800): splits
the per-tile cost into a fixed part (prologue, epilogue, scheduling) and a per-k-tile part.

  python tools/gemm8_ksweep.py [--M 7712 --N 4800] [--grid 0]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeech_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=241 * 32)
    ap.add_argument("--N", type=int, default=4800)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--epi", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for K in (64, 128, 256, 512, 800, 1600, 3200, 6400):
        x = torch.randn(a.M, K, device=dev, dtype=torch.bfloat16)
        W = torch.randn(a.N, K, device=dev, dtype=torch.bfloat16)
        o = torch.empty(a.M, a.N, device=dev, dtype=torch.bfloat16 if a.epi == 0 else torch.float32)
        us = min(timeit(lambda: G.gemm8(x, W, o, epi=a.epi, splits=1, max_grid=a.grid)) for _ in range(3))
        tiles = -(-a.M // 256) * -(-a.N // 256)
        print(json.dumps({"M": a.M, "N": a.N, "K": K, "us": round(us, 1), "tiles": tiles,
                          "tflops": round(2.0 * a.M * a.N * K / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
