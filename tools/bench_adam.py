#!/usr/bin/env python3
"""Fused Adam + EMA + bf16 shadow over a headline-sized arena (46.2 M parameters): time per
step and effective HBM bandwidth (38 B/parameter: p, g, m, v, ema read; p, m, v, ema and
the bf16 copy written).   python tools/bench_adam.py [--n 46200000]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from deepspeech_amd.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=46_200_000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--grids", type=str, default="0",
                    help="max_grid values to time (0: the kernel's default; -G: block-contiguous with G blocks)")
    ap.add_argument("--rounds", type=int, default=1)
    a = ap.parse_args()
    C = _ext.ext()
    d = torch.device("cuda")
    p, g, m, v, e = (torch.randn(a.n, device=d) for _ in range(5))
    v.abs_()
    p16 = torch.empty(a.n, device=d, dtype=torch.bfloat16)
    grids = [int(x) for x in a.grids.split(",")]
    for grid in grids * a.rounds:          # interleaved rounds (box drift)
        fn = lambda: C.adam_ema(p, g, m, v, e, p16, 1e-4, 0.9, 0.999, 1e-8, 1.0, 0.999, None, grid)  # noqa: E731
        for _ in range(3):
            fn()
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(a.iters):
            fn()
        t.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(t) / a.iters * 1e3
        print(json.dumps({"so": os.environ.get("DS2_EXT_SO", "in-tree"), "max_grid": grid, "us": round(us, 1),
                          "TBps": round(38 * a.n / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
