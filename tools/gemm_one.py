#!/usr/bin/env python3
"""Run ONE csrc/gemm.hip configuration repeatedly (for rocprofv3 counter passes).

  python tools/gemm_one.py --shape proj800 --cfg 1 --iters 20
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeech_amd.ops import gemm as G  # noqa: E402

SHAPES = {   # name: (M, N, K, a_col, b_col, batch)
    "proj800": (7712, 4800, 800, False, False, 1),
    "proj2400": (7712, 4800, 2400, False, False, 1),
    "dx800": (7712, 800, 4800, False, True, 1),
    "dx800rr": (7712, 800, 4800, False, False, 1),
    "dW800": (4800, 800, 7712, True, True, 1),
    "dU": (2400, 800, 7712, True, True, 2),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="proj800", choices=sorted(SHAPES))
    ap.add_argument("--cfg", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    M, N, K, ac, bc, batch = SHAPES[a.shape]
    dev = torch.device("cuda")
    bf = torch.bfloat16
    sa = (K, M) if ac else (M, K)
    sb = (K, N) if bc else (N, K)
    if batch > 1:
        sa, sb = (batch,) + sa, (batch,) + sb
    A = torch.randn(sa, device=dev).to(bf)
    B = torch.randn(sb, device=dev).to(bf)
    epi = 1 if ac else 0
    C = torch.empty(((batch,) if batch > 1 else ()) + (M, N), device=dev,
                    dtype=torch.float32 if epi else bf)
    for _ in range(a.iters):
        G.gemm(A, B, C, M, N, K, ac, bc, epi, 1.0, None, a.cfg)
    torch.cuda.synchronize()
    print("done", a.shape, a.cfg)


if __name__ == "__main__":
    main()
