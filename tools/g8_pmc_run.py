#!/usr/bin/env python3
"""A few launches of one GEMM for a rocprofv3 --pmc pass (scripts/pmc_gemm.sh):
  python tools/g8_pmc_run.py --M 7712 --N 4800 --K 800 [--impl gemm8|cfg7]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeech_amd.ops import gemm as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=7712)
ap.add_argument("--N", type=int, default=4800)
ap.add_argument("--K", type=int, default=800)
ap.add_argument("--impl", default="gemm8")
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda")
x = torch.randn(a.M, a.K, device=dev, dtype=torch.bfloat16)
W = torch.randn(a.N, a.K, device=dev, dtype=torch.bfloat16) * 0.05
b = torch.randn(a.N, device=dev, dtype=torch.bfloat16)
o = torch.empty(a.M, a.N, device=dev, dtype=torch.bfloat16)
for _ in range(a.iters):
    if a.impl == "gemm8":
        G.gemm8(x, W, o, 0, 1.0, b, splits=1)
    else:
        G.gemm(x, W, o, a.M, a.N, a.K, False, False, 0, 1.0, b, int(a.impl[3:]))
torch.cuda.synchronize()
print("ok")
