#!/usr/bin/env python3
"""Minimal driver for rocprofv3 counter passes over csrc/gemm8.hip: the grouped weight-gradient
tail of the 7 x bi-ReLU-1760 model (column-column operands) and a row-row projection of the same
FLOP scale, a few launches each (kernel names tell the two apart: gemm8_kernel<false,1,1> /
<false,0,0>).

  rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- python3 tools/prof_gemm8.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeech_amd.ops import gemm as G  # noqa: E402


def main():
    dev, bf, M = torch.device("cuda"), torch.bfloat16, 241 * 32
    mem = []
    for li in range(7):
        D = 2400 if li == 0 else 1760
        dgh = torch.randn(2, M, 1760, device=dev, dtype=bf)
        h = torch.randn(2, M, 1760, device=dev, dtype=bf)
        dgx = torch.randn(M, 3520, device=dev, dtype=bf)
        x = torch.randn(M, D, device=dev, dtype=bf)
        mem += [(dgh[0], h[0], torch.empty(1760, 1760, device=dev)), (dgh[1], h[1], torch.empty(1760, 1760, device=dev)),
                (dgx, x, torch.empty(3520, D, device=dev))]
    x = torch.randn(M, 1760, device=dev, dtype=bf)
    W = torch.randn(7680, 1760, device=dev, dtype=bf)
    o = torch.empty(M, 7680, device=dev, dtype=bf)
    for _ in range(3):
        G.gemm8_group(mem)
        G.gemm8(x, W, o, 0, 1.0, None, splits=1)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
