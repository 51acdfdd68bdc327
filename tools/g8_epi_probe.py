#!/usr/bin/env python3
"""Time gemm8 projection shapes in this process's extension (DS2_EXT_SO selects a variant build):
  DS2_EXT_SO=ab/_C_nostore....so python tools/g8_epi_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeech_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


dev = torch.device("cuda")
for (M, N, K) in [(7712, 4800, 800), (7712, 4800, 1600), (7712, 4800, 2400), (7712, 7680, 1280)]:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    t = min(timeit(lambda: G.gemm8(x, W, o, 0, 1.0, b, splits=1)) for _ in range(5))
    print("%s M=%d N=%d K=%d: %.1f us (%.0f TF/s)" % (os.path.basename(os.environ.get("DS2_EXT_SO", "in-tree")), M, N, K,
                                                   t, 2.0 * M * N * K / t / 1e6), flush=True)
