#!/usr/bin/env python3
"""What slows the BPTT kernel down when weight-gradient GEMMs run beside it?

Times ONE bidirectional GRU-800 layer's backward recurrence (B=32, T=241, headline shape)
alone and with a side-stream load running concurrently:
  dU       the recurrent weight-gradient batched GEMM exactly as the engine issues it
           (hipBLASLt, bf16 -> fp32, K = 7712: streams ~100 MB through L2),
  stream   a pure HBM streaming reduction (no reuse, L2 pollution only),
  compute  small L2-resident GEMMs (MFMA-bound, little HBM traffic; power / clock effect),
and prints the BPTT time per case (HIP events around the recurrence backward only).

  python tools/interference.py [--iters 10]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--H", type=int, default=800)
    a = ap.parse_args()
    from deepspeech_amd.ops import rnn as RNN
    dev = torch.device("cuda")
    N, H, T, G = 32, a.H, 241, 3
    plan = RNN.plan_for(N, H, "gru", 2, dev)
    torch.manual_seed(0)
    gx = (torch.randn(T, N, 2 * G * H, device=dev) * 0.5).bfloat16().requires_grad_(True)
    Us = [(torch.randn(G * H, H, device=dev) / H ** 0.5).bfloat16().requires_grad_(True) for _ in range(2)]
    bh = [torch.zeros(G * H, device=dev, requires_grad=True) for _ in range(2)]
    lens = torch.full((N,), T, dtype=torch.int32, device=dev)
    dy = torch.randn(T, N, H, device=dev).bfloat16()

    # side loads
    K = T * N
    g3 = torch.randn(2, G * H, K, device=dev).bfloat16()
    h3 = torch.randn(2, K, H, device=dev).bfloat16()
    out = torch.empty(2, G * H, H, device=dev)
    big = torch.randn(64 * 1024 * 1024, device=dev)           # 256 MB > MALL
    sa = torch.randn(8, 1024, 1024, device=dev).bfloat16()     # 16 MB working set, L2/MALL-resident
    sb = torch.randn(8, 1024, 1024, device=dev).bfloat16()
    side = torch.cuda.Stream()

    def load(kind):
        if kind == "dU":
            torch.bmm(g3, h3, out_dtype=torch.float32, out=out)
        elif kind == "dU_x2":
            for _ in range(2):
                torch.bmm(g3, h3, out_dtype=torch.float32, out=out)
        elif kind == "dU_x4":
            for _ in range(4):
                torch.bmm(g3, h3, out_dtype=torch.float32, out=out)
        elif kind == "stream":
            for _ in range(4):
                big.sum()
        elif kind == "compute":
            for _ in range(12):
                torch.bmm(sa, sb)

    def bptt_once(kind):
        y = RNN.BiRecurrence.apply(gx, lens, Us[0], Us[1], bh[0], bh[1], plan)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        side.wait_stream(torch.cuda.current_stream())
        e0.record()
        y.backward(dy)                                     # BPTT dispatched first, as in a step
        e1.record()
        if kind != "none":
            with torch.cuda.stream(side):
                s0.record()
                load(kind)
                s1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1), (s0.elapsed_time(s1) if kind != "none" else 0.0)

    # side-load times alone
    alone = {}
    for kind in ("dU", "dU_x2", "dU_x4", "stream", "compute"):
        load(kind)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        load(kind)
        e1.record()
        torch.cuda.synchronize()
        alone[kind] = round(e0.elapsed_time(e1), 4)
    kinds = ("none", "dU", "dU_x2", "dU_x4", "stream", "compute")
    res = {k: [] for k in kinds}
    side_t = {k: [] for k in kinds}
    for _ in range(2):
        for k in kinds:
            bptt_once(k)                                   # warm
    for _ in range(a.iters):
        for k in kinds:                                    # interleaved (rule 24)
            b, s = bptt_once(k)
            res[k].append(b)
            side_t[k].append(s)
    med = lambda v: sorted(v)[len(v) // 2]
    print(json.dumps({"bptt_ms": {k: round(med(v), 4) for k, v in res.items()},
                      "side_ms_concurrent": {k: round(med(v), 4) for k, v in side_t.items() if k != "none"},
                      "side_ms_alone": alone}))


if __name__ == "__main__":
    main()
