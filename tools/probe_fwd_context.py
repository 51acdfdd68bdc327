#!/usr/bin/env python3
"""Does what runs before the persistent forward recurrence change its time? Times one BiGRU-800
forward recurrence (headline shape) with HIP events in three contexts: right behind another
forward, right behind a projection-sized gemm8 (MFMA-heavy), and behind an idle gap.

  python tools/probe_fwd_context.py [--K 2400]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=2400)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--grad", action="store_true", help="training mode: activations saved for BPTT")
    a = ap.parse_args()
    from deepspeech_amd.ops import rnn as RNN
    from deepspeech_amd.ops import gemm as G
    dev = torch.device("cuda")
    N, H, T = 32, 800, 241
    plan = RNN.plan_for(N, H, "gru", 2, dev)
    rg = a.grad
    gx = (torch.randn(T, N, 2 * 3 * H, device=dev) * 0.5).bfloat16().requires_grad_(rg)
    Us = [(torch.randn(3 * H, H, device=dev) / H ** 0.5).bfloat16().requires_grad_(rg) for _ in range(2)]
    bh = [torch.zeros(3 * H, device=dev, requires_grad=rg) for _ in range(2)]
    lens = torch.full((N,), T, dtype=torch.int32, device=dev)
    x = torch.randn(T * N, a.K, device=dev, dtype=torch.bfloat16)
    W = torch.randn(6 * H, a.K, device=dev, dtype=torch.bfloat16)
    o = torch.empty(T * N, 6 * H, device=dev, dtype=torch.bfloat16)

    def fwd():
        with torch.set_grad_enabled(rg):
            return RNN.BiRecurrence.apply(gx, lens, Us[0], Us[1], bh[0], bh[1], plan)

    def gemm():
        G.gemm8(x, W, o, epi=0, splits=1)

    def idle():
        torch.cuda._sleep(2_000_000)

    for _ in range(3):
        fwd(), gemm()
    torch.cuda.synchronize()
    res = {}
    for name, pre in (("after fwd", fwd), ("after gemm8", gemm), ("after idle", idle),
                      ("after 2x gemm8", lambda: (gemm(), gemm())), ("after fwd", fwd)):
        ts = []
        for _ in range(a.iters):
            pre()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fwd()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) * 1000.0)
        ts.sort()
        res[name] = ts[len(ts) // 2]
        print(json.dumps({"context": name, "median_us": round(ts[len(ts) // 2], 1), "min_us": round(ts[0], 1)}),
              flush=True)


if __name__ == "__main__":
    main()
