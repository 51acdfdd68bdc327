#!/usr/bin/env python3
"""Config 5's recurrence kernels on one bidirectional GRU layer, interleaved in one process
(HIP events, median of --iters): the fp8 forward (csrc/rnn_fp8.hip rnnf8h_fwd_kernel), the fp8
BPTT on its saved states (rnnf8_bwd_kernel: one XCD per group) and the bf16 reduce-scatter BPTT
on the same states (csrc/rnn_xcd.hip rnnrs_bwd_kernel, 40-workgroup groups across XCDs).

  python tools/bench_rnn_fp8.py [--H 1280] [--N 32] [--T 241] [--iters 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=1280)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--T", type=int, default=241)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from deepspeech_amd.ops import rnn as RNN
    dev = torch.device("cuda")
    H, N, T = a.H, a.N, a.T
    plan = RNN.plan_for(N, H, "gru", 2, dev)
    assert RNN.fp8_bptt_ok(plan, N), "geometry not served by the fp8 kernels"
    torch.manual_seed(0)
    gx = (torch.randn(T, N, 6 * H, device=dev) * 0.5).to(torch.bfloat16)
    lens = torch.full((N,), T, device=dev, dtype=torch.int32)
    U = [(torch.randn(3 * H, H, device=dev) * (1.5 / H ** 0.5)).to(torch.bfloat16) for _ in range(2)]
    bh = [torch.randn(3 * H, device=dev) * 0.1 for _ in range(2)]
    dy = torch.randn(T, N, H, device=dev).to(torch.bfloat16)
    state = {}

    def fwd():
        state["out"] = RNN._run_fwd_fp8(gx, lens, U, bh, plan)

    def bwd8():
        _, (hx, hs, gates) = state["out"]
        RNN._run_bwd_fp8(dy, lens, U, hs, gates, plan, 6 * H)

    def bwd16():
        _, (hx, hs, gates) = state["out"]
        RNN._run_bwd(dy, lens, U, hx, hs, gates, plan, 6 * H)

    cases = {"fwd fp8": fwd, "bptt fp8 (one XCD per group)": bwd8, "bptt bf16 (reduce-scatter)": bwd16}
    fwd()
    for fn in cases.values():
        fn()
    torch.cuda.synchronize()
    RNN.check_errors()
    times = {k: [] for k in cases}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.iters):
        for k, fn in cases.items():
            ev0.record()
            fn()
            ev1.record()
            torch.cuda.synchronize()
            times[k].append(ev0.elapsed_time(ev1))
    RNN.check_errors()
    for k, v in times.items():
        v.sort()
        ms = v[len(v) // 2]
        print(json.dumps({"case": k, "H": H, "N": N, "T": T, "ms_per_layer": round(ms, 4),
                          "us_per_step": round(1000 * ms / T, 3)}), flush=True)


if __name__ == "__main__":
    main()
