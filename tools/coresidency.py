#!/usr/bin/env python3
"""Does the persistent recurrence stay co-resident (no spin timeout) while RCCL-like channel
blocks hold CUs?  DP-readiness check on ONE GPU.

A headline recurrence layer (bidirectional GRU-800, B=32, T2=241: 200 co-resident
workgroups) runs forward + BPTT while a second stream runs ``blocks`` spinning workgroups
(csrc/stats.hip spin_kernel, ``threads`` threads and ``lds`` bytes of LDS each) for
``spin_ms`` — the footprint of an all-reduce's RCCL channels. Orders:
  before  the spinners are launched first (a bucket all-reduce in flight when the layer starts)
  after   the layer is launched first (an all-reduce issued from a backward hook)
Prints one JSON line per case: layer ms, spin ms, and whether any recurrence kernel hit its
spin timeout (RNN.check_errors()).

  python tools/coresidency.py [--blocks 32 64] [--spin_ms 2] [--iters 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def run(blocks_list, threads, lds, spin_ms, iters, H=800, N=32, T=241, fp8=False):
    """fp8: a whole BiGRU layer of BASELINE config 5's fp8 mode instead (e4m3 forward
    recurrence and fp8 BPTT, csrc/rnn_fp8.hip; input projection and weight gradients
    included), H = 1280 by default there."""
    from deepspeech_amd.ops import _ext
    from deepspeech_amd.ops import rnn as RNN
    C = _ext.ext()
    dev = torch.device("cuda")
    G = 3
    torch.manual_seed(0)
    lens = torch.full((N,), T, dtype=torch.int32, device=dev)
    dy = torch.randn(T, N, H, device=dev).bfloat16()
    done = torch.zeros(1, device=dev, dtype=torch.int32)
    side = torch.cuda.Stream()
    ticks = int(spin_ms * 1e5)           # s_memrealtime: 100 MHz
    if fp8:
        from deepspeech_amd.models import DeepSpeech2
        m = DeepSpeech2(num_filters=32, num_hidden=H, num_rnn_layers=2, cell="gru").to(dev)
        m.set_engine("hip", torch.bfloat16, fp8=True)
        lay = m.rnn[1]
        x = (torch.randn(T, N, H, device=dev) * 0.5).bfloat16().requires_grad_(True)

        def layer():
            y = RNN.recurrent_layer_hip(lay, x, lens, 1)
            y.backward(dy)
            RNN.join_wgrad_streams()
    else:
        plan = RNN.plan_for(N, H, "gru", 2, dev)
        gx = (torch.randn(T, N, 2 * G * H, device=dev) * 0.5).bfloat16().requires_grad_(True)
        Us = [(torch.randn(G * H, H, device=dev) / H ** 0.5).bfloat16().requires_grad_(True) for _ in range(2)]
        bh = [torch.zeros(G * H, device=dev, requires_grad=True) for _ in range(2)]

        def layer():
            y = RNN.BiRecurrence.apply(gx, lens, Us[0], Us[1], bh[0], bh[1], plan)
            y.backward(dy)

    def case(blocks, order):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        side.wait_stream(torch.cuda.current_stream())

        def spin():
            with torch.cuda.stream(side):
                s0.record()
                C.spin(ticks, blocks, threads, lds, done)
                s1.record()
        if blocks and order == "before":
            spin()
        e0.record()
        layer()
        e1.record()
        if blocks and order == "after":
            spin()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1), (s0.elapsed_time(s1) if blocks else 0.0)

    for _ in range(2):
        case(0, "none")
    torch.cuda.synchronize()
    RNN.check_errors()
    out = []
    base = sorted(case(0, "none")[0] for _ in range(iters))[iters // 2]
    for blocks in blocks_list:
        for order in ("before", "after"):
            ts, ss = [], []
            err = None
            for _ in range(iters):
                t, s = case(blocks, order)
                ts.append(t)
                ss.append(s)
            try:
                RNN.check_errors()
            except RuntimeError as e:
                err = str(e)
            out.append({"blocks": blocks, "threads": threads, "lds": lds, "spin_ms": spin_ms, "order": order,
                        "layer_ms": round(sorted(ts)[iters // 2], 4), "layer_ms_alone": round(base, 4),
                        "spin_ms_measured": round(sorted(ss)[iters // 2], 4), "timeout": err})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, nargs="+", default=[32, 64])
    ap.add_argument("--threads", type=int, default=256)
    ap.add_argument("--lds", type=int, default=16384)
    ap.add_argument("--spin_ms", type=float, default=2.0)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    for r in run(a.blocks, a.threads, a.lds, a.spin_ms, a.iters):
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
