#!/usr/bin/env python3
"""Per-tile phase times of the persistent conv2 forward / data-gradient kernels at the headline
geometry (batch 32, 1000 frames): the kernels' optional trace stamps (s_memrealtime, 100 MHz) of
workgroups 0..7, wave 0, for their first 16 tiles -> median microseconds per phase.

  python tools/conv_timeline.py [--N 32] [--T 1000]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

PHASES = ("wait rows", "mfma loop", "reduce", "epilogue", "issue next")


def summarize(tr):
    t = tr.view(8, 16, 6).double() / 100.0            # us
    out = {}
    for k, name in enumerate(PHASES):
        d = (t[:, :, k + 1] - t[:, :, k]).flatten()
        d = d[(t[:, :, 0].flatten() > 0) & (d >= 0)]
        out[name] = round(d.median().item(), 3) if d.numel() else None
    tile = (t[:, 1:, 0] - t[:, :-1, 0]).flatten()
    tile = tile[(t[:, 1:, 0].flatten() > 0) & (t[:, :-1, 0].flatten() > 0)]
    out["tile period"] = round(tile.median().item(), 3) if tile.numel() else None
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--T", type=int, default=1000)
    a = ap.parse_args()
    from deepspeech_amd.ops import _ext
    C_ = _ext.ext()
    dev = torch.device("cuda")
    ncu = _ext.num_cus(0)
    T1, F1 = (a.T - 20) // 2 + 1, 79
    T2, F2 = (T1 - 10) // 2 + 1, 75
    N = a.N
    torch.manual_seed(0)
    x = torch.rand(N, T1, F1, 32, device=dev).bfloat16()
    w = (torch.randn(32, 32, 10, 5, device=dev) * 0.05).bfloat16()
    b = torch.randn(32, device=dev)
    y = torch.empty(N, T2, F2, 32, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(N, T2, F2, 32, device=dev).bfloat16()
    dx = torch.empty(N, T1, F1, 32, device=dev, dtype=torch.bfloat16)
    grid = 2 * ncu
    part = torch.empty(grid * 64, device=dev)
    mean, inv = torch.zeros(32, device=dev), torch.ones(32, device=dev)
    g, be = torch.ones(32, device=dev), torch.zeros(32, device=dev)
    for name, run in (("conv2_fwd", lambda tr: C_.conv2_fwd(x, w, b, y, part, grid, tr)),
                      ("conv2_dgrad", lambda tr: C_.conv2_dgrad(dy, w, dx, grid, None, None, None, None, None,
                                                                None, tr)),
                      ("conv2_dgrad+bn", lambda tr: C_.conv2_dgrad(dy, w, dx, grid, x, mean, inv, g, be, part,
                                                                   tr))):
        tr = torch.zeros(8 * 16 * 6, device=dev, dtype=torch.int64)
        run(None)
        run(tr)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(5):
            run(None)
        ev1.record()
        torch.cuda.synchronize()
        rec = {"kernel": name, "us": round(ev0.elapsed_time(ev1) / 5 * 1e3, 1), "grid": grid}
        rec.update(summarize(tr.cpu()))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
