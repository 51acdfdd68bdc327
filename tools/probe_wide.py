#!/usr/bin/env python3
"""Residency / placement probe of the XCD recurrence kernels for a geometry: runs the forward
and then the BPTT once each (short spin timeout), reports each launch's error bits and, from
the census words the launch leaves behind, how many members of each group reported and on
which XCC.

  DS2_RNN_TIMEOUT_S=2 python tools/probe_wide.py --cell rnn_relu --H 1760 --N 32 --T 20
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cell", default="rnn_relu")
    ap.add_argument("--H", type=int, default=1760)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--T", type=int, default=20)
    ap.add_argument("--ndir", type=int, default=2)
    a = ap.parse_args()
    import torch
    from deepspeech_amd.ops import rnn as RNN
    dev = torch.device("cuda")
    plan = RNN.plan_for(a.N, a.H, a.cell, a.ndir, dev)
    print("plan", plan)
    G = RNN.GATES[a.cell]
    torch.manual_seed(0)
    gx = (torch.randn(a.T, a.N, a.ndir * G * a.H, device=dev) * 0.5).to(torch.bfloat16)
    lens = torch.full((a.N,), a.T, device=dev, dtype=torch.int32)
    U = [(torch.randn(G * a.H, a.H, device=dev) * 0.02).to(torch.bfloat16) for _ in range(a.ndir)]
    bh = [None, None]
    err = RNN.error_word(dev)
    seen = {}
    orig_af, orig_ab = RNN._alloc_fwd, RNN._alloc_bwd

    def alloc_fwd(*args, **kw):
        b = orig_af(*args, **kw)
        seen["census"] = b.census
        return b

    def alloc_bwd(*args, **kw):
        r = orig_ab(*args, **kw)
        seen["census"] = r[0]
        return r

    RNN._alloc_fwd, RNN._alloc_bwd = alloc_fwd, alloc_bwd
    P = a.H // 32

    for what in ("fwd", "bwd"):
        err.zero_()
        torch.cuda.synchronize()
        if what == "fwd":
            y, saved = RNN._run_fwd(gx, lens, U + [None] * (2 - a.ndir), bh, plan)
        else:
            hx, hs, gates = saved
            dy = (torch.randn(a.T, a.N, a.H, device=dev) * 0.1).to(torch.bfloat16)
            RNN._run_bwd(dy, lens, U + [None] * (2 - a.ndir), hx, hs, gates, plan, a.ndir * G * a.H)
        torch.cuda.synchronize()
        print(what, "error bits 0x%x" % int(err.item()))
        c = seen["census"].view(-1, P).cpu()
        for g in range(c.shape[0]):
            vals = [int(v) & 0xffffffff for v in c[g].tolist()]
            missing = [m for m, v in enumerate(vals) if v == 0xffffffff]
            hist = collections.Counter(v for v in vals if v != 0xffffffff)
            print("  group %d: %d/%d members reported, XCCs %s, missing members %s" %
                  (g, P - len(missing), P, dict(hist), missing[:16]))


if __name__ == "__main__":
    main()
