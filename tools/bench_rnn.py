#!/usr/bin/env python3
"""Micro-benchmark + phase breakdown of the persistent recurrence kernels.

  python tools/bench_rnn.py [--cell gru] [--H 800] [--N 32] [--T 241] [--stamps]

Times forward and backward of ONE bidirectional layer (the recurrence only) with HIP
events, interleaving the variants in one process (cdna_hip_programming.md §5.4 rule 24).
With --stamps, re-runs the s_memtime diagnostic build and prints the average cycles per
step in each phase (wait / load+MFMA / reduce / epilogue / publish / rest) over all
workgroups — read the SHARES, not the absolute time, of that build.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

PHASES = ["wait", "load+mfma", "reduce", "epilogue", "publish", "rest(stores+prefetch)"]
# csrc/rnn_xcd.hip stamps: wave 0 phases + the memory wave's duty time and its barrier-#2 wait
XPHASES = ["gather(w0)", "sync1", "mfma(w0)", "sync2", "epilogue", "(mode)", "memwave duties", "memwave sync1"]


def run(cell, N, H, T, ndir, nw, mode, iters, stamps=False):
    from deepspeech_amd.ops import rnn as RNN
    dev = torch.device("cuda")
    RNN._FORCE_NW = nw if nw else 0
    os.environ["DS2_RNN_MODE"] = mode
    RNN._plan_cache.clear()
    plan = RNN.plan_for(N, H, cell, ndir, dev)
    G = RNN.GATES[cell]
    torch.manual_seed(0)
    gx = (torch.randn(T, N, ndir * G * H, device=dev) * 0.5).bfloat16().requires_grad_(True)
    Us = [(torch.randn(G * H, H, device=dev) / H ** 0.5).bfloat16().requires_grad_(True) for _ in range(ndir)]
    bh = [torch.zeros(G * H, device=dev, requires_grad=True) if cell == "gru" else None for _ in range(ndir)]
    lens = torch.full((N,), T, dtype=torch.int32, device=dev)
    dy = torch.randn(T, N, H, device=dev).bfloat16()

    def fwd():
        return RNN.BiRecurrence.apply(gx, lens, Us[0], Us[1] if ndir == 2 else None, bh[0],
                                      bh[1] if ndir == 2 else None, plan)

    if stamps:
        RNN.STAMP_LOG = []
    y = fwd()
    y.backward(dy)
    torch.cuda.synchronize()
    RNN.check_errors()
    res = {"plan": plan.__dict__}
    if stamps:
        log = RNN.STAMP_LOG
        RNN.STAMP_LOG = None
        for kind, p, t in log:
            names = XPHASES if p.kind == "xcd" else PHASES
            w = t[:, :len(names)].double() / T
            active = w.sum(1) > 0
            w = w[active]
            if w.shape[0] == 0:            # this kernel records no stamps
                continue
            res[kind + "_cycles_per_step"] = {ph: [round(float(w[:, i].mean()), 0), round(float(w[:, i].min()), 0),
                                                   round(float(w[:, i].max()), 0)] for i, ph in enumerate(names)}
            if p.kind == "xcd":
                # slot 5 of wave 0 holds the census verdict + 10 (11: XCD-local plain stores, 10: sc1)
                modes = t[:, 5][active].tolist()
                res[kind + "_groups_xcd_local"] = "%d of %d workgroups" % (sum(1 for m in modes if m == 11), len(modes))
        return res
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    tf, tb = [], []
    for _ in range(iters):
        ev[0].record()
        y = fwd()
        ev[1].record()
        ev[2].record()
        y.backward(dy)
        ev[3].record()
        torch.cuda.synchronize()
        tf.append(ev[0].elapsed_time(ev[1]))
        tb.append(ev[2].elapsed_time(ev[3]))
    RNN.check_errors()
    tf.sort(), tb.sort()
    res.update(fwd_ms=tf[len(tf) // 2], bwd_ms=tb[len(tb) // 2],
               fwd_us_per_step=1000 * tf[len(tf) // 2] / T, bwd_us_per_step=1000 * tb[len(tb) // 2] / T)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cell", default="gru")
    ap.add_argument("--H", type=int, default=800)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--T", type=int, default=241)
    ap.add_argument("--ndir", type=int, default=2)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--nw", type=str, default="0,4,8")
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--kernels", type=str, default="xcd,v1", help="recurrence generations to time")
    ap.add_argument("--knobs", type=str, default="0", help="xcd diagnostic knob sets to time (results are "
                    "wrong when set). Forward: 1 no prefetch, 2 no deferred stores, 4 no MFMA. Reduce-scatter "
                    "BPTT: 4 no exchange wait, 8 no publish MFMA, 32 no publish stores (with 4), 64 fp32 "
                    "partials instead of tagged bf16 (results correct)")
    a = ap.parse_args()
    if any(int(k) & 46 for k in a.knobs.split(",")):   # timing-only bits 2 | 4 | 8 | 32 (ops/rnn.py)
        os.environ["DS2_TIMING_ONLY"] = "1"
    for proto in a.kernels.split(","):
      for nw in ([int(x) for x in a.nw.split(",")] if proto == "v1" else [int(k) for k in a.knobs.split(",")]):
        if proto == "xcd":
            RNN_mod = __import__("deepspeech_amd.ops.rnn", fromlist=["x"])
            RNN_mod.RNNX_KNOBS = nw
        for mode in (("v1",) if proto == "v1" else ("auto",)):
            try:
                r = run(a.cell, a.N, a.H, a.T, a.ndir, nw, mode, a.iters)
                print(json.dumps({"kernel": proto, "nw": nw, "mode": mode,
                                  **{k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}}), flush=True)
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"kernel": proto, "nw": nw, "mode": mode, "error": str(e)[:200]}), flush=True)
      if a.stamps:
        if proto == "xcd":
            __import__("deepspeech_amd.ops.rnn", fromlist=["x"]).RNNX_KNOBS = int(os.environ.get("DS2_RNNX_KNOBS", "0"))
        r = run(a.cell, a.N, a.H, a.T, a.ndir, 0, "auto", 1, stamps=True)
        print(json.dumps({"kernel": proto, "stamps [mean,min,max] cycles/step": r}), flush=True)


if __name__ == "__main__":
    main()
