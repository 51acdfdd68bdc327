#!/usr/bin/env python3
"""Find the first step at which two trainers on the same batches stop being bitwise equal.

  python tools/graph_diverge.py --mode auto|graph|sync [--frames 100,300] [--H 256]

mode auto / graph: Trainer(step_graphs=...) against the eager Trainer; mode sync: an eager
Trainer that synchronises the device after every step against one that never does (a
timing-dependent race in the eager multi-stream step shows up there).
"""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="auto")
    ap.add_argument("--frames", default="100,300")
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--N", type=int, default=8)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--nosync", action="store_true", help="compare only at the end")
    ap.add_argument("--no_env", action="store_true", help="do not apply utils/setenvs.py")
    ap.add_argument("--tail", type=int, default=0, help="extra alternating steps over the shapes at the end")
    a = ap.parse_args()
    if not a.no_env:
        from deepspeech_amd.utils.setenvs import setenvs
        setenvs([])
    import torch
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.trainer import LRSchedule, Trainer
    dev = torch.device("cuda:0")
    torch.manual_seed(2)
    base = DeepSpeech2(num_filters=32, num_hidden=a.H, num_rnn_layers=a.layers, cell="gru").to(dev)
    frames = [int(x) for x in a.frames.split(",")]
    feeds = {T: FixedShapeBatches(a.N, max_frames=T, seed=T, pool=2) for T in frames}
    order = [T for T in frames for _ in range(a.steps)] + [frames[i % len(frames)] for i in range(a.tail)]

    def pad(b):
        S = b["labels"].shape[1]
        b = dict(b)
        b["labels"] = torch.nn.functional.pad(b["labels"], (0, 32 * (-(-S // 32)) - S))
        return b
    batches = [pad(to_device(feeds[T].next(), dev)) for T in order]
    A = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), LRSchedule(1e-3, 4, 0.7))
    kw = {} if a.mode == "sync" else {"step_graphs": (a.mode if a.mode == "auto" else True), "graph_warmup": 1}
    B = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), LRSchedule(1e-3, 4, 0.7), **kw)
    names = ["flat", "grad", "m", "v", "ema", "p16"]
    for i, b in enumerate(batches):
        la = A.step(b)
        lb = B.step(b)
        if a.nosync and i + 1 < len(batches):
            continue
        torch.cuda.synchronize()
        sa = [A.arena.flat, A.arena.grad, A.opt.m, A.opt.v, A.opt.ema, A.arena.p16]
        sb = [B.arena.flat, B.arena.grad, B.opt.m, B.opt.v, B.opt.ema, B.arena.p16]
        bad = []
        for n, x, y in zip(names, sa, sb):
            if not torch.equal(x, y):
                d = (x.float() - y.float()).abs()
                idx = int(d.argmax())
                pname = next((nm for nm, (o, c) in zip(A.arena.names, A.arena.offsets) if o <= idx < o + c), "?")
                bad.append("%s(max %.3g at %s, %d elems)" % (n, float(d.max()), pname, int((d > 0).sum())))
        st = B._shapes.get(B.graph_key(b)) if hasattr(B, "_shapes") else None
        phase = "" if st is None else "mode=%s seen=%d spans=%d graph=%s" % (st.mode, st.seen, len(st.spans), st.graph is not None)
        print("step %2d T=%d loss %s %s | %s %s" % (i, b["feats"].shape[1], float(la), float(lb),
                                                   "OK" if not bad else "DIFF " + " ".join(bad), phase), flush=True)
    print("modes", getattr(B, "graph_modes", None))


if __name__ == "__main__":
    main()
