#!/usr/bin/env python3
"""Which PyTorch ops still launch device work inside a headline training step (VERDICT r5 weak
item 8: torch glue between the HIP kernels), with the Python stack that issued each.

  python tools/glue_ops.py [--frames 1000] [--steps 2]

Profiles a few steps after warm-up with torch.profiler (stacks on) and prints every aten op
that spent device time, grouped by its issuing stack, per step."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deepspeech_amd.utils.setenvs import setenvs  # noqa: E402

setenvs([])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--hidden", type=int, default=800)
    ap.add_argument("--layers", type=int, default=5)
    a = ap.parse_args()
    import torch
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.trainer import LRSchedule, Trainer
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=32, num_hidden=a.hidden, num_rnn_layers=a.layers, cell="gru").to(dev)
    m.set_engine("hip", torch.bfloat16)
    tr = Trainer(m, LRSchedule(1e-4, 10 ** 9, 0.9), defer_update=True)
    b = to_device(FixedShapeBatches(32, max_frames=a.frames, seed=0, pool=1).next(), dev)
    for _ in range(5):
        tr.step(b)
    torch.cuda.synchronize()
    # every aten op dispatched during the steps (TorchDispatchMode sees the ops autograd and the
    # fused ops' Python glue issue, with the issuing Python frame); views, allocations and
    # metadata ops launch nothing and are left out
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    quiet = ("view", "empty", "as_strided", "_reshape_alias", "detach", "t.", "transpose", "expand", "slice",
             "select", "unsqueeze", "squeeze", "permute", "alias", "split", "unbind", "_unsafe_view", "lift_fresh",
             "is_same_size", "set_", "record_stream", "reshape", "size", "stride", "numel", "dim", "sym_")
    agg = {}

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func.name())
            if not any(q in name for q in quiet):
                fr = [f for f in traceback.extract_stack()[:-1] if "deepspeech_amd" in f.filename or "tools" in f.filename]
                where = tuple("%s:%d %s" % (os.path.relpath(f.filename, ROOT), f.lineno, f.name) for f in fr[-3:])
                agg[(name, where)] = agg.get((name, where), 0) + 1
            return func(*args, **(kwargs or {}))
    with Log():
        for _ in range(a.steps):
            tr.step(b)
        tr.flush()
    torch.cuda.synchronize()
    print("aten ops dispatched per %d steps (count, op, issuing frames):" % a.steps)
    for (name, where), n in sorted(agg.items(), key=lambda kv: -kv[1]):
        print("%4d  %s" % (n, name))
        for w in where:
            print("          %s" % w)


if __name__ == "__main__":
    main()
