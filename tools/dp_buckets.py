#!/usr/bin/env python3
"""Per-bucket timing of the data-parallel gradient path on ONE GPU (world size 1 over RCCL,
``--force_dp`` machinery): for every gradient bucket of the headline model, the bytes it
puts on the wire, when its collective is issued on the ordering stream (= when its last
gradient landed) and when the collective and its per-bucket Adam range finished, all in ms
from the start of the step's backward. Markdown table on stdout.

  python tools/dp_buckets.py [--bucket_mb 32] [--steps 5] [--allreduce_bf16]

Device events are recorded on the ordering stream around each collective (GradBucketer.
_collective) and around each optimizer range, and on the main stream at the start of
backward; the numbers are the median over --steps timed steps.
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeech_amd.utils.setenvs import setenvs  # noqa: E402

setenvs([])          # the hardware-queue floor and RCCL settings, before HIP initialises


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bucket_mb", type=float, default=32.0)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--allreduce_bf16", action="store_true")
    ap.add_argument("--num_hidden", type=int, default=800)
    ap.add_argument("--num_rnn_layers", type=int, default=5)
    a = ap.parse_args()
    import torch
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.parallel import grad_sync as GS
    from deepspeech_amd.parallel.dist import init_distributed, shutdown
    from deepspeech_amd.trainer import LRSchedule, Trainer

    ctx = init_distributed("cuda", force_group=True)
    dev = ctx.device
    torch.manual_seed(0)
    model = DeepSpeech2(num_filters=32, num_hidden=a.num_hidden, num_rnn_layers=a.num_rnn_layers, cell="gru",
                        stack_fix=True, seq_bn="frozen").to(dev)
    model.set_engine("hip", torch.bfloat16)
    tr = Trainer(model, LRSchedule(1e-4, 10 ** 9, 0.9), moving_avg_decay=0.9999, world_size=1,
                 bucket_mb=a.bucket_mb, allreduce_bf16=a.allreduce_bf16, force_buckets=True)
    bk = tr.bucketer
    rec = {}

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    orig_coll = GS.GradBucketer._collective

    def coll(self, b, g):
        rec.setdefault(b, {})["issue"] = ev()          # on the ordering stream
        w = orig_coll(self, b, g)
        w.wait()                                       # ordering stream waits for the collective
        rec[b]["done"] = ev()
        return w

    GS.GradBucketer._collective = coll
    orig_set = bk.set_optimizer

    def set_opt(fn):
        def timed(lo, hi):
            b = next(i for i, (s, e, _) in enumerate(bk.buckets) if s == lo)
            rec.setdefault(b, {})["opt0"] = ev()
            fn(lo, hi)
            rec[b]["opt1"] = ev()
        orig_set(timed)

    bk.set_optimizer = set_opt
    batch = to_device(FixedShapeBatches(32, max_frames=1000, seed=1, pool=1).next(), dev)
    orig_backward = torch.Tensor.backward
    t0 = {}

    def backward(self, *args, **kw):
        t0["e"] = ev()
        return orig_backward(self, *args, **kw)

    torch.Tensor.backward = backward
    for _ in range(3):
        tr.step(batch)
    rows = {}
    for _ in range(a.steps):
        rec.clear()
        tr.step(batch)
        torch.cuda.synchronize()
        for b, r in rec.items():
            d = rows.setdefault(b, {"issue": [], "done": [], "opt1": []})
            for k in d:
                if k in r:
                    d[k].append(t0["e"].elapsed_time(r[k]))
    torch.Tensor.backward = orig_backward
    names = tr.arena.names
    print("| bucket | parameters | MB on the wire | issued (ms after backward start) | all-reduce done | "
          "Adam range done |")
    print("|---|---|---|---|---|---|")
    es = 2 if a.allreduce_bf16 else 4
    for b, (s, e, idx) in enumerate(bk.buckets):
        d = rows.get(b, {})
        med = {k: (statistics.median(v) if v else float("nan")) for k, v in d.items()}
        ps = ", ".join(names[i] for i in idx)
        if len(ps) > 60:
            ps = "%s ... %s (%d)" % (names[idx[0]], names[idx[-1]], len(idx))
        print("| %d | %s | %.2f | %.3f | %.3f | %.3f |" % (b, ps, (e - s) * es / 2 ** 20, med.get("issue", float("nan")),
                                                        med.get("done", float("nan")),
                                                        med.get("opt1", float("nan"))))
    shutdown(ctx)


if __name__ == "__main__":
    main()
