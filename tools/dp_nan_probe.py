#!/usr/bin/env python3
"""Repeated data-parallel training steps at the config-5 fp8 geometry on one GPU (2 gloo ranks):
after each step, report the recurrence error word and which arena gradients / weights are
non-finite on this rank. Launch with torch.distributed.run --nproc-per-node 2 (DS2_DIST_BACKEND=gloo)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
os.environ.setdefault("DS2_DP_GEOM", "config5")
import torch  # noqa: E402

import dp_gpu_worker as W  # noqa: E402
from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device  # noqa: E402
from deepspeech_amd.ops import rnn as RNN  # noqa: E402
from deepspeech_amd.parallel.dist import init_distributed  # noqa: E402
from deepspeech_amd.trainer import LRSchedule, Trainer  # noqa: E402


def main():
    ctx = init_distributed("cuda")
    dev = ctx.device
    reps = int(os.environ.get("REPS", "6"))
    batch = to_device(FixedShapeBatches(W.geom()["batch"], max_frames=300, seed=100 + ctx.rank, pool=1).next(), dev)
    for rep in range(reps):
        tr = Trainer(W.model(dev), LRSchedule(1e-3, 10 ** 6, 0.9), world_size=ctx.world_size,
                     bucket_mb=W.geom()["bucket_mb"])
        loss = tr.step(batch)
        torch.cuda.synchronize()
        err = int(RNN.error_word(dev).item())
        RNN.error_word(dev).zero_()
        badg = [(n, int((~torch.isfinite(tr.arena.grad[o:o + c])).sum())) for n, (o, c) in
                zip(tr.arena.names, tr.arena.offsets)]
        badg = [(n, k) for n, k in badg if k]
        badw = sum(int((~torch.isfinite(tr.arena.flat[o:o + c])).sum()) for o, c in tr.arena.offsets)
        print("rank %d rep %d loss %.4f err 0x%x nonfinite w %d grads %s" % (
            ctx.rank, rep, float(loss), err, badw, badg[:6]), flush=True)
        del tr
    torch.distributed.barrier()


if __name__ == "__main__":
    main()
