#!/usr/bin/env python3
"""Measure the library-GEMM solutions (PyTorch TunableOp over hipBLASLt / rocBLAS) for the
GEMM shapes of EVERY length bucket of the reference's dummy epoch (src/deepSpeech_dummy.py:
9-16, 100 ... 1500 frames), headline model (2 x conv(32) + 5 x BiGRU-800, batch 32).

The shipped table (deepspeech_amd/tuning/tunableop_gfx950.csv) first covered only the
benchmark shapes; every other bucket fell back to hipBLASLt's default heuristic (VERDICT r1
item 7). Run on an MI355X; the new rows land in --out and are merged into the shipped table
(existing rows win) with --merge. Only the NN data-gradient GEMMs go through TunableOp; the
weight gradients (fp32-output mm / bmm) keep hipBLASLt's heuristic.

  python tools/tune_buckets.py --out gpurun_out/tunableop_buckets.csv      (on the GPU)
  python tools/tune_buckets.py --merge gpurun_out/tunableop_buckets.csv    (anywhere)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def merge(path: str) -> None:
    from deepspeech_amd.ops.gemm_tuning import TABLE
    with open(TABLE) as f:
        old = [ln.rstrip("\n") for ln in f if ln.strip()]
    keys = {tuple(ln.split(",")[:2]) for ln in old}
    new = []
    with open(path) as f:
        for ln in f:
            ln = ln.rstrip("\n")
            if not ln.strip() or ln.startswith("Validator"):
                continue
            k = tuple(ln.split(",")[:2])
            if k not in keys:
                keys.add(k)
                new.append(ln)
    with open(TABLE, "w") as f:
        f.write("\n".join(old + new) + "\n")
    print("merged %d new rows into %s (%d total)" % (len(new), TABLE, len(old) + len(new)))


def tune(out: str, frames, batch: int) -> None:
    from deepspeech_amd.ops.gemm_tuning import enable_tuned_gemms
    from deepspeech_amd.utils.setenvs import setenvs
    setenvs([])
    import torch
    enable_tuned_gemms(mode="tune", out=out)     # before the model's own (idempotent) call
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.trainer import LRSchedule, Trainer
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = DeepSpeech2(num_filters=32, num_hidden=800, num_rnn_layers=5, cell="gru").to(dev)
    model.set_engine("hip", torch.bfloat16)
    tr = Trainer(model, LRSchedule(1e-5, 10 ** 9, 0.9))
    for fr in frames:
        b = to_device(FixedShapeBatches(batch, max_frames=fr, seed=fr, pool=1).next(), dev)
        for _ in range(2):                 # first step tunes every new shape, second uses them
            tr.step(b)
        torch.cuda.synchronize()
        print("bucket %d frames tuned" % fr, flush=True)
    wf = getattr(torch.cuda.tunable, "write_file", None)     # older torch; 2.10 writes at exit
    if wf is not None:
        wf()
    print("results go to", out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/tunableop_buckets.csv")
    ap.add_argument("--merge", default="")
    ap.add_argument("--frames", default=",".join(str(100 * i) for i in range(1, 16)))
    ap.add_argument("--batch_size", type=int, default=32)
    a = ap.parse_args()
    if a.merge:
        merge(a.merge)
    else:
        tune(a.out, [int(x) for x in a.frames.split(",")], a.batch_size)


if __name__ == "__main__":
    main()
