#!/usr/bin/env python3
"""Loader-fed vs pre-staged training throughput per length bucket (headline model).

For every bucket of the reference's dummy epoch (src/deepSpeech_dummy.py:9-16: 100 ... 1500
frames, one length per batch) the same training step is timed twice:
  staged  batches already resident on the GPU (what bench.py measures)
  loader  batches produced on the host each step (numpy generation + labels) and uploaded
          through data/prefetch.py (pinned ring + copy stream + event), as train.py runs
and audio-s/s of both, their ratio, plus a whole-epoch walk in SortaGrad order.

  python tools/bench_loader.py [--steps 8] [--warmup 3] [--epoch_steps 60]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deepspeech_amd.utils.setenvs import setenvs  # noqa: E402

setenvs([])
import torch  # noqa: E402


class _Bucket:
    def __init__(self, walk, i):
        self.walk, self.i = walk, i

    def next(self):
        return self.walk.batch_for(self.i)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch_size", type=int, default=32)
    ap.add_argument("--epoch_steps", type=int, default=60)
    a = ap.parse_args()
    from deepspeech_amd.data.prefetch import DevicePrefetcher
    from deepspeech_amd.data.synthetic import UTT_LENGTHS, DummyBucketWalk, to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.ops import rnn as RNN
    from deepspeech_amd.trainer import LRSchedule, Trainer
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = DeepSpeech2(num_filters=32, num_hidden=800, num_rnn_layers=5, cell="gru").to(dev)
    model.set_engine("hip", torch.bfloat16)
    tr = Trainer(model, LRSchedule(1e-5, 10 ** 9, 0.9))
    walk = DummyBucketWalk(a.batch_size, seed=1)

    def timed(get_batch, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        audio = 0.0
        for _ in range(n):
            hb, b = get_batch()
            tr.step(b)
            audio += hb.audio_seconds
        torch.cuda.synchronize()
        return time.perf_counter() - t0, audio

    for i in sorted(set(range(len(UTT_LENGTHS))), key=lambda j: UTT_LENGTHS[j]):
        if UTT_LENGTHS[i] in [UTT_LENGTHS[j] for j in range(i)]:
            continue
        staged = [walk.batch_for(i) for _ in range(2)]
        dstaged = [(h, to_device(h, dev)) for h in staged]
        k = [0]

        def get_staged():
            k[0] += 1
            return dstaged[k[0] % 2]
        timed(get_staged, a.warmup)
        ts, au_s = timed(get_staged, a.steps)
        pf = DevicePrefetcher(_Bucket(walk, i), dev, depth=2)
        timed(pf.next, a.warmup)
        tl, au_l = timed(pf.next, a.steps)
        pf.close()
        RNN.check_errors()
        print(json.dumps({"frames": UTT_LENGTHS[i], "staged_ms": round(1e3 * ts / a.steps, 3),
                          "loader_ms": round(1e3 * tl / a.steps, 3),
                          "staged_audio_s_per_s": round(au_s / ts, 1), "loader_audio_s_per_s": round(au_l / tl, 1),
                          "loader_vs_staged": round((au_l / tl) / (au_s / ts), 4)}), flush=True)
    # the SortaGrad epoch order itself (ascending buckets), loader-fed
    walk2 = DummyBucketWalk(a.batch_size, seed=2)
    pf = DevicePrefetcher(walk2, dev, depth=2)
    timed(pf.next, a.warmup)
    t, au = timed(pf.next, a.epoch_steps)
    pf.close()
    print(json.dumps({"epoch_walk_steps": a.epoch_steps, "audio_s_per_s": round(au / t, 1),
                      "ms_per_step": round(1e3 * t / a.epoch_steps, 3)}), flush=True)


if __name__ == "__main__":
    main()
