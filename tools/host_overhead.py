#!/usr/bin/env python3
"""Host enqueue time vs GPU time of the headline training step, per bucket length.

For each padded length in --frames, times K steps twice: the host-side loop alone (time
until the Python loop has enqueued all K steps, no synchronisation inside) and the full
wall time to the final synchronize. If host time per step approaches the wall time per
step the step is launch-bound and host overhead adds straight to ms/step (the short
SortaGrad buckets of src/deepSpeech_dummy.py:9-11,54-87 are the case that matters).
  python tools/host_overhead.py --steps 30 --frames 100,200,400,1000 [--graph]
--graph times the captured-step path (Trainer(step_graphs=True)) instead of eager;
--force_dp runs the data-parallel machinery at world size 1 over RCCL (bench.py --force_dp),
with --graph its captured step (Trainer(dp_graphs=True)).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--num_hidden", type=int, default=800)
    ap.add_argument("--num_rnn_layers", type=int, default=5)
    ap.add_argument("--frames", type=str, default="1000")
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--force_dp", action="store_true")
    ap.add_argument("--cprofile", type=int, default=0, help="print the N top host functions of the timed loop")
    a = ap.parse_args()
    from deepspeech_amd.utils.setenvs import setenvs
    setenvs([])
    import torch
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.trainer import Trainer, LRSchedule
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=32, num_hidden=a.num_hidden, num_rnn_layers=a.num_rnn_layers, cell="gru").to(dev)
    m.set_engine("hip", torch.bfloat16)
    kw = {"step_graphs": True, "dp_graphs": True} if a.graph else {}
    ctx = None
    if a.force_dp:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        from deepspeech_amd.parallel.dist import init_distributed
        ctx = init_distributed("cuda", force_group=True)
        kw["force_buckets"] = True
    tr = Trainer(m, LRSchedule(1e-4, 10 ** 9, 0.9), defer_update=True, **kw)
    print("| frames | host enqueue ms/step | wall ms/step | audio-s/s |")
    print("|---|---|---|---|")
    for fr in [int(x) for x in a.frames.split(",")]:
        batch = to_device(FixedShapeBatches(32, max_frames=fr, seed=0, pool=1).next(), dev)
        audio = float(batch["seq_lens"].sum().item()) / 100.0
        for _ in range(5):
            tr.step(batch)
        torch.cuda.synchronize()
        prof = None
        if a.cprofile:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            tr.step(batch)
        t1 = time.perf_counter()
        if prof is not None:
            prof.disable()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        wall = (t2 - t0) / a.steps
        print("| %d | %.3f | %.3f | %.0f |" % (fr, 1e3 * (t1 - t0) / a.steps, 1e3 * wall, audio / wall),
              flush=True)
        if prof is not None:
            import io
            import pstats
            buf = io.StringIO()
            pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(a.cprofile)
            print(buf.getvalue(), flush=True)
    if a.graph:
        print("graph modes:", {k[1]: v[0] for k, v in tr.graph_modes.items()} or
              {k[1]: "graph" for k in tr._graphs})
    if ctx is not None:
        from deepspeech_amd.parallel.dist import shutdown
        shutdown(ctx)


if __name__ == "__main__":
    main()
