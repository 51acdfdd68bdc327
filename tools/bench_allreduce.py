#!/usr/bin/env python3
"""Collective bandwidth of the data-parallel path (nccl-tests conventions), one JSON line per
message size on rank 0:

  algbw = bytes / time,   busbw = algbw * 2 (n - 1) / n   (all-reduce, ring-equivalent traffic)

  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
         tools/bench_allreduce.py [--sizes_mb 1,4,16,32,64,128,256] [--dtype fp32] [--op all_reduce]

Uses the same process-group setup and platform environment as training (RCCL over xGMI on
MI355X, `utils/setenvs.py` channel budget; gloo on CPU, where it only checks the plumbing).
The gradient buckets of the headline model are 32 MB (`--bucket_mb`), so the 16-64 MB rows
are the ones that matter for the backward overlap.
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
import torch  # noqa: E402,F401  (importing torch does not initialise the GPU)
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes_mb", default="1,4,16,32,64,128,256")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--op", default="all_reduce", choices=["all_reduce", "reduce_scatter", "all_gather"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks on this node when no launcher is active (parallel/launch.py)")
    a = ap.parse_args()
    from deepspeech_amd.parallel.launch import check_world, maybe_spawn
    code = maybe_spawn(a.gpus, os.path.abspath(__file__), sys.argv[1:])
    if code is not None:
        sys.exit(code)
    check_world(a.gpus)
    from deepspeech_amd.parallel.dist import init_distributed
    ctx = init_distributed("auto" if a.device == "auto" else a.device, force_group=True)
    n = ctx.world_size
    dev = ctx.device
    gpu = dev.type == "cuda"
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    esz = torch.tensor([], dtype=dt).element_size()

    def sync():
        if gpu:
            torch.cuda.synchronize(dev)

    for mb in [float(x) for x in a.sizes_mb.split(",")]:
        numel = max(n, int(mb * 2 ** 20 / esz) // n * n)
        x = torch.ones(numel, device=dev, dtype=dt)
        out = torch.empty(numel // n if a.op == "reduce_scatter" else numel, device=dev, dtype=dt)

        def op():
            if a.op == "all_reduce":
                dist.all_reduce(x)
            elif a.op == "reduce_scatter":
                dist.reduce_scatter_tensor(out, x)
            else:
                dist.all_gather_into_tensor(x, x[: numel // n].contiguous())
        for _ in range(a.warmup):
            op()
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            op()
        sync()
        dt_s = (time.perf_counter() - t0) / a.iters
        # slowest rank defines the collective time
        t = torch.tensor([dt_s], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt_s = float(t)
        nbytes = numel * esz
        algbw = nbytes / dt_s / 1e9
        factor = 2 * (n - 1) / n if a.op == "all_reduce" else (n - 1) / n
        if ctx.rank == 0:
            print(json.dumps({"op": a.op, "backend": dist.get_backend(), "world": n, "dtype": a.dtype,
                              "bytes": nbytes, "time_us": round(dt_s * 1e6, 1), "algbw_GBps": round(algbw, 2),
                              "busbw_GBps": round(algbw * factor, 2)}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
