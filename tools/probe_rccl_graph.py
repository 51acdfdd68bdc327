#!/usr/bin/env python3
"""Can an RCCL all-reduce be captured into a HIP graph on this image (torch.distributed
"nccl" = RCCL, world size 1)? One variant per process (a crash ends only that variant):

  python tools/probe_rccl_graph.py            # runs every variant as a child process
  python tools/probe_rccl_graph.py --variant sync

variants:
  sync      all_reduce on the capture stream itself
  async     all_reduce(async_op=True) issued from a side stream, work.wait() there, joined back
  eager2    sync, with a second eager all_reduce between capture and replay (graph mixing)
  side_sync all_reduce (blocking form) issued from a side stream joined into the capture
  main_async all_reduce(async_op=True) on the capture stream, work.wait() there
  side_async_norec  async, with TORCH_NCCL_AVOID_RECORD_STREAMS=1
"""
import argparse
import os
import subprocess
import sys


def run(variant: str) -> None:
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    import torch
    import torch.distributed as dist
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    dev = torch.device("cuda", 0)
    x = torch.ones(1 << 20, device=dev)
    y = torch.zeros_like(x)
    dist.all_reduce(x)                       # communicator initialised eagerly first
    torch.cuda.synchronize()
    print(variant, "eager ok", flush=True)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(device=dev)
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        y.copy_(x * 2)
        if variant == "side_sync":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                dist.all_reduce(y)
            torch.cuda.current_stream().wait_stream(side)
        elif variant == "main_async":
            w = dist.all_reduce(y, async_op=True)
            w.wait()
        elif variant.startswith("side_async") or variant == "async":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w = dist.all_reduce(y, async_op=True)
                w.wait()
            torch.cuda.current_stream().wait_stream(side)
        else:
            dist.all_reduce(y)
        y.add_(1)
    print(variant, "captured", flush=True)
    for i in range(3):
        x.fill_(float(i + 1))
        g.replay()
        if variant == "eager2":
            dist.all_reduce(x)
        torch.cuda.synchronize()
        want = 2.0 * (i + 1) + 1
        assert float(y[0]) == want and float(y[-1]) == want, (float(y[0]), want)
    print(variant, "replay ok", flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="")
    a = ap.parse_args()
    if a.variant:
        run(a.variant)
        return
    rc = 0
    for i, v in enumerate(("sync", "async", "eager2", "side_sync", "main_async", "side_async_norec")):
        env = dict(os.environ, MASTER_PORT=str(29571 + i))
        if v.endswith("norec"):
            env["TORCH_NCCL_AVOID_RECORD_STREAMS"] = "1"
        r = subprocess.run([sys.executable, __file__, "--variant", v], env=env, capture_output=True, text=True,
                           timeout=120)
        lines = [l for l in (r.stdout + r.stderr).splitlines() if "amdgpu.ids" not in l]
        print("== %s: rc %d" % (v, r.returncode))
        print("\n".join(lines[-8:]))
        rc = rc or r.returncode
    sys.exit(0)


if __name__ == "__main__":
    main()
