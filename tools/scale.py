#!/usr/bin/env python3
"""Single-node data-parallel scaling harness (SURVEY §7.1 ``bench/``, §5.8).

Runs the headline training benchmark at 1, 2, 4, 8 ranks (capped at the GPUs present) and
the RCCL all-reduce bandwidth at the gradient-bucket size on the largest world, then prints
ONE table: ms/step, whole-job and per-GPU audio-s/s, weak-scaling efficiency against the
1-GPU run, and the bus bandwidth of the bucket-sized all-reduce (fp32 and bf16 wire dtype).

  python tools/scale.py [--worlds 1,2,4,8] [--steps 20 --warmup 5] [--out gpurun_out/scale]
                        [-- <extra bench.py args, e.g. --num_hidden 1280 --num_rnn_layers 7>]

Each run is a child process (bench.py starts its own ranks, parallel/launch.py) under its own
time limit; the harness itself never initialises the GPU. The chain stops at the first
failing run (its exit code is returned), so a faulting world size is not followed by more GPU
work. The table goes to stdout and, with --out, to ``scale.md`` / ``scale.json``.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpu_count() -> int:
    # on this image (PyTorch 2.10 + ROCm 7) counting devices does not initialise them:
    # torch.cuda.device_count uses the non-initialising enumeration (the pool's own notes say the
    # same), so the parent still never brings up HIP before it starts the ranks; an explicit
    # HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES is honoured by it
    try:
        import torch
        return int(torch.cuda.device_count())
    except Exception:
        return 0


def _json_lines(text: str):
    rows = []
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{"):
            try:
                rows.append(json.loads(line))
            except ValueError:
                pass
    return rows


def _run(cmd, timeout_s, log_path=None):
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout_s)
    if log_path:
        with open(log_path, "w") as f:
            f.write("$ %s\n%s\n---- stderr ----\n%s" % (" ".join(cmd), r.stdout, r.stderr))
    return r, time.time() - t0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bucket_mb", type=float, default=32.0)
    ap.add_argument("--timeout", type=int, default=300, help="per-run limit (s)")
    ap.add_argument("--out", default="")
    ap.add_argument("--cpu", action="store_true", help="gloo on the CPU (plumbing check)")
    a = ap.parse_args(argv)
    worlds = [int(w) for w in a.worlds.split(",")]
    if not a.cpu:
        have = _gpu_count()
        if have < 1:
            print("no GPU visible (use --cpu for a gloo plumbing run)", file=sys.stderr)
            return 2
        worlds = [w for w in worlds if w <= have]
    if a.out:
        os.makedirs(a.out, exist_ok=True)
    env_note = {}
    if a.cpu:
        os.environ["CUDA_VISIBLE_DEVICES"] = ""
        env_note["backend"] = "gloo (cpu)"
    rows = []
    for w in worlds:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(w), "--steps", str(a.steps),
               "--warmup", str(a.warmup), "--bucket_mb", str(a.bucket_mb), "--no_infer"] + extra
        r, wall = _run(cmd, a.timeout, os.path.join(a.out, "bench_n%d.log" % w) if a.out else None)
        got = _json_lines(r.stdout)
        if r.returncode != 0 or len(got) != 1:
            print("bench at %d rank(s) failed (rc=%d)\n%s\n%s" % (w, r.returncode, r.stdout[-2000:],
                                                                  r.stderr[-3000:]), file=sys.stderr)
            return r.returncode or 1
        got[0]["wall_s"] = round(wall, 1)
        rows.append(got[0])
        print("n=%d  %.3f ms/step  %.0f audio-s/s" % (w, got[0]["ms_per_step"], got[0]["value"]), flush=True)
    # all-reduce bus bandwidth at the bucket size, on the largest world (fp32 and bf16 wire)
    busbw = {}
    wmax = max(worlds)
    if wmax > 1:
        for dt in ("fp32", "bf16"):
            cmd = [sys.executable, os.path.join(ROOT, "tools", "bench_allreduce.py"), "--gpus", str(wmax),
                   "--sizes_mb", "%g,%g" % (a.bucket_mb, 4 * a.bucket_mb), "--dtype", dt, "--iters", "20",
                   "--warmup", "5"] + (["--device", "cpu"] if a.cpu else [])
            r, _ = _run(cmd, a.timeout, os.path.join(a.out, "allreduce_%s.log" % dt) if a.out else None)
            if r.returncode != 0:
                print("all-reduce bench failed (rc=%d)\n%s" % (r.returncode, r.stderr[-3000:]), file=sys.stderr)
                return r.returncode or 1
            busbw[dt] = _json_lines(r.stdout)
    base = rows[0]["value"] / rows[0]["n_gpus"]
    lines = ["| GPUs | ms/step | audio-s/s (job) | audio-s/s per GPU | weak-scaling eff. | global batch |",
             "|---|---|---|---|---|---|"]
    for row in rows:
        n = row["n_gpus"]
        eff = row["value"] / n / base
        lines.append("| %d | %.3f | %.0f | %.0f | %.1f %% | %d |" % (
            n, row["ms_per_step"], row["value"], row["value"] / n, 100 * eff, row["config"]["global_batch"]))
    for dt, bw in busbw.items():
        for b in bw:
            lines.append("")
            lines.append("all-reduce %s, %d ranks, %.1f MB: %.1f us, algbw %.1f GB/s, busbw %.1f GB/s (%s)" % (
                dt, b["world"], b["bytes"] / 2 ** 20, b["time_us"], b["algbw_GBps"], b["busbw_GBps"], b["backend"]))
    table = "\n".join(lines)
    print(table)
    if a.out:
        with open(os.path.join(a.out, "scale.md"), "w") as f:
            f.write(table + "\n")
        with open(os.path.join(a.out, "scale.json"), "w") as f:
            json.dump({"runs": rows, "allreduce": busbw, "extra_args": extra, **env_note}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
