#!/usr/bin/env python3
"""Cross-stream signalling without a marker packet: gap between a 192-MB multi_fill kernel and
the next kernel on its stream when another stream must wait for the fill, with the event
(a) recorded behind the fill (hipEventRecord: a marker packet in the fill's queue) or
(b) bound to the fill's own launch (hipExtLaunchKernel stop event, csrc/common.h ds2_launch),
and a check that the waiting stream reads the finished fill (it copies the buffer's tail,
which the grid-stride fill writes last, and compares it with this iteration's pattern).

  rocprofv3 --kernel-trace -d gpurun_out/extev -o run -- python3 tools/probe_ext_event.py
  python3 tools/probe_ext_event.py --analyze gpurun_out/extev/run_results.db
"""
import argparse
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = ["plain", "record + side wait", "ext light + side wait", "ext timing + side wait",
         "ext nofence + side wait"]


def run(reps: int):
    import torch
    from deepspeech_amd.ops import _ext
    C = _ext.ext()
    dev = torch.device("cuda")
    big = torch.empty(48 * 1024 * 1024, device=dev, dtype=torch.int32)   # 192 MB
    small = torch.ones(1024, device=dev)
    chk = torch.empty(4096, device=dev, dtype=torch.int32)
    main = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    light = C.event_new(0)                       # hipEventDisableTiming
    timing = C.event_new(0x1)                    # hipEventBlockingSync: timing kept
    nofence = C.event_new(0x2 | 0x20000000)      # DisableTiming | DisableSystemFence
    bad = 0
    it = 0
    for rep in range(reps):
        for ci, case in enumerate(CASES):
            it += 1
            pat = 1000 + it
            torch.cuda._sleep(5_000_000)         # host runs ahead of the device
            small.fill_(float(ci))
            ev = {"ext light + side wait": light, "ext timing + side wait": timing,
                  "ext nofence + side wait": nofence}.get(case)
            if ev is not None:
                C.arm_stop_event(ev)
            C.multi_fill([big], [pat])
            if ev is not None:
                assert not C.disarm_stop_event(), "stop event not taken by the launch"
            if case == "record + side wait":
                C.event_record(light, main.cuda_stream)
                ev = light
            if ev is not None:
                C.event_wait(side.cuda_stream, ev)
                with torch.cuda.stream(side):
                    chk.copy_(big[-4096:])
            small.neg_()
            torch.cuda.synchronize()
            if ev is not None and not bool((chk == pat).all()):
                bad += 1
                print(f"STALE READ: case {case!r} rep {rep}", flush=True)
    print(f"stale reads: {bad}", flush=True)
    return bad


def analyze(db):
    con = sqlite3.connect(db)
    ks = con.execute("select name, start, end from kernels order by start").fetchall()
    gaps = {c: [] for c in CASES}
    n = 0
    for i, (name, st, en) in enumerate(ks):
        if "multi_fill" not in name:
            continue
        nxt = next((k for k in ks[i + 1:] if "neg" in k[0].lower()), None)
        if nxt is None:
            continue
        gaps[CASES[n % len(CASES)]].append((nxt[1] - en) / 1e3)
        n += 1
    for c, g in gaps.items():
        g.sort()
        med = g[len(g) // 2] if g else float("nan")
        print(f"{c:26s} gap after the fill: median {med:6.1f} us  all {[round(x, 1) for x in g]}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", default="")
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        sys.exit(1 if run(a.reps) else 0)
