#!/usr/bin/env python3
"""Gap between two kernels on one stream when event records sit between them: run under
rocprofv3 --kernel-trace and read the gaps with --analyze.

  rocprofv3 --kernel-trace -d gpurun_out/evgap -o run -- python3 tools/probe_event_gap.py
  python3 tools/probe_event_gap.py --analyze gpurun_out/evgap/run_results.db
"""
import argparse
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = ["plain", "1 record", "3 records", "record+wait", "other-stream record", "light record",
         "3 light records", "nofence record", "light record+wait"]


def run():
    import torch
    dev = torch.device("cuda")
    big = torch.empty(48 * 1024 * 1024, device=dev)          # 192 MB written by the "big" kernel
    small = torch.empty(1024, device=dev)
    other = torch.cuda.Stream()
    s = torch.cuda.current_stream()
    from deepspeech_amd.ops import _ext
    C = _ext.ext()
    light = C.event_new(0)
    nofence = C.event_new(0x2 | 0x20000000)      # hipEventDisableTiming | hipEventDisableSystemFence
    for rep in range(6):
        for ci, case in enumerate(CASES):
            torch.cuda._sleep(5_000_000)                      # host runs ahead of the device
            small.fill_(float(ci))                            # case marker (fill value is in no trace; order is)
            big.mul_(1.0001)
            if case == "1 record":
                torch.cuda.Event().record(s)
            elif case == "3 records":
                for _ in range(3):
                    torch.cuda.Event().record(s)
            elif case == "record+wait":
                s.wait_stream(other)
            elif case == "other-stream record":
                torch.cuda.Event().record(other)
            elif case == "light record":
                C.event_record(light, s.cuda_stream)
            elif case == "3 light records":
                for _ in range(3):
                    C.event_record(light, s.cuda_stream)
            elif case == "nofence record":
                C.event_record(nofence, s.cuda_stream)
            elif case == "light record+wait":
                C.stream_wait(s.cuda_stream, other.cuda_stream)
            small.add_(1.0)
            torch.cuda.synchronize()


def analyze(db):
    con = sqlite3.connect(db)
    ks = con.execute("select name, start, end from kernels order by start").fetchall()
    gaps = {c: [] for c in CASES}
    i = 0
    seq = []
    for k in ks:
        seq.append(k)
    # pattern per case: sleep, fill(small), mul(big), add(small)
    idx = 0
    n = 0
    while idx + 3 < len(seq):
        a, f, m, d = seq[idx:idx + 4]
        if "sleep" in a[0].lower() and "mul" in m[0].lower().replace("mulfunctor", "mul") or "Mul" in m[0]:
            case = CASES[n % len(CASES)]
            gaps[case].append((d[1] - m[2]) / 1e3)
            n += 1
            idx += 4
        else:
            idx += 1
    for c, g in gaps.items():
        g.sort()
        print(f"{c:22s} gap after the 192-MB kernel: median {g[len(g) // 2] if g else float('nan'):6.1f} us  all {[round(x, 1) for x in g]}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", default="")
    a = ap.parse_args()
    analyze(a.analyze) if a.analyze else run()
