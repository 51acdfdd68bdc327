#!/usr/bin/env python3
"""Does TunableOp tune the fp32-output (out_dtype) weight-gradient GEMMs? Times dW / dU of the
headline step with default heuristics, then with TunableOp tuning on, and prints the rows
TunableOp wrote (if any).   python tools/probe_tunable_wgrad.py OUT.csv"""
import os
import sys

out_csv = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tunable_wgrad.csv")
import torch  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


dev = torch.device("cuda")
bf = torch.bfloat16
K = 241 * 32
cases = []
for rows, cols, batch in ((4800, 800, 1), (4800, 2400, 1), (2400, 800, 2)):
    g = torch.randn(batch, K, rows, device=dev, dtype=bf)
    x = torch.randn(batch, K, cols, device=dev, dtype=bf)
    o = torch.empty(batch, rows, cols, device=dev, dtype=torch.float32)
    if batch == 1:
        fn = (lambda g=g, x=x, o=o: torch.mm(g[0].t(), x[0], out_dtype=torch.float32, out=o[0]))
    else:
        fn = (lambda g=g, x=x, o=o: torch.bmm(g.transpose(1, 2), x, out_dtype=torch.float32, out=o))
    cases.append(((rows, cols, batch), fn))
for shp, fn in cases:
    print("default", shp, round(timeit(fn), 1), flush=True)
import torch.cuda.tunable as tun  # noqa: E402
tun.enable(True)
tun.tuning_enable(True)
tun.set_filename(out_csv)
for shp, fn in cases:
    fn()
    torch.cuda.synchronize()
print('results:', tun.get_results(), flush=True)
tun.tuning_enable(False)
for shp, fn in cases:
    print("tunable", shp, round(timeit(fn), 1), flush=True)
for f in sorted(os.listdir(os.path.dirname(out_csv))):
    if f.startswith(os.path.basename(out_csv).split(".")[0]):
        print("==", f)
        print(open(os.path.join(os.path.dirname(out_csv), f)).read())
