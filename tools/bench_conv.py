#!/usr/bin/env python3
"""Conv front-end kernels alone (headline geometry: batch 32, 1000 frames, 32 filters):
forward + backward of FrontendCL timed with HIP events, plus a rocprof-friendly loop.
  python tools/bench_conv.py [--iters 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.ops import frontend as FE
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=32, num_hidden=800, num_rnn_layers=1, cell="gru").to(dev)
    m.set_engine("hip", torch.bfloat16)
    m.train()
    x = torch.randn(32, 1000, 161, device=dev).bfloat16().requires_grad_(False)
    y = FE.frontend_hip(m, x)
    dy = torch.randn_like(y)
    def step():
        out = FE.frontend_hip(m, x)
        out.backward(dy)
    for _ in range(3):
        step()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(a.iters):
        step()
    e.record()
    torch.cuda.synchronize()
    print(json.dumps({"so": os.environ.get("DS2_EXT_SO", "in-tree"),
                      "frontend_fwd_bwd_us": round(s.elapsed_time(e) / a.iters * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
