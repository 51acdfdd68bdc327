#!/usr/bin/env python3
"""Streaming-inference real-time factor (BASELINE.json config 4: unidirectional GRU + CTC
beam-search decoder on one MI355X).

  python tools/bench_infer.py [--layers 5] [--hidden 800] [--seconds 20] [--chunks 0.25,0.5,1.0]
                              [--batches 1,32] [--decoders greedy,beam]

RTF = compute seconds / audio seconds per stream (B concurrent streams share each chunk
launch, so B streams at RTF r serve B * (1 / r) x real time). Random-init weights and
synthetic 161-bin features (no checkpoint or dataset offline). One JSON line per setting.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deepspeech_amd.infer import rtf  # noqa: E402
from deepspeech_amd.models import DeepSpeech2  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=5)
    ap.add_argument("--hidden", type=int, default=800)
    ap.add_argument("--cell", default="gru")
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--chunks", default="0.25,0.5,1.0")
    ap.add_argument("--batches", default="1,32")
    ap.add_argument("--decoders", default="greedy,beam")
    ap.add_argument("--beam_width", type=int, default=16)
    ap.add_argument("--engine", default="hip")
    a = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    eng = a.engine if dev.type == "cuda" else "ref"
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=32, num_hidden=a.hidden, num_rnn_layers=a.layers, cell=a.cell,
                    bidirectional=False).to(dev)
    m.set_engine(eng, torch.bfloat16 if eng == "hip" else torch.float32)
    rtf(m, seconds=2.0, chunk_s=0.5, batch=1)          # warm-up (plans, kernels, allocator)
    for B in [int(x) for x in a.batches.split(",")]:
        for c in [float(x) for x in a.chunks.split(",")]:
            for d in a.decoders.split(","):
                r, _ = rtf(m, seconds=a.seconds, chunk_s=c, batch=B, decoder=d, beam_width=a.beam_width)
                print(json.dumps({"metric": "streaming RTF (lower is better)", "model": "DS2 2xconv(32) + %dx uni-%s-%d"
                                  % (a.layers, a.cell.upper(), a.hidden), "engine": eng, "streams": B,
                                  "chunk_s": c, "decoder": d, "beam_width": a.beam_width if d == "beam" else None,
                                  "rtf": round(r, 5), "x_realtime_per_stream": round(1.0 / r, 1) if r > 0 else None,
                                  "x_realtime_total": round(B / r, 1) if r > 0 else None,
                                  "audio_s": a.seconds, "data": "synthetic features, random-init weights"}),
                      flush=True)


if __name__ == "__main__":
    main()
