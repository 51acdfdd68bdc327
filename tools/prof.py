#!/usr/bin/env python3
"""Per-layer time breakdown of a chrome trace (reference: tools/prof.py of yxlao/deepSpeech,
which buckets TF timeline ops into conv1/bn1/relu1/.../rnn cell i fwd/bwd/ctc/EMA phases).

  python tools/prof.py --input train_dir/profiling.json [--output Output] [--threshold-us 50]

Input: the torch.profiler chrome trace written by the train driver's --debug step (or
bench.py --profile_dir). The engine marks phases with record_function ranges named like
the reference's layers (deepspeech_amd/utils/trace.py: conv1_forward, bn1_relu1_forward,
rnn_forward_cell_0, rnn_backward_cell_0, softmax_forward, ctc_forward,
ExponentialMovingAverage, ...). Every GPU kernel is attributed to the innermost phase
whose host range issued its launch (launch -> kernel by correlation id).

Per phase it reports: kernels, kernel time (sum of kernel durations), span (first kernel
start to last kernel end), idle gaps inside the span (total, and the part from gaps
shorter than --threshold-us, the reference's wall_time_thres) and writes
<output>/layers_exeTime.csv, <output>/layers_gaps.csv and <output>/kernels.csv.
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeech_amd.utils.prof import analyse, format_table, load_events, write_outputs  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--input", "-i", required=True)
    ap.add_argument("--output", "-o", default="Output")
    ap.add_argument("--threshold-us", type=float, default=50.0)
    a = ap.parse_args(argv)
    out, rows = analyse(load_events(a.input), a.threshold_us)
    write_outputs(out, rows, a.output)
    print(format_table(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
