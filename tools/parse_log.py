#!/usr/bin/env python3
"""Summarise a training run's timing logs (reference: tools/parse_log.py of yxlao/deepSpeech,
which sums tfprof per-layer times into prf1.txt / prf2.txt).

  python tools/parse_log.py --train_dir <dir> [--log train.log]

Reads what the train driver writes:
  * <train_dir>/profile_layers.txt  per-phase kernel time of the --debug step (written
    from the chrome trace by deepspeech_amd/utils/prof.py), and
  * the driver's stdout log (optional): "step N, loss = L (E examples/sec; S sec/batch;
    A audio-sec/sec)" lines.
Writes prf1.txt (ms per layer: conv, bn+relu, each RNN cell fwd+bwd, softmax, ctc, EMA)
and prf2.txt (RNN cells: forward vs backward ms) into the train dir and prints both.
"""
import argparse
import os
import re
import sys

LINE = re.compile(r"step (\d+), loss = ([-\d.naif]+) \(([\d.]+) examples/sec; ([\d.]+) sec/batch(?:; ([\d.]+) dummy sec/batch)?"
                  r"(?:; ([\d.]+) audio-sec/sec)?\)")
CELL = re.compile(r"rnn_(forward|backward)_cell_(\d+)")


def read_layers(path):
    out = {}
    with open(path) as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 3 and parts[0] != "layer":
                try:
                    out[parts[0]] = float(parts[2])
                except ValueError:
                    pass
    return out


def group(layers):
    g = {}
    for name, ms in layers.items():
        m = CELL.match(name)
        if m:
            key = "rnn_cell_%s" % m.group(2)
        elif name.startswith("conv"):
            key = name.split("_")[0]
        elif name.startswith("bn"):
            key = name.split("_")[0] + "_relu"
        else:
            key = name.replace("_forward", "").replace("_backward", "")
        g[key] = g.get(key, 0.0) + ms
    return g


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--train_dir", required=True)
    ap.add_argument("--log", default="")
    a = ap.parse_args(argv)
    lp = os.path.join(a.train_dir, "profile_layers.txt")
    lines1, lines2 = [], []
    if os.path.exists(lp):
        layers = read_layers(lp)
        for k, v in sorted(group(layers).items(), key=lambda kv: -kv[1]):
            lines1.append("%-28s %10.3f ms" % (k, v))
        cells = {}
        for name, ms in layers.items():
            m = CELL.match(name)
            if m:
                cells.setdefault(int(m.group(2)), [0.0, 0.0])[0 if m.group(1) == "forward" else 1] += ms
        for i in sorted(cells):
            lines2.append("rnn cell %d: forward %9.3f ms  backward %9.3f ms" % (i, cells[i][0], cells[i][1]))
    if a.log and os.path.exists(a.log):
        rates = []
        with open(a.log) as f:
            for line in f:
                m = LINE.search(line)
                if m:
                    rates.append((int(m.group(1)), float(m.group(3)), float(m.group(4)),
                                  float(m.group(6)) if m.group(6) else float("nan")))
        if rates:
            s, ex, sb, aps = rates[-1]
            lines1.append("last log line: step %d  %.1f examples/sec  %.4f sec/batch  %.1f audio-sec/sec"
                          % (s, ex, sb, aps))
    with open(os.path.join(a.train_dir, "prf1.txt"), "w") as f:
        f.write("\n".join(lines1) + "\n")
    with open(os.path.join(a.train_dir, "prf2.txt"), "w") as f:
        f.write("\n".join(lines2) + "\n")
    print("\n".join(lines1))
    print("\n".join(lines2))
    return 0


if __name__ == "__main__":
    sys.exit(main())
