#!/usr/bin/env python3
"""Run a few synchronised training steps of the headline model with per-step timing and a
Python stack dump if a step stalls (debug aid for stream / partition changes)."""
import faulthandler
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device  # noqa: E402
from deepspeech_amd.models import DeepSpeech2  # noqa: E402
from deepspeech_amd.trainer import LRSchedule, Trainer  # noqa: E402


def main():
    faulthandler.dump_traceback_later(40, repeat=True)
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    engine = sys.argv[2] if len(sys.argv) > 2 else "hip"
    lr = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-4
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=32, num_hidden=800, num_rnn_layers=5, cell="gru").to(dev)
    m.set_engine(engine, torch.bfloat16 if engine == "hip" else torch.float32)
    tr = Trainer(m, LRSchedule(lr, 1000, 0.9))
    batch = to_device(FixedShapeBatches(32, max_frames=1000, seed=1, pool=1).next(), dev)
    for i in range(steps):
        t0 = time.time()
        loss = tr.step(batch)
        torch.cuda.synchronize()
        print("step %d loss %.3f %.2f ms" % (i, float(loss), 1e3 * (time.time() - t0)), flush=True)
    from deepspeech_amd.ops import rnn as RNN
    RNN.check_errors() if hasattr(RNN, "check_errors") else None
    print("ok", flush=True)


if __name__ == "__main__":
    main()
