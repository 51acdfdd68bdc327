"""Measured library-GEMM selection for the HIP engine (PyTorch TunableOp over hipBLASLt +
rocBLAS solutions).

The plain projection GEMMs (recurrent input projections and their data gradients, the FC
head) stay library GEMMs. hipBLASLt's heuristic pick is far from the best solution for
several DeepSpeech2 shapes on gfx950 (e.g. the first layer's [7712 x 2400] x [2400 x 4800]
projection: 264 us heuristic vs 168 us best). ``deepspeech_amd/tuning/tunableop_gfx950.csv``
holds the solutions measured on MI355X for the benchmark configurations; with it loaded,
PyTorch dispatches those shapes to the measured-fastest solution and everything else to the
default heuristic. Tuning is OFF at run time (no timing runs inside training steps).

  enable_tuned_gemms(mode="tune", out=PATH)   tune unseen shapes too and write them to PATH
                                              (tools/tune_buckets.py); merge the rows by hand
"""
from __future__ import annotations

import os

TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning",
                     "tunableop_gfx950.csv")
_done = False


def enable_tuned_gemms(mode: str = "1", out: str = "") -> bool:
    """Load the measured GEMM table once per process (idempotent). Returns True if active.
    mode "0": do not load it; "tune": also tune unseen shapes, written to ``out``."""
    global _done
    if _done:
        return True
    if mode == "0":
        return False
    import torch
    if not torch.cuda.is_available() or not hasattr(torch.cuda, "tunable"):
        return False
    tun = torch.cuda.tunable
    tun.enable(True)
    if mode == "tune":
        tun.tuning_enable(True)
        tun.set_filename(out or "tunableop_new.csv")
        if os.path.exists(TABLE):
            tun.read_file(TABLE)
    else:
        tun.tuning_enable(False)
        tun.record_untuned_enable(False)
        # point the writer at a scratch name so the shipped table is never rewritten
        tun.set_filename(out or os.path.join("/tmp", "ds2_tunableop_unused.csv"))
        if os.path.exists(TABLE):
            tun.read_file(TABLE)
    _done = True
    return True
