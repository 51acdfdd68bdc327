"""Named phase ranges for profiling (roctx via torch.profiler.record_function).

Phase names follow the reference's per-layer profiler (tools/prof.py:15-53 of the
reference: conv1_forward, bn1_forward, rnn_forward_cell_<i>, rnn_backward_cell_<i>,
softmax_forward, ctc_forward, ExponentialMovingAverage, ...), so traces of this engine can
be broken down per layer the same way (tools/prof.py here).

Ranges cost a few microseconds of host time each, so they are OFF unless enabled
(``enable(True)``: the train driver does it for its --debug step; ``DS2_TRACE=1`` turns
them on globally). Inside a disabled range nothing is recorded.
"""
from __future__ import annotations

import contextlib
import os

_enabled = os.environ.get("DS2_TRACE", "0") == "1"


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = bool(on)


def enabled() -> bool:
    return _enabled


def phase(name: str):
    """Context manager marking a named phase (no-op when tracing is disabled)."""
    if not _enabled:
        return contextlib.nullcontext()
    import torch
    return torch.profiler.record_function(name)


# canonical phase names (reference tools/prof.py layers_names)
def conv(i: int, bwd: bool = False) -> str:
    return "conv%d_%s" % (i, "backward" if bwd else "forward")


def bn(i: int, bwd: bool = False) -> str:
    return "bn%d_relu%d_%s" % (i, i, "backward" if bwd else "forward")


def rnn_cell(i: int, bwd: bool = False) -> str:
    return "rnn_%s_cell_%d" % ("backward" if bwd else "forward", i)


SOFTMAX_F, SOFTMAX_B = "softmax_forward", "softmax_backward"
CTC_F, CTC_B = "ctc_forward", "ctc_backward"
EMA = "ExponentialMovingAverage"
ALLREDUCE = "allreduce"
