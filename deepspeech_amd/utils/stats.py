"""Tensor summaries and the per-step divergence watch.

* :func:`histogram` — tf.summary.histogram + tf.nn.zero_fraction of a tensor in one pass:
  on the GPU csrc/stats.hip ``hist_stats`` (TensorFlow's default exponential buckets
  +-1e-12 * 1.1^i, LDS-accumulated counts, per-workgroup min/max/sum/sum-sq/zero partials);
  on the CPU the same buckets with numpy. Reference: ``_activation_summary``
  (src/helper_routines.py:15-28) at conv1/conv2/rnn/logits (src/deepSpeech_NCHW.py:134,158,
  183,199) and the gradient / variable histograms of ``add_summaries``
  (src/deepSpeech_train.py:401-416).
* :class:`NonfiniteWatch` — the reference asserts ``not isnan(loss)`` after EVERY step
  (src/deepSpeech_train.py:325), which costs a host sync per step. Here a device step
  counter and a sticky first-non-finite-step word are updated by one tiny launch per step;
  the host reads them wherever it synchronises anyway (logging, checkpoints, the end of
  training) and reports the exact step that diverged.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

NPOS = 775
NBUCKET = 2 * NPOS + 1


def tf_bucket_limits() -> np.ndarray:
    """TensorFlow's default histogram bucket limits (tensorflow/core/lib/histogram):
    -DBL_MAX, ..., -1e-12, 0, 1e-12, 1.1e-12, ..., ~1e20, DBL_MAX."""
    pos = []
    v = 1e-12
    while v < 1e20 and len(pos) < NPOS - 1:
        pos.append(v)
        v *= 1.1
    while len(pos) < NPOS - 1:        # (774 limits by construction)
        pos.append(pos[-1] * 1.1)
    pos.append(np.finfo(np.float64).max)
    pos = np.array(pos, dtype=np.float64)
    return np.concatenate([-pos[::-1], [0.0], pos])


_LIMITS = None


def limits() -> np.ndarray:
    global _LIMITS
    if _LIMITS is None:
        _LIMITS = tf_bucket_limits()
    return _LIMITS


@dataclass
class HistStats:
    min: float
    max: float
    num: float
    sum: float
    sum_sq: float
    zeros: float
    nonfinite: float
    counts: np.ndarray          # [NBUCKET] counts per bucket of limits()

    @property
    def zero_fraction(self) -> float:
        return self.zeros / max(1.0, self.num)


def _bucket_index_np(v: np.ndarray) -> np.ndarray:
    a = np.abs(v)
    with np.errstate(divide="ignore"):
        i = np.floor(np.log(np.maximum(a, 1e-30) * 1e12) / np.log(1.1)).astype(np.int64)
    i = np.clip(i, 0, NPOS - 1)
    pos = np.minimum(NPOS + 2 + i, NBUCKET - 1)
    neg = np.maximum(NPOS - 1 - i, 0)
    out = np.where(v > 0, pos, neg)
    return np.where(a >= 1e-12, out, NPOS)


def histogram(t: torch.Tensor) -> HistStats:
    """One-pass histogram + moments + zero fraction of ``t`` (any shape, fp32/bf16)."""
    t = t.detach()
    if t.is_cuda and t.dtype in (torch.float32, torch.bfloat16):
        from ..ops import _ext
        C = _ext.ext()
        x = t.contiguous().view(-1)
        counts = torch.zeros(NBUCKET, device=t.device, dtype=torch.int32)
        nb = int(C.hist_blocks(x.numel()))
        part = torch.empty(nb, 6, device=t.device, dtype=torch.float32)
        C.hist_stats(x, counts, part)
        p = part.double()
        r = torch.stack([p[:, 0].min(), p[:, 1].max(), p[:, 2].sum(), p[:, 3].sum(), p[:, 4].sum(),
                         p[:, 5].sum()]).cpu().numpy()
        c = counts.cpu().numpy().astype(np.int64)
        n = float(c.sum())
        return HistStats(min=float(r[0]), max=float(r[1]), num=n, sum=float(r[2]), sum_sq=float(r[3]),
                         zeros=float(r[4]), nonfinite=float(r[5]), counts=c)
    v = t.float().cpu().numpy().ravel().astype(np.float64)
    fin = np.isfinite(v)
    bad = float((~fin).sum())
    v = v[fin]
    c = np.bincount(_bucket_index_np(v), minlength=NBUCKET).astype(np.int64) if v.size else np.zeros(NBUCKET, np.int64)
    return HistStats(min=float(v.min()) if v.size else 0.0, max=float(v.max()) if v.size else 0.0,
                     num=float(v.size), sum=float(v.sum()), sum_sq=float((v * v).sum()),
                     zeros=float((v == 0).sum()), nonfinite=bad, counts=c)


class NonfiniteWatch:
    """Device-side sticky record of the first step whose loss was NaN/Inf."""

    def __init__(self, device: torch.device):
        self.device = device
        self.counter = torch.zeros(1, device=device, dtype=torch.int32)
        self.first_bad = torch.full((1,), -1, device=device, dtype=torch.int32)
        self._base = 0

    def reset(self, base_step: int) -> None:
        """Step numbering starts at ``base_step`` (resume)."""
        self._base = int(base_step)
        self.counter.zero_()
        self.first_bad.fill_(-1)

    def update(self, loss: torch.Tensor) -> None:
        loss = loss.detach().float().reshape(1)
        if loss.is_cuda:
            from ..ops import _ext
            _ext.ext().nonfinite_watch(loss.contiguous(), self.counter, self.first_bad)
            return
        s = int(self.counter.item())
        if not bool(torch.isfinite(loss).all()) and int(self.first_bad.item()) < 0:
            self.first_bad.fill_(s)
        self.counter.add_(1)

    def first_bad_step(self) -> Optional[int]:
        """Host read (call where the host synchronises anyway). None if every step was finite."""
        v = int(self.first_bad.item())
        return None if v < 0 else self._base + v
