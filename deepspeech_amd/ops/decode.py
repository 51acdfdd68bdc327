"""CTC decoding entry points.

greedy: csrc/decode.hip on the GPU (argmax + merge repeats + drop blank + path score in one
        kernel per utterance; reference tf.nn.ctc_greedy_decoder, src/deepSpeech_test.py:212-215),
        plain PyTorch (ops/reference.py) on the CPU.
beam:   CTC prefix beam search in the native host runtime (runtime/decoder.cpp), one thread
        per utterance.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from .. import BLANK
from . import reference as R


def greedy_decode(logits: torch.Tensor, lens: torch.Tensor, blank: int = BLANK,
                  with_scores: bool = False):
    """logits [T, N, K] time-major (raw logits or log-probs) -> label lists (and the
    greedy-path log-probabilities when ``with_scores``)."""
    if logits.is_cuda:
        from . import _ext
        T, N, _ = logits.shape
        lg = logits if logits.dtype in (torch.float32, torch.bfloat16) else logits.float()
        lg = lg.contiguous()
        lens_d = lens.to(device=lg.device, dtype=torch.int32).contiguous()
        labels = torch.empty(N, T, device=lg.device, dtype=torch.int32)
        counts = torch.empty(N, device=lg.device, dtype=torch.int32)
        score = torch.empty(N, device=lg.device, dtype=torch.float32)
        _ext.ext().ctc_greedy(lg, lens_d, labels, counts, blank, score)
        counts_h = counts.cpu().tolist()
        lab_h = labels.cpu().numpy()
        out = [lab_h[n, :counts_h[n]].tolist() for n in range(N)]
        return (out, score.cpu()) if with_scores else out
    lp = torch.log_softmax(logits.float(), -1)
    out = R.greedy_decode(lp, lens, blank)
    if not with_scores:
        return out
    L = lens.cpu()
    sc = torch.stack([lp[: int(L[n]), n].max(-1).values.sum() for n in range(lp.shape[1])])
    return out, sc


def beam_decode(logits: torch.Tensor, lens: torch.Tensor, beam_width: int = 16, blank: int = BLANK,
                prune: float = -10.0) -> List[List[int]]:
    from ..runtime import native
    lp = torch.log_softmax(logits.float(), dim=-1).cpu().numpy()
    return native.load().beam_search_batch(lp, lens.cpu().numpy().astype(np.int32), beam_width, blank, prune)
