"""Pure-PyTorch reference implementations ("engine=ref").

These are the golden model for every HIP kernel test and the CPU plumbing path
(BASELINE config 1). They follow the reference's semantics op by op:

* clipped ReLU            — src/custom_ops.py:99-104
* get_rnn_seqlen          — src/deepSpeech.py:38-48
* ReLU-RNN cell (+SBN)    — src/custom_ops.py:36-72 (CustomRNNCell2)
* bidirectional dynamic RNN with per-utterance reversal and zero outputs past the
  length, directions summed — src/custom_ops.py:75-96, TF bidirectional_dynamic_rnn
* CTC loss (blank = last class, mean over batch) — src/deepSpeech_NCHW.py:204-228
* greedy CTC decoder      — src/deepSpeech_test.py:212-215

The GRU cell is the cuDNN/"reset-after" form so the recurrent product of all three
gates is one GEMM:  r,z = sigma(gx_rz + U_rz h + b_rz); n = tanh(gx_n + r*(U_n h + b_hn));
h' = (1-z) n + z h.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from .. import BLANK

RELU_CLIP = 20.0
SBN_EPS = 1e-5


def clipped_relu(x: torch.Tensor, cap: float = RELU_CLIP) -> torch.Tensor:
    return torch.clamp(x, min=0.0, max=cap)


def get_rnn_seqlen(seq_lens: torch.Tensor) -> torch.Tensor:
    """T2 = ceil((ceil((T-19)/2) - 9)/2) of the reference (src/deepSpeech.py:38-48).

    For integer T this is floor((floor((T-18)/2) - 8)/2) = floor((T-34)/4): two integer
    kernels instead of a float64 round trip (exact for every integer, negative included)."""
    s = seq_lens.to(torch.int32) if seq_lens.dtype != torch.int32 else seq_lens
    return torch.div(s - 34, 4, rounding_mode="floor").to(torch.int32)


def reverse_index(lens: torch.Tensor, T: int) -> torch.Tensor:
    """idx[t, b] = lens[b]-1-t for t < lens[b] else t  (TF ReverseSequence semantics)."""
    t = torch.arange(T, device=lens.device).unsqueeze(1)          # [T,1]
    L = lens.to(torch.long).unsqueeze(0)                          # [1,N]
    return torch.where(t < L, L - 1 - t, t.expand(T, L.shape[1]))


def reverse_sequence(x: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
    """Reverse x[T, N, ...] within each utterance's length (time-major)."""
    T = x.shape[0]
    idx = reverse_index(lens, T)
    idx = idx.view(T, idx.shape[1], *([1] * (x.dim() - 2))).expand_as(x)
    return torch.gather(x, 0, idx)


def time_mask(lens: torch.Tensor, T: int, dtype=torch.bool) -> torch.Tensor:
    """[T, N] mask, True where t < lens[b]."""
    t = torch.arange(T, device=lens.device).unsqueeze(1)
    return (t < lens.to(torch.long).unsqueeze(0)).to(dtype)


def seq_batch_norm(y: torch.Tensor, lens: torch.Tensor, mode: str,
                   moving_mean: Optional[torch.Tensor] = None,
                   moving_var: Optional[torch.Tensor] = None,
                   training: bool = True, momentum: float = 0.5) -> torch.Tensor:
    """Sequence-wise BN of the input projection y[T, N, D].

    mode 'frozen': normalise with the (never-updated) moving stats — reference parity
    (src/custom_ops.py:184-199, quirk Q3): y * 1/sqrt(var+eps) with mean 0 / var 1.
    mode 'batch' : DS2-paper sequence-wise BN — statistics over every valid (t, n)
    row during training (running stats updated), moving stats in eval.
    mode 'none'  : identity.
    """
    if mode == "none":
        return y
    if mode == "frozen" or not training:
        mean = moving_mean if moving_mean is not None else torch.zeros(y.shape[-1], device=y.device)
        var = moving_var if moving_var is not None else torch.ones(y.shape[-1], device=y.device)
        return (y - mean.to(y.dtype)) * torch.rsqrt(var.to(y.dtype) + SBN_EPS)
    T, N, D = y.shape
    m = time_mask(lens, T, y.dtype).unsqueeze(-1)               # [T,N,1]
    cnt = m.sum().clamp(min=1.0)
    mean = (y * m).sum(dim=(0, 1)) / cnt
    var = (((y - mean) * m) ** 2).sum(dim=(0, 1)) / cnt
    if moving_mean is not None:
        with torch.no_grad():
            moving_mean.mul_(momentum).add_((1 - momentum) * mean.detach().float())
            moving_var.mul_(momentum).add_((1 - momentum) * var.detach().float())
    return (y - mean) * torch.rsqrt(var + SBN_EPS)


# ---------------------------------------------------------------------------------
# single-direction recurrences over a precomputed input projection gx[T, N, G*H]
# ---------------------------------------------------------------------------------
def _mm_in(h: torch.Tensor, mm_dtype) -> torch.Tensor:
    """Operand rounding of the recurrent product (the HIP kernels feed h to MFMA in bf16
    while keeping the state itself in fp32); identity when mm_dtype is None."""
    return h if mm_dtype is None else h.to(mm_dtype).to(h.dtype)


def rnn_relu_scan(gx: torch.Tensor, U: torch.Tensor, lens: torch.Tensor,
                  h0: Optional[torch.Tensor] = None, cap: float = RELU_CLIP, mm_dtype=None
                  ) -> Tuple[torch.Tensor, torch.Tensor]:
    """h_t = min(relu(gx_t + U h_{t-1}), cap); gx already holds SBN(Wx) + B.

    Returns (outputs[T,N,H] with zeros past each length, final state[N,H])."""
    T, N, H = gx.shape
    h = gx.new_zeros(N, H) if h0 is None else h0
    mask = time_mask(lens, T).unsqueeze(-1)
    outs = []
    Ut = U.t()
    for t in range(T):
        hn = torch.clamp(gx[t] + _mm_in(h, mm_dtype) @ Ut, 0.0, cap)
        m = mask[t]
        outs.append(torch.where(m, hn, torch.zeros_like(hn)))
        h = torch.where(m, hn, h)
    return torch.stack(outs, 0), h


def gru_scan(gx: torch.Tensor, U: torch.Tensor, b_h: torch.Tensor, lens: torch.Tensor,
             h0: Optional[torch.Tensor] = None, mm_dtype=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Reset-after GRU over gx[T,N,3H] (gate order r, z, n)."""
    T, N, G3 = gx.shape
    H = G3 // 3
    h = gx.new_zeros(N, H) if h0 is None else h0
    mask = time_mask(lens, T).unsqueeze(-1)
    outs = []
    Ut = U.t()
    for t in range(T):
        gh = _mm_in(h, mm_dtype) @ Ut + b_h
        r = torch.sigmoid(gx[t, :, :H] + gh[:, :H])
        z = torch.sigmoid(gx[t, :, H:2 * H] + gh[:, H:2 * H])
        n = torch.tanh(gx[t, :, 2 * H:] + r * gh[:, 2 * H:])
        hn = (1.0 - z) * n + z * h
        m = mask[t]
        outs.append(torch.where(m, hn, torch.zeros_like(hn)))
        h = torch.where(m, hn, h)
    return torch.stack(outs, 0), h


def recurrent_scan(cell: str, gx, U, b_h, lens, h0=None, mm_dtype=None):
    if cell == "rnn_relu":
        return rnn_relu_scan(gx, U, lens, h0, mm_dtype=mm_dtype)
    if cell == "gru":
        return gru_scan(gx, U, b_h, lens, h0, mm_dtype=mm_dtype)
    raise ValueError(cell)


def birnn_ref(cell: str, gx_f: torch.Tensor, gx_b: Optional[torch.Tensor],
              U_f, U_b, bh_f, bh_b, lens: torch.Tensor, mm_dtype=None) -> torch.Tensor:
    """Bidirectional layer over precomputed projections; returns fw + bw (Q2)."""
    y_f, _ = recurrent_scan(cell, gx_f, U_f, bh_f, lens, mm_dtype=mm_dtype)
    if gx_b is None:
        return y_f
    y_b_rev, _ = recurrent_scan(cell, reverse_sequence(gx_b, lens), U_b, bh_b, lens, mm_dtype=mm_dtype)
    return y_f + reverse_sequence(y_b_rev, lens)


# ---------------------------------------------------------------------------------
# CTC
# ---------------------------------------------------------------------------------
def collapse_repeated(labels: Sequence[int]) -> List[int]:
    out: List[int] = []
    for c in labels:
        if not out or out[-1] != c:
            out.append(c)
    return out


def ctc_loss_ref(logits: torch.Tensor, targets: torch.Tensor, logit_lens: torch.Tensor,
                 target_lens: torch.Tensor, blank: int = BLANK,
                 zero_infinity: bool = True) -> torch.Tensor:
    """Per-utterance CTC negative log-likelihood over time-major logits [T, N, K].

    Returns the vector of losses [N] (fp32); the model reduces it with mean like
    tf.reduce_mean(ctc_loss) (src/deepSpeech_NCHW.py:225-226)."""
    lp = F.log_softmax(logits.float(), dim=-1)
    return F.ctc_loss(lp, targets, logit_lens.long(), target_lens.long(), blank=blank,
                      reduction="none", zero_infinity=zero_infinity)


def greedy_decode(logits: torch.Tensor, lens: torch.Tensor, blank: int = BLANK) -> List[List[int]]:
    """tf.nn.ctc_greedy_decoder(merge_repeated=True): argmax, merge repeats, drop blank."""
    best = logits.argmax(-1).cpu()            # [T, N]
    lens = lens.cpu()
    out = []
    for b in range(best.shape[1]):
        seq = best[: int(lens[b]), b].tolist()
        res, prev = [], None
        for c in seq:
            if c != prev and c != blank:
                res.append(c)
            prev = c
        out.append(res)
    return out
