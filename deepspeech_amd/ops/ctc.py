"""CTC loss on the HIP engine: fused log-softmax + alpha/beta + gradient (csrc/ctc.hip).

Like TF's CTCLoss op (reference src/deepSpeech_NCHW.py:225), the gradient with respect
to the logits is produced by the forward kernel and only scaled in backward.
"""
from __future__ import annotations

import torch

from .. import BLANK
from . import _ext
from ..utils import trace as TR


class CTCLossFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, lens, labels, label_lens, blank: int, zero_infinity: bool):
        C = _ext.ext()
        T, N, K = logits.shape
        dev = logits.device
        logits = logits.contiguous()
        if logits.dtype not in (torch.float32, torch.bfloat16):
            logits = logits.float()
        labels = labels.to(device=dev, dtype=torch.int32).contiguous()
        if labels.dim() == 1:
            labels = labels.view(N, -1)
        Lmax = max(1, labels.shape[1])
        if labels.shape[1] == 0:
            labels = torch.zeros(N, 1, device=dev, dtype=torch.int32)
        lens = lens.to(device=dev, dtype=torch.int32).contiguous()
        label_lens = label_lens.to(device=dev, dtype=torch.int32).contiguous()
        loss = torch.empty(N, device=dev, dtype=torch.float32)
        grad = torch.empty_like(logits)
        ws = torch.empty(int(C.ctc_ws_floats(T, N, labels.shape[1])), device=dev, dtype=torch.float32)
        C.ctc_fused(logits, lens, labels, label_lens, loss, grad, ws, blank, zero_infinity)
        ctx.save_for_backward(grad)
        ctx.in_dtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, gloss):
        with TR.phase(TR.CTC_B):
            (grad,) = ctx.saved_tensors
            return CTCLossFused._scale(grad, gloss)

    @staticmethod
    def _scale(grad, gloss):
        g = grad * gloss.to(grad.dtype).view(1, -1, 1)
        return g, None, None, None, None, None


class CTCMeanFused(CTCLossFused):
    """Mean CTC loss over the batch. The gradient for the mean is the saved per-utterance
    gradient times gloss / N, one scalar-broadcast multiply (instead of the mean's expand +
    divide and a per-utterance broadcast multiply)."""

    @staticmethod
    def forward(ctx, logits, lens, labels, label_lens, blank: int, zero_infinity: bool):
        loss = CTCLossFused.forward(ctx, logits, lens, labels, label_lens, blank, zero_infinity)
        ctx.n = loss.numel()
        return loss.mean()

    @staticmethod
    def backward(ctx, gloss):
        with TR.phase(TR.CTC_B):
            (grad,) = ctx.saved_tensors
            return grad * (gloss / ctx.n), None, None, None, None, None


def ctc_mean_loss_hip(logits: torch.Tensor, lens: torch.Tensor, labels: torch.Tensor,
                      label_lens: torch.Tensor, blank: int = BLANK, zero_infinity: bool = True) -> torch.Tensor:
    """Mean CTC loss over the batch (fp32 scalar)."""
    with TR.phase(TR.CTC_F):
        return CTCMeanFused.apply(logits, lens, labels, label_lens, blank, zero_infinity)


def ctc_loss_hip(logits: torch.Tensor, lens: torch.Tensor, labels: torch.Tensor,
                 label_lens: torch.Tensor, blank: int = BLANK, zero_infinity: bool = True) -> torch.Tensor:
    """Per-utterance CTC loss [N] (fp32)."""
    with TR.phase(TR.CTC_F):
        return CTCLossFused.apply(logits, lens, labels, label_lens, blank, zero_infinity)
