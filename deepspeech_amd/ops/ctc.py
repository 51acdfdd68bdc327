"""CTC loss on the HIP engine: fused log-softmax + alpha/beta + gradient (csrc/ctc.hip).

Like TF's CTCLoss op (reference src/deepSpeech_NCHW.py:225), the gradient with respect
to the logits is produced by the forward kernel and only scaled in backward.
"""
from __future__ import annotations

import os
import threading

import torch

_FC_SPLIT_MAX = 16         # split-K ceiling of the FC head's weight-gradient GEMM

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


_watch_ctx = threading.local()
# batch-mean loss and the divergence watch inside the CTC gradient launch (False: torch's mean
# and a separate watch launch; measured same box, 3 rounds, graph steps: 100 frames 1.483-1.485
# vs 1.486-1.495 ms, 200 frames 2.171-2.174 vs 2.177-2.182 ms; headline within spread)
_FUSE_LOSS = True


class loss_watch:
    """Context of one training step's forward: the fused head + CTC (FusedHeadCTC) writes the
    batch-mean loss and runs the step's divergence watch (utils/stats.py NonfiniteWatch:
    counter / first-bad words) inside its gradient launch, instead of a reduction kernel and a
    1-thread kernel behind it. ``consumed`` is False when no fused head took it (the reference
    engine, a CPU watch): the caller then runs ``watch.update(loss)`` itself."""

    def __init__(self, watch):
        self.watch = watch
        self.consumed = False
        self._prev = None

    def __enter__(self):
        self._prev = getattr(_watch_ctx, "cur", None)
        _watch_ctx.cur = self
        return self

    def __exit__(self, *exc):
        _watch_ctx.cur = self._prev
        return False


class FusedHeadCTC(torch.autograd.Function):
    """Mean CTC loss of the FC head's logits without materialising them (training path).

    forward : csrc/ctc.hip ds2_head_ctc — FC on MFMA + log-softmax in registers -> lp
              workspace -> alpha/beta recursion -> G = dloss_b/dlogits [T*N, 32] bf16
    backward: scale = gloss / N as a DEVICE scalar folded into the GEMM epilogues (no sync)
              dh     = scale * G W_fc          csrc/gemm.hip, critical path (feeds the top BPTT)
              dW_fc  = scale * G^T h           csrc/gemm.hip, weight-gradient side stream
              db_fc  = scale * sum_rows G      side stream
    Reference: FC src/deepSpeech_NCHW.py:188-198, CTC :225 (blank = last class)."""

    @staticmethod
    def forward(ctx, h, weight, bias, lens, labels, label_lens, blank: int, zero_infinity: bool):
        from .optim import arena_of
        C = _ext.ext()
        T, N, H = h.shape
        K = weight.shape[0]
        dev = h.device
        if arena_of(weight) is not None:
            arena_of(weight).await_params(weight, bias)      # a carried optimizer update (Trainer)
        h = h.to(torch.bfloat16).contiguous()
        w16 = weight.bf16 if arena_of(weight) is not None else weight.detach().to(torch.bfloat16).contiguous()
        b16 = bias.bf16 if arena_of(bias) is not None else bias.detach().to(torch.bfloat16).contiguous()
        labels = labels.to(device=dev, dtype=torch.int32).contiguous()
        if labels.dim() == 1:
            labels = labels.view(N, -1)
        if labels.shape[1] == 0:
            labels = torch.zeros(N, 1, device=dev, dtype=torch.int32)
        lens = lens.to(device=dev, dtype=torch.int32).contiguous()
        label_lens = label_lens.to(device=dev, dtype=torch.int32).contiguous()
        loss = torch.empty(N, device=dev, dtype=torch.float32)
        G = torch.empty(T * N, 32, device=dev, dtype=torch.bfloat16)
        ws = torch.empty(int(C.ctc_ws_floats(T, N, labels.shape[1])), device=dev, dtype=torch.float32)
        if not _FUSE_LOSS:
            C.head_ctc(h, w16, b16, lens, labels, label_lens, loss, G, ws, blank, zero_infinity)
            ctx.save_for_backward(h, G, w16)
            ctx.params = (weight, bias)
            ctx.K = K
            return loss.mean()
        mean = torch.empty((), device=dev, dtype=torch.float32)
        lw = getattr(_watch_ctx, "cur", None)
        watch = {}
        if lw is not None and not lw.consumed and lw.watch.counter.device == dev:
            watch = dict(counter=lw.watch.counter, first_bad=lw.watch.first_bad)
            lw.consumed = True
        C.head_ctc(h, w16, b16, lens, labels, label_lens, loss, G, ws, blank, zero_infinity, mean=mean, **watch)
        ctx.save_for_backward(h, G, w16)
        ctx.params = (weight, bias)
        ctx.K = K
        return mean

    @staticmethod
    def backward(ctx, gloss):
        with TR.phase(TR.CTC_B):
            return FusedHeadCTC._backward(ctx, gloss)

    @staticmethod
    def _backward(ctx, gloss):
        from . import gemm as GM
        from .optim import arena_of, emit_grad
        from .rnn import _stream_wait, wgrad_stream
        h, G, w16 = ctx.saved_tensors
        weight, bias = ctx.params
        T, N, H = h.shape
        K = ctx.K
        M = T * N
        # the upstream gradient stays a device scalar (no host sync); 1/N goes into the host
        # alpha of the critical-path dh GEMM, so no division kernel runs on the main stream
        g32 = gloss.to(torch.float32).reshape(1).contiguous()
        h2 = h.view(M, H)
        dh = None
        if ctx.needs_input_grad[0]:
            dh = torch.empty(M, H, device=h.device, dtype=torch.bfloat16)
            # K = 32 padded classes; rows >= K of W_fc are never loaded (Kl) and meet G's zero columns
            GM.gemm(G, w16, dh, M, H, 32, False, True, 0, 1.0 / N, None, alpha_dev=g32, Kl=K)
            dh = dh.view(T, N, H)
        side = wgrad_stream(h.device, arena_of(weight)) if arena_of(bias) is not None else None
        if side is None:
            gw, gb = FusedHeadCTC._weight_grads(weight, bias, G, h2, g32, 1.0 / N, K)
            return dh, gw, gb, None, None, None, None, None
        _stream_wait(side, torch.cuda.current_stream(h.device))
        arena_of(weight).wgrad.hold(G, h2, g32)
        with torch.cuda.stream(side):
            gw, gb = FusedHeadCTC._weight_grads(weight, bias, G, h2, g32, 1.0 / N, K)
        return dh, gw, gb, None, None, None, None, None

    @staticmethod
    def _weight_grads(weight, bias, G, h2, scale, inv_n, K):
        """dW_fc and db_fc, both scaled by the device scalar ``scale`` times the host ``inv_n``
        (folded into the GEMM and reduction epilogues: no division kernel)."""
        from . import gemm as GM
        from .optim import arena_of, emit_grad
        M, H = h2.shape
        a = arena_of(weight)
        # dW_fc = G^T h: a [K x H] output (7 column tiles) over M = T*N tokens. Split over the
        # token dimension as a batch of S partial GEMMs (7 -> 7*S workgroups; the unsplit
        # call ran 110 us on 7 CUs beside the top BPTT) and sum the partials.
        S = 1
        while S < _FC_SPLIT_MAX and M % (2 * S) == 0:
            S *= 2
        if S > 1:
            parts = torch.empty(S, K, H, device=h2.device, dtype=torch.float32)
            GM.gemm(G.view(S, M // S, G.shape[1]), h2.view(S, M // S, H), parts, K, H, M // S, True, True, 1, inv_n,
                    None, alpha_dev=scale, Ml=32)
        if a is not None:
            if S > 1:
                if weight.main_grad.is_contiguous():
                    # the S partials summed straight into the arena (csrc/reduce.hip col_sum)
                    _ext.ext().col_sum([parts.view(1, S, K * H)], [weight.main_grad], [not a.first_write(weight)])
                elif a.first_write(weight):
                    torch.sum(parts, 0, out=weight.main_grad)
                else:
                    weight.main_grad.add_(parts.sum(0))
            else:
                # M = K rows stored; G is read as a [M_rows, 32]-column col-mode operand (Ml = 32)
                GM.gemm(G, h2, weight.main_grad, K, H, M, True, True, 1 if a.first_write(weight) else 2, inv_n, None,
                        alpha_dev=scale, Ml=32)
            a.grad_done(weight)
            gw = None
        elif S > 1:
            gw = parts.sum(0)
        else:
            out = torch.empty(K, H, device=h2.device, dtype=torch.float32)
            GM.gemm(G, h2, out, K, H, M, True, True, 1, inv_n, None, alpha_dev=scale, Ml=32)
            gw = out
        ab = arena_of(bias)
        if ab is not None and G.is_cuda and bias.main_grad.is_contiguous():
            # db = scale * column sums of G in one launch straight into the arena (csrc/reduce.hip)
            _ext.ext().fc_bias_grad(G, K, scale, float(inv_n), bias.main_grad.view(-1), not ab.first_write(bias))
            ab.grad_done(bias)
            return gw, None
        gb = emit_grad(bias, G[:, :K].sum(0, dtype=torch.float32) * (scale * inv_n))
        return gw, gb


def head_ctc_mean_loss_hip(h: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, lens: torch.Tensor,
                           labels: torch.Tensor, label_lens: torch.Tensor, blank: int = BLANK,
                           zero_infinity: bool = True) -> torch.Tensor:
    """FC head + mean CTC loss in one fused op (HIP engine training path)."""
    with TR.phase(TR.CTC_F):
        return FusedHeadCTC.apply(h, weight, bias, lens, labels, label_lens, blank, zero_infinity)


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
