"""Flat parameter arena + fused Adam/EMA optimizer.

Reference: tf.train.AdamOptimizer(lr) + ExponentialMovingAverage(decay, global_step)
(src/deepSpeech_train.py:430,457-465) with the staircase exponential-decay LR of
:231-250.

All trainable parameters live as views in ONE contiguous fp32 buffer (``flat``) with
gradients as views in ``grad``. That makes
  * the whole optimizer step one streaming kernel (csrc/optim.hip) on the GPU,
  * gradient all-reduce buckets plain contiguous slices (parallel/grad_sync.py),
  * zero_grad one memset.
The arena is laid out in REVERSE parameter registration order, which is the order
backward produces gradients (FC first, conv1 last), so early buckets fill first.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional, Tuple

import torch
import torch.nn as nn

from . import _ext


class ParamArena:
    def __init__(self, model: nn.Module, align: int = 64):
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        named = list(reversed(named))
        self.names: List[str] = [n for n, _ in named]
        self.params: List[nn.Parameter] = [p for _, p in named]
        dev = self.params[0].device
        self.offsets: List[Tuple[int, int]] = []
        off = 0
        for p in self.params:
            n = p.numel()
            self.offsets.append((off, n))
            off += -(-n // align) * align           # 256-B aligned views
        self.numel = off
        self.flat = torch.zeros(off, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(off, device=dev, dtype=torch.float32)
        for p, (o, n) in zip(self.params, self.offsets):
            self.flat[o:o + n].copy_(p.data.reshape(-1).float())
            p.data = self.flat[o:o + n].view_as(p)
            p.grad = self.grad[o:o + n].view_as(p)

    def zero_grad(self) -> None:
        self.grad.zero_()
        # re-attach in case an op replaced a .grad (e.g. set_to_none elsewhere)
        for p, (o, n) in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + n].data_ptr():
                p.grad = self.grad[o:o + n].view_as(p)

    def views(self, buf: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {n: buf[o:o + c].view_as(p) for n, p, (o, c) in zip(self.names, self.params, self.offsets)}

    def param_range(self, name: str) -> Tuple[int, int]:
        i = self.names.index(name)
        return self.offsets[i]


def exponential_decay(initial_lr: float, step: int, decay_steps: int, decay_rate: float,
                      staircase: bool = True) -> float:
    """tf.train.exponential_decay (src/deepSpeech_train.py:245-249)."""
    p = step / float(max(1, decay_steps))
    if staircase:
        p = math.floor(p)
    return initial_lr * (decay_rate ** p)


class FusedAdamEMA:
    """Adam (TF epsilon-hat form) + weight EMA over a ParamArena."""

    def __init__(self, arena: ParamArena, lr: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 ema_decay: Optional[float] = 0.9999, bf16_copy: bool = False):
        self.arena = arena
        self.lr = lr
        self.b1, self.b2 = betas
        self.eps = eps
        self.ema_decay = ema_decay
        dev = arena.flat.device
        self.m = torch.zeros_like(arena.flat)
        self.v = torch.zeros_like(arena.flat)
        self.ema = arena.flat.clone() if ema_decay is not None else None
        self.p16 = (torch.empty(arena.numel, device=dev, dtype=torch.bfloat16) if bf16_copy else None)
        self.t = 0          # number of applied updates (Adam bias-correction power)
        self.use_hip = dev.type == "cuda"
        if self.p16 is not None and self.use_hip:
            _ext.ext().cast_bf16(arena.flat, self.p16)
        self._norm_part = None
        self._bad = None

    # TF ExponentialMovingAverage with num_updates: min(decay, (1+n)/(10+n))
    def ema_keep(self, global_step: int) -> float:
        return min(self.ema_decay, (1.0 + global_step) / (10.0 + global_step))

    def grad_norm_and_finite(self, gscale: float = 1.0) -> Tuple[torch.Tensor, torch.Tensor]:
        """(||g||_2, non-finite flag) as device tensors (no host sync)."""
        g = self.arena.grad
        if self.use_hip:
            C = _ext.ext()
            if self._norm_part is None:
                nb = int(C.grad_norm_blocks(g.numel()))
                self._norm_part = torch.empty(nb, device=g.device, dtype=torch.float32)
                self._bad = torch.zeros(1, device=g.device, dtype=torch.int32)
            self._bad.zero_()
            C.grad_norm(g, gscale, self._norm_part, self._bad)
            return self._norm_part.sum().sqrt(), self._bad
        gg = g * gscale
        return gg.norm(), (~torch.isfinite(gg)).any().to(torch.int32).view(1)

    @torch.no_grad()
    def step(self, lr: float, global_step: int, gscale: float = 1.0,
             skip_flag: Optional[torch.Tensor] = None) -> None:
        self.t += 1
        lr_t = lr * math.sqrt(1.0 - self.b2 ** self.t) / (1.0 - self.b1 ** self.t)
        keep = self.ema_keep(global_step) if self.ema is not None else 0.0
        a = self.arena
        if self.use_hip:
            _ext.ext().adam_ema(a.flat, a.grad, self.m, self.v, self.ema, self.p16, lr_t, self.b1, self.b2,
                                self.eps, gscale, keep, skip_flag)
            return
        if skip_flag is not None and int(skip_flag.item()) != 0:
            return
        g = a.grad * gscale
        self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
        self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
        a.flat.sub_(lr_t * self.m / (self.v.sqrt() + self.eps))
        if self.ema is not None:
            self.ema.copy_(a.flat + keep * (self.ema - a.flat))
        if self.p16 is not None:
            self.p16.copy_(a.flat)

    def state_dict(self) -> Dict[str, object]:
        return {"m": self.m, "v": self.v, "ema": self.ema, "t": self.t}

    def load_state_dict(self, sd: Dict[str, object]) -> None:
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        if self.ema is not None and sd.get("ema") is not None:
            self.ema.copy_(sd["ema"])
        self.t = int(sd["t"])
