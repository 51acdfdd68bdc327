"""Conv front-end on the HIP engine.

conv1/conv2 run as bf16 convolutions; their BatchNorm + clipped-ReLU epilogues are the
fused kernels of csrc/bn_act.hip. The conv2 epilogue writes the RNN input directly in
time-major [T2, N, C*F2] order (reference transpose+reshape, src/deepSpeech_NCHW.py:166-168).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext

BN_EPS = 1e-3
BN_MOMENTUM = 0.01


class BNClip(torch.autograd.Function):
    """out = clip(BN_train(y) * gamma + beta, 0, 20); layout 0 = NCHW, 1 = [T, N, C*F]."""

    @staticmethod
    def forward(ctx, y, gamma, beta, run_mean, run_var, training: bool, layout: int, out_dtype):
        C_ = _ext.ext()
        y = y.contiguous()
        N, C, T, Fd = y.shape
        dev = y.device
        gamma = gamma.float().contiguous()
        beta = beta.float().contiguous()
        if training:
            nb = int(C_.bn_chunks(N, T, Fd))
            part = torch.empty(C * nb * 2, device=dev, dtype=torch.float32)
            mean = torch.empty(C, device=dev, dtype=torch.float32)
            invstd = torch.empty(C, device=dev, dtype=torch.float32)
            C_.bn_stats(y, part, BN_EPS, mean, invstd, run_mean, run_var, BN_MOMENTUM)
        else:
            mean = run_mean.float().contiguous()
            invstd = torch.rsqrt(run_var.float() + BN_EPS).contiguous()
        if layout == 0:
            out = torch.empty(N, C, T, Fd, device=dev, dtype=out_dtype)
        else:
            out = torch.empty(T, N, C * Fd, device=dev, dtype=out_dtype)
        C_.bn_apply(y, mean, invstd, gamma, beta, out, layout)
        ctx.save_for_backward(y, mean, invstd, gamma, beta)
        ctx.layout = layout
        ctx.training = training
        return out

    @staticmethod
    def backward(ctx, dout):
        if not ctx.training:
            raise RuntimeError("BNClip backward is only defined in training mode")
        C_ = _ext.ext()
        y, mean, invstd, gamma, beta = ctx.saved_tensors
        N, C, T, Fd = y.shape
        dout = dout.contiguous()
        nb = int(C_.bn_chunks(N, T, Fd))
        part = torch.empty(C * nb * 2, device=y.device, dtype=torch.float32)
        dgamma = torch.empty(C, device=y.device, dtype=torch.float32)
        dbeta = torch.empty(C, device=y.device, dtype=torch.float32)
        dy = torch.empty_like(y)
        C_.bn_bwd(dout, y, mean, invstd, gamma, beta, part, dgamma, dbeta, dy, ctx.layout)
        return dy, dgamma, dbeta, None, None, None, None, None


def conv_block_hip(block, x: torch.Tensor, layout: int) -> torch.Tensor:
    dt = x.dtype
    y = F.conv2d(x, block.weight.to(dt), block.bias.to(dt), stride=block.stride)
    return BNClip.apply(y, block.bn_gamma, block.bn_beta, block.running_mean, block.running_var,
                        block.training, layout, dt)


def frontend_hip(model, feats: torch.Tensor) -> torch.Tensor:
    x = feats.unsqueeze(1)
    x = conv_block_hip(model.conv1, x, 0)
    return conv_block_hip(model.conv2, x, 1)
