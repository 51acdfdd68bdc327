"""Conv front-end on the HIP engine.

conv1/conv2 run as bf16 convolutions; their BatchNorm + clipped-ReLU epilogues are the
fused kernels of csrc/bn_act.hip. The conv2 epilogue writes the RNN input directly in
time-major [T2, N, C*F2] order (reference transpose+reshape, src/deepSpeech_NCHW.py:166-168).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext
from .optim import arena_of, emit_grad
from ..utils import trace as TR

BN_EPS = 1e-3
BN_MOMENTUM = 0.01


class BNClip(torch.autograd.Function):
    """out = clip(BN_train(y) * gamma + beta, 0, 20); layout 0 = NCHW, 1 = [T, N, C*F]."""

    @staticmethod
    def forward(ctx, y, gamma, beta, run_mean, run_var, training: bool, layout: int, out_dtype, idx: int = 0):
        C_ = _ext.ext()
        y = y.contiguous()
        N, C, T, Fd = y.shape
        dev = y.device
        gamma_p, beta_p = gamma, beta
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
        ctx.g_param, ctx.b_param = gamma_p, beta_p
        ctx.layout = layout
        ctx.training = training
        ctx.idx = idx
        return out

    @staticmethod
    def backward(ctx, dout):
        if not ctx.training:
            raise RuntimeError("BNClip backward is only defined in training mode")
        with TR.phase(TR.bn(ctx.idx, True)):
            return BNClip._backward(ctx, dout)

    @staticmethod
    def _backward(ctx, dout):
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
        return dy, emit_grad(ctx.g_param, dgamma), emit_grad(ctx.b_param, dbeta), None, None, None, None, None, None


class ConvFused(torch.autograd.Function):
    """bf16 conv2d (library kernel) whose weight gradient goes straight to the fp32 arena.

    The conv bias feeds a train-mode BatchNorm, whose mean subtraction removes any
    per-channel shift: its gradient is identically zero (sum over N,T,F of the BN input
    gradient), so no reduction is launched for it in training mode."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, bias_grad_zero: bool, idx: int = 0):
        w16 = weight.bf16 if arena_of(weight) is not None else weight.to(torch.bfloat16)
        b16 = bias.bf16 if arena_of(bias) is not None else bias.to(torch.bfloat16)
        x16 = x.to(torch.bfloat16)
        y = F.conv2d(x16, w16, b16, stride=stride)
        ctx.save_for_backward(x16, w16)
        ctx.stride = stride
        ctx.params = (weight, bias)
        ctx.bias_grad_zero = bias_grad_zero
        ctx.idx = idx
        return y

    @staticmethod
    def backward(ctx, dy):
        with TR.phase(TR.conv(ctx.idx, True)):
            return ConvFused._backward(ctx, dy)

    @staticmethod
    def _backward(ctx, dy):
        x16, w16 = ctx.saved_tensors
        weight, bias = ctx.params
        need_x = ctx.needs_input_grad[0]
        dy = dy.contiguous()
        gi, gw, gb = torch.ops.aten.convolution_backward(
            dy, x16, w16, [w16.shape[0]], list(ctx.stride), [0, 0], [1, 1], False, [0, 0], 1,
            [need_x, True, not ctx.bias_grad_zero])
        gw_out = emit_grad(weight, gw.float())
        if ctx.bias_grad_zero:
            if arena_of(bias) is not None:
                arena_of(bias).grad_done(bias)    # main_grad already zeroed by zero_grad()
                gb_out = None
            else:
                gb_out = torch.zeros_like(bias)
        else:
            gb_out = emit_grad(bias, gb.float())
        return (gi if need_x else None), gw_out, gb_out, None, None, None


def conv_block_hip(block, x: torch.Tensor, layout: int, idx: int) -> torch.Tensor:
    dt = torch.bfloat16
    with TR.phase(TR.conv(idx)):
        y = ConvFused.apply(x, block.weight, block.bias, tuple(block.stride), bool(block.training), idx)
    with TR.phase(TR.bn(idx)):
        return BNClip.apply(y, block.bn_gamma, block.bn_beta, block.running_mean, block.running_var,
                            block.training, layout, dt, idx)


def frontend_hip(model, feats: torch.Tensor) -> torch.Tensor:
    x = feats.unsqueeze(1)
    x = conv_block_hip(model.conv1, x, 0, 1)
    return conv_block_hip(model.conv2, x, 1, 2)


class FusedHead(torch.autograd.Function):
    """Time-major logits = h W_fc^T + b_fc (bf16), weight gradients straight to the arena."""

    @staticmethod
    def forward(ctx, h, weight, bias):
        T, N, H = h.shape
        w16 = weight.bf16 if arena_of(weight) is not None else weight.to(torch.bfloat16)
        b16 = bias.bf16 if arena_of(bias) is not None else bias.to(torch.bfloat16)
        h2 = h.to(torch.bfloat16).reshape(T * N, H)
        out = torch.addmm(b16, h2, w16.t()).view(T, N, -1)
        ctx.save_for_backward(h2, w16)
        ctx.params = (weight, bias)
        return out

    @staticmethod
    def backward(ctx, dout):
        with TR.phase(TR.SOFTMAX_B):
            return FusedHead._backward(ctx, dout)

    @staticmethod
    def _backward(ctx, dout):
        h2, w16 = ctx.saved_tensors
        weight, bias = ctx.params
        T, N, K = dout.shape
        d2 = dout.to(torch.bfloat16).reshape(T * N, K)
        dh = torch.mm(d2, w16).view(T, N, -1) if ctx.needs_input_grad[0] else None
        from .optim import mm_into
        gw = mm_into(weight, d2.t(), h2)
        if gw is None:
            arena_of(weight).grad_done(weight)
        gb = emit_grad(bias, d2.sum(0, dtype=torch.float32))
        return dh, gw, gb
