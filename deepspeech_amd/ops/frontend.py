"""Conv front-end on the HIP engine.

Default (32 filters, the reference geometry): FrontendCL — the channels-last implicit-GEMM
MFMA kernels of csrc/conv_frontend.hip for conv fwd / dgrad / wgrad with BatchNorm
statistics fused into the conv epilogues and channels-last BN + clipped-ReLU kernels; the
conv2 BN apply writes the RNN input directly in time-major [T2, N, C*F2] order (reference
transpose+reshape, src/deepSpeech_NCHW.py:166-168).

Other filter counts: library bf16 convolutions (ConvFused) with the NCHW BN + clip kernels
of csrc/bn_act.hip (BNClip).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _ext
from .optim import arena_of, emit_grad
from ..utils import trace as TR

_HEAD_SIDE = True         # FC-head weight gradient on the side stream

BN_EPS = 1e-3
BN_MOMENTUM = 0.01



# conv1 weight-gradient workgroups per CU (its 67.5 KB of LDS allows two)
_C1W_BPC = 1

# conv2's weight gradient on a stream of its own, beside the conv2 data gradient -> BN1 ->
# conv1 weight-gradient chain it does not feed. Off by default (DS2_CONV_WSIDE=1 turns it on):
# single device 7.345 vs 7.354-7.361 ms/step (noise level), but the data-parallel step ran
# 9.36-9.44 instead of 7.63 ms/step with it and its kernel trace showed ~0.7 ms of idle gaps
# at the end of the single-device step too, a host-side stall not explained this round
# (profiles/r6_negative_results.md)
_CONV_WSIDE = os.environ.get("DS2_CONV_WSIDE", "0") == "1"
_conv_streams = {}



def _conv_side_stream(dev, w):
    """The conv2 weight-gradient stream, or None (off, no GPU, a single-stream capture, or a
    gradient bucketer attached: the data-parallel step measured 9.36-9.44 ms/step with it
    against 7.63 without at world 1, scripts/r6_dpcheck.sh, so DP keeps it in line)."""
    a = arena_of(w)
    if not _CONV_WSIDE or dev.type != "cuda" or (a is not None and (a.wgrad.single_stream or
                                                                  getattr(a, "_ready_cbs", None))):
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _conv_streams.get(idx)
    if s is None:
        s = _conv_streams[idx] = torch.cuda.Stream(device=torch.device("cuda", idx))
    return s

def bn_eval_stats(block, eps: float):
    """(mean, invstd) for eval: running statistics (fused variant) or the debiased EMA of
    the moments (moments_ema variant, NHWC graph)."""
    if getattr(block, "bn", "fused") == "moments_ema":
        m, v = block.ema_moments()
        return m.float().contiguous(), torch.rsqrt(v.float() + eps).contiguous()
    return block.running_mean.float().contiguous(), torch.rsqrt(block.running_var.float() + eps).contiguous()


def bn_track(block, mean: torch.Tensor, invstd: torch.Tensor, eps: float) -> None:
    """moments_ema variant: feed the batch moments (variance recovered from invstd) into the
    zero-debiased EMA (the kernels' own running-stat update went to scratch buffers)."""
    if getattr(block, "bn", "fused") == "moments_ema":
        block.ema_update(mean, invstd.pow(-2) - eps)


def _stat_buffers(block, dev):
    """Running-stat buffers the kernels update in place: the block's own for the fused
    variant, scratch for moments_ema (tracked by bn_track instead)."""
    if getattr(block, "bn", "fused") == "moments_ema":
        return torch.zeros(block.bn_gamma.numel(), device=dev), torch.ones(block.bn_gamma.numel(), device=dev)
    return block.running_mean, block.running_var


class BNClip(torch.autograd.Function):
    """out = clip(BN_train(y) * gamma + beta, 0, 20); layout 0 = NCHW, 1 = [T, N, C*F]."""

    @staticmethod
    def forward(ctx, y, gamma, beta, run_mean, run_var, training: bool, layout: int, out_dtype, idx: int = 0,
                block=None):
        C_ = _ext.ext()
        y = y.contiguous()
        N, C, T, Fd = y.shape
        dev = y.device
        gamma_p, beta_p = gamma, beta
        gamma = gamma.float().contiguous()
        beta = beta.float().contiguous()
        eps = getattr(block, "bn_eps", BN_EPS)
        if training:
            nb = int(C_.bn_chunks(N, T, Fd))
            part = torch.empty(C * nb * 2, device=dev, dtype=torch.float32)
            mean = torch.empty(C, device=dev, dtype=torch.float32)
            invstd = torch.empty(C, device=dev, dtype=torch.float32)
            if block is not None:
                run_mean, run_var = _stat_buffers(block, dev)
            C_.bn_stats(y, part, eps, mean, invstd, run_mean, run_var, BN_MOMENTUM)
            if block is not None:
                bn_track(block, mean, invstd, eps)
        elif block is not None:
            mean, invstd = bn_eval_stats(block, eps)
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
        return (dy, emit_grad(ctx.g_param, dgamma), emit_grad(ctx.b_param, dbeta), None, None, None, None, None, None,
                None)


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
            gb_out = _zero_grad_of(bias)
        else:
            gb_out = emit_grad(bias, gb.float())
        return (gi if need_x else None), gw_out, gb_out, None, None, None


def conv_block_hip(block, x: torch.Tensor, layout: int, idx: int) -> torch.Tensor:
    dt = torch.bfloat16
    with TR.phase(TR.conv(idx)):
        y = ConvFused.apply(x, block.weight, block.bias, tuple(block.stride), bool(block.training), idx)
    with TR.phase(TR.bn(idx)):
        return BNClip.apply(y, block.bn_gamma, block.bn_beta, block.running_mean, block.running_var,
                            block.training, layout, dt, idx, block)


def _bf16_of(p: torch.Tensor) -> torch.Tensor:
    return p.bf16 if arena_of(p) is not None else p.detach().to(torch.bfloat16).contiguous()


def _grad_buffer(p: torch.Tensor):
    """(fp32 buffer a kernel may overwrite with p's full gradient, written_in_place)."""
    a = arena_of(p)
    if a is not None and a.first_write(p):
        return p.main_grad, True
    return torch.empty(p.shape, device=p.device, dtype=torch.float32), False


def _deliver(p: torch.Tensor, buf: torch.Tensor, in_place: bool):
    if in_place:
        arena_of(p).grad_done(p)
        return None
    return emit_grad(p, buf)


def _zero_grad_of(p: torch.Tensor):
    """Gradient of a conv bias that feeds a train-mode BatchNorm: identically zero."""
    a = arena_of(p)
    if a is not None:
        if a.first_write(p) and not a.known_zero(p):
            p.main_grad.zero_()     # the arena may be zeroed lazily: write the zeros
        a.grad_done(p)
        a.set_known_zero(p)         # until another op writes it, later steps need no kernel
        return None
    return torch.zeros_like(p)


class FrontendCL(torch.autograd.Function):
    """Whole conv front-end on the channels-last MFMA kernels of csrc/conv_frontend.hip.

    feats [N, T, F0] -> time-major RNN input [T2, N, 32*F2] (bf16). Forward: conv1 (+bias,
    BN statistics in the epilogue) -> BN finalize -> BN+clip apply -> conv2 (+bias, stats)
    -> finalize -> BN+clip apply with the time-major transpose in the store. Backward:
    BN2 backward (reads the time-major gradient through an LDS transpose) -> conv2 wgrad
    (fp32 straight into the arena) and dgrad -> BN1 backward -> conv1 wgrad. Reference:
    src/deepSpeech_NCHW.py:110-168, src/custom_ops.py:99-160."""

    @staticmethod
    def forward(ctx, feats, w1, b1, g1, be1, w2, b2, g2, be2, model):
        C_ = _ext.ext()
        dev = feats.device
        if arena_of(w1) is not None:
            arena_of(w1).await_params(w1, b1, g1, be1, w2, b2, g2, be2)
        x = feats.to(torch.bfloat16).contiguous()
        N, T, F0 = x.shape
        T1, F1 = (T - 20) // 2 + 1, (F0 - 5) // 2 + 1
        T2, F2 = (T1 - 10) // 2 + 1, F1 - 4
        c1, c2 = model.conv1, model.conv2
        training = bool(c1.training)
        f32 = dict(device=dev, dtype=torch.float32)
        bf = dict(device=dev, dtype=torch.bfloat16)
        ncu = _ext.num_cus(dev.index or 0)

        def stats(part, nb, M, blk):
            eps = getattr(blk, "bn_eps", BN_EPS)
            if training:
                mean = torch.empty(32, **f32)
                inv = torch.empty(32, **f32)
                rm, rv = _stat_buffers(blk, dev)
                C_.bn_cl_finalize(part, nb, float(M), eps, mean, inv, rm, rv, BN_MOMENTUM)
                bn_track(blk, mean, inv, eps)
                return mean, inv
            return bn_eval_stats(blk, eps)

        g1f, be1f = g1.detach().float().contiguous(), be1.detach().float().contiguous()
        g2f, be2f = g2.detach().float().contiguous(), be2.detach().float().contiguous()
        with TR.phase(TR.conv(1)):
            y1 = torch.empty(N, T1, F1, 32, **bf)
            nb1 = int(C_.conv1_fwd_grid(N, T1))
            part1 = torch.empty(nb1 * 64, **f32)
            C_.conv1_fwd(x, _bf16_of(w1), b1.detach().float().contiguous(), y1, part1)
        with TR.phase(TR.bn(1)):
            mean1, inv1 = stats(part1, nb1, N * T1 * F1, c1)
            z1 = torch.empty_like(y1)
            C_.bn_cl_apply(y1, mean1, inv1, g1f, be1f, z1, False)
        w2_16 = _bf16_of(w2)
        with TR.phase(TR.conv(2)):
            y2 = torch.empty(N, T2, F2, 32, **bf)
            grid = max(1, min(N * T2, 2 * ncu))                 # two workgroups per CU
            part2 = torch.empty(grid * 64, **f32)
            C_.conv2_fwd(z1, w2_16, b2.detach().float().contiguous(), y2, part2, grid)
        with TR.phase(TR.bn(2)):
            mean2, inv2 = stats(part2, grid, N * T2 * F2, c2)
            out = torch.empty(T2, N, 32 * F2, **bf)
            C_.bn_cl_apply(y2, mean2, inv2, g2f, be2f, out, True)
        if getattr(model, "capture", False):
            model.act_taps["conv1"] = z1.detach()      # [N, T1, F1, C] channels-last
            model.act_taps["conv2"] = out.detach()     # time-major [T2, N, C*F2]
        ctx.save_for_backward(x, y1, z1, y2, mean1, inv1, mean2, inv2, g1f, be1f, g2f, be2f, w2_16)
        ctx.params = (w1, b1, g1, be1, w2, b2, g2, be2)
        ctx.training = training
        ctx.ncu = ncu
        return out

    @staticmethod
    def backward(ctx, dout):
        if not ctx.training:
            raise RuntimeError("FrontendCL backward is only defined in training mode")
        C_ = _ext.ext()
        x, y1, z1, y2, mean1, inv1, mean2, inv2, g1f, be1f, g2f, be2f, w2_16 = ctx.saved_tensors
        w1, b1, g1, be1, w2, b2, g2, be2 = ctx.params
        dev = x.device
        f32 = dict(device=dev, dtype=torch.float32)
        dout = dout.to(torch.bfloat16).contiguous()
        N, T2, F2, _ = y2.shape
        T1 = y1.shape[1]
        grid = max(1, min(N * T2, ctx.ncu))
        nb2 = max(1, min(N * T2, 1024))
        part = torch.empty(max(2 * ctx.ncu, nb2) * 64, **f32)
        with TR.phase(TR.bn(2, True)):
            (dg2, ipg2), (db2, ipb2) = _grad_buffer(g2), _grad_buffer(be2)
            dy2 = torch.empty_like(y2)
            C_.bn_cl_bwd(dout, y2, mean2, inv2, g2f, be2f, part, nb2, dg2, db2, dy2, True)
        side = _conv_side_stream(dev, w2)
        main = torch.cuda.current_stream(dev) if side is not None else None
        with TR.phase(TR.conv(2, True)):
            wpart = torch.empty(int(C_.conv2_wgrad_part_floats(grid)), **f32)
            dw2, ip2 = _grad_buffer(w2)
            # in line (no side stream): conv2's weight gradient goes AFTER the dgrad -> BN1 ->
            # conv1-wgrad chain, which then shares the tail with the grouped weight-gradient
            # launch instead of running alone after it (7.298-7.314 vs 7.308-7.333 ms/step,
            # scripts/r6_wlast.sh)
            if side is not None:
                # dy2, z1 and wpart are freed on the main stream only after it has joined
                # the side stream below, so no allocator block is reused under the kernel
                from .rnn import _stream_wait
                _stream_wait(side, main)
                with torch.cuda.stream(side):
                    C_.conv2_wgrad(dy2, z1, wpart, dw2, grid)
            dz1 = torch.empty_like(y1)
            # two workgroups per CU; the epilogue also leaves conv1's BN-backward sums in part
            dgrid = max(1, min(N * ((T1 + 1) // 2), 2 * ctx.ncu))
            C_.conv2_dgrad(dy2, w2_16, dz1, dgrid, y1, mean1, inv1, g1f, be1f, part)
            # conv2.weight is reported below, after its GEMM and after the dgrad: a bucket whose
            # last reporter it is may launch its all-reduce + optimizer range (which rewrites the
            # bf16 shadow w2_16) at that call, so every reader of w2_16 must be on the stream
        gg2, gb2, gbias2 = _deliver(g2, dg2, ipg2), _deliver(be2, db2, ipb2), _zero_grad_of(b2)
        with TR.phase(TR.bn(1, True)):
            (dg1, ipg1), (db1, ipb1) = _grad_buffer(g1), _grad_buffer(be1)
            # the sums came out of the dgrad epilogue; the apply pass runs inside conv1_wgrad's
            # staging (dy1 never materialised), so only dgamma / dbeta here
            C_.bn_cl_bwd(dz1, y1, mean1, inv1, g1f, be1f, part, dgrid, dg1, db1, dz1, False, part_ready=2)
        with TR.phase(TR.conv(1, True)):
            g1grid = max(1, min(N * ((T1 + 3) // 4), _C1W_BPC * ctx.ncu))
            wpart1 = torch.empty(int(C_.conv1_wgrad_part_floats(g1grid)), **f32)
            dw1, ip1 = _grad_buffer(w1)
            C_.conv1_wgrad(dz1, x, wpart1, dw1, g1grid, y1, mean1, inv1, g1f, be1f, db1, dg1)
            if side is not None:
                # conv2's weight gradient joins here and is reported from the main stream
                _stream_wait(main, side)
                gw2 = _deliver(w2, dw2, ip2)
            else:
                C_.conv2_wgrad(dy2, z1, wpart, dw2, grid)
                gw2 = _deliver(w2, dw2, ip2)
            gw1 = _deliver(w1, dw1, ip1)
        gg1, gb1, gbias1 = _deliver(g1, dg1, ipg1), _deliver(be1, db1, ipb1), _zero_grad_of(b1)
        return None, gw1, gbias1, gg1, gb1, gw2, gbias2, gg2, gb2, None


def cl_supported(model, feats: torch.Tensor) -> bool:
    """The channels-last MFMA front-end covers the reference geometry (32 filters and
    F1 = (F0-5)/2+1 <= 80 frequency positions, i.e. up to 163 bins); other widths take the
    library-conv path below."""
    if model.num_filters != 32 or feats.dim() != 3:
        return False
    F1 = (feats.shape[2] - 5) // 2 + 1
    return 9 <= F1 <= 80 and feats.shape[1] >= 38


def frontend_hip(model, feats: torch.Tensor) -> torch.Tensor:
    if cl_supported(model, feats) and os.environ.get("DS2_CONV", "hip") == "hip":
        c1, c2 = model.conv1, model.conv2
        return FrontendCL.apply(feats, c1.weight, c1.bias, c1.bn_gamma, c1.bn_beta,
                                c2.weight, c2.bias, c2.bn_gamma, c2.bn_beta, model)
    x = feats.unsqueeze(1)
    x = conv_block_hip(model.conv1, x, 0, 1)
    if getattr(model, "capture", False):
        model.act_taps["conv1"] = x.detach()
    x = conv_block_hip(model.conv2, x, 1, 2)
    if getattr(model, "capture", False):
        model.act_taps["conv2"] = x.detach()
    return x


class FusedHead(torch.autograd.Function):
    """Time-major logits = h W_fc^T + b_fc (bf16), weight gradients straight to the arena."""

    @staticmethod
    def forward(ctx, h, weight, bias):
        T, N, H = h.shape
        if arena_of(weight) is not None:
            arena_of(weight).await_params(weight, bias)      # a carried optimizer update (Trainer)
        w16 = weight.bf16 if arena_of(weight) is not None else weight.to(torch.bfloat16)
        b16 = bias.bf16 if arena_of(bias) is not None else bias.to(torch.bfloat16)
        h2 = h.to(torch.bfloat16).reshape(T * N, H).contiguous()
        K = w16.shape[0]
        if K <= 32 and H % 32 == 0:
            # csrc/ctc.hip fc_lsm_kernel: MFMA FC, W_fc staged in LDS, logits in bf16
            out = torch.empty(T, N, K, device=h.device, dtype=torch.bfloat16)
            _ext.ext().fc_logits(h2, w16.contiguous(), b16.contiguous(), out)
        else:
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
        # arena-managed weights: dW and the bias sum run on the weight-gradient side stream,
        # so the top recurrent layer's BPTT starts right after dh (they were ~75 us on the
        # critical path); the Trainer joins that stream before Adam
        from .rnn import _stream_wait, wgrad_stream
        side = (wgrad_stream(d2.device, arena_of(weight)) if (arena_of(bias) is not None and _HEAD_SIDE)
                else None)
        if side is None:
            gw, gb = FusedHead._weight_grads(weight, bias, d2, h2)
            return dh, gw, gb
        _stream_wait(side, torch.cuda.current_stream(d2.device))
        arena_of(weight).wgrad.hold(d2, h2)
        with torch.cuda.stream(side):
            gw, gb = FusedHead._weight_grads(weight, bias, d2, h2)
        return dh, gw, gb

    @staticmethod
    def _weight_grads(weight, bias, d2, h2):
        from .optim import mm_into
        gw = mm_into(weight, d2.t(), h2)
        if gw is None:
            arena_of(weight).grad_done(weight)
        gb = emit_grad(bias, d2.sum(0, dtype=torch.float32))
        return gw, gb
