"""DeepSpeech2 network: 2-D conv front-end -> stacked (bi)directional RNN/GRU -> FC.

Reference graph: src/deepSpeech_NCHW.py:81-201 (NCHW default) and src/deepSpeech.py:81-203.

  conv1  [20x5] stride (2,2) VALID, 1 -> C,  bias -0.05, BN(eps 1e-3), clipped ReLU(20)
  conv2  [10x5] stride (2,1) VALID, C -> C,  bias -0.05, BN(eps 1e-3), clipped ReLU(20)
  [N,C,T2,F2] -> time-major [T2, N, C*F2]        (src/deepSpeech_NCHW.py:166-168)
  L x recurrent layer (cell: rnn_relu | gru), directions summed (Q2)
  FC H -> 29 classes, time-major logits            (src/deepSpeech_NCHW.py:188-198)

Two engines share these parameters:
  * ``ref`` — pure PyTorch (CPU golden model, any device);
  * ``hip`` — gfx950 kernels: fused BN+clip(+time-major store), persistent
    bidirectional recurrence, fused CTC (see deepspeech_amd/ops).

Reference quirks handled explicitly:
  Q1 stack_fix, Q2 sum of directions, Q3 seq_bn='frozen', Q4 proper BN train/eval,
  Q7 dynamic batch sizes.
"""
from __future__ import annotations

import os
import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import FREQ_BINS, NUM_CLASSES
from ..ops import reference as R

CONV_BN_EPS = 1e-3
GATES = {"rnn_relu": 1, "gru": 3}


def tf_fans(shape) -> Tuple[int, int]:
    """Fan computation of TF's variance_scaling / glorot initialisers for a TF shape."""
    if len(shape) == 2:
        return shape[0], shape[1]
    receptive = 1
    for d in shape[:-2]:
        receptive *= d
    return shape[-2] * receptive, shape[-1] * receptive


def he_trunc_normal_(t: torch.Tensor, tf_shape) -> torch.Tensor:
    """variance_scaling_initializer(factor=2, FAN_IN, uniform=False) of TF 1.x contrib:
    truncated normal with stddev sqrt(1.3*factor/fan_in) (src/helper_routines.py:65-72)."""
    fan_in, _ = tf_fans(tf_shape)
    std = math.sqrt(1.3 * 2.0 / fan_in)
    with torch.no_grad():
        nn.init.trunc_normal_(t, mean=0.0, std=std, a=-2 * std, b=2 * std)
    return t


def glorot_uniform_(t: torch.Tensor, tf_shape) -> torch.Tensor:
    """TF's default get_variable initializer (glorot_uniform) for the RNN W/U."""
    fan_in, fan_out = tf_fans(tf_shape)
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        t.uniform_(-lim, lim)
    return t


def conv_out_len(T: int) -> Tuple[int, int]:
    t1 = (T - 20) // 2 + 1
    t2 = (t1 - 10) // 2 + 1
    return t1, t2


def freq_out(F_in: int = FREQ_BINS) -> Tuple[int, int]:
    f1 = (F_in - 5) // 2 + 1
    f2 = f1 - 5 + 1
    return f1, f2


NHWC_BN_EPS = 1e-5
NHWC_BN_DECAY = 0.5



# False: the features' cast and the rnn lengths as torch ops (A/B)
_PREP_FUSED = True

class ConvBlock(nn.Module):
    """conv + bias + BatchNorm + clipped ReLU.

    bn='fused' (NCHW graph, src/deepSpeech_NCHW.py:110-158 / custom_ops.batch_norm2):
        fused batch norm, eps 1e-3, batch statistics in training; running statistics
        (momentum 0.01) in eval (quirk Q4: the reference also used batch stats in eval).
    bn='moments_ema' (NHWC graph, src/deepSpeech.py:110-158 / custom_ops.batch_norm,
        src/custom_ops.py:163-181): tf.nn.moments over (N, T, F) per channel, eps 1e-5,
        ExponentialMovingAverage(decay 0.5, zero_debias) of the batch mean / variance,
        whose debiased values normalise in eval."""

    def __init__(self, cin: int, cout: int, kernel: Tuple[int, int], stride: Tuple[int, int], bn: str = "fused"):
        super().__init__()
        if bn not in ("fused", "moments_ema"):
            raise ValueError(bn)
        self.stride = stride
        self.bn = bn
        self.bn_eps = CONV_BN_EPS if bn == "fused" else NHWC_BN_EPS
        self.weight = nn.Parameter(torch.empty(cout, cin, *kernel))
        self.bias = nn.Parameter(torch.full((cout,), -0.05))
        self.bn_gamma = nn.Parameter(torch.ones(cout))
        self.bn_beta = nn.Parameter(torch.zeros(cout))
        self.register_buffer("running_mean", torch.zeros(cout))
        self.register_buffer("running_var", torch.ones(cout))
        # zero-debiased EMA state of the moments (TF: <shadow>/biased, <shadow>/local_step)
        self.register_buffer("ema_mean_biased", torch.zeros(cout))
        self.register_buffer("ema_var_biased", torch.zeros(cout))
        self.register_buffer("ema_steps", torch.zeros((), dtype=torch.float32))
        # TF HWIO shape for initialisation parity
        he_trunc_normal_(self.weight, [kernel[0], kernel[1], cin, cout])

    @torch.no_grad()
    def ema_update(self, mean: torch.Tensor, var: torch.Tensor) -> None:
        """biased <- decay*biased + (1-decay)*value; local_step += 1 (TF zero-debias)."""
        d = NHWC_BN_DECAY
        self.ema_mean_biased.mul_(d).add_(mean.detach().float(), alpha=1 - d)
        self.ema_var_biased.mul_(d).add_(var.detach().float(), alpha=1 - d)
        self.ema_steps.add_(1.0)

    def ema_moments(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """Debiased EMA mean / variance (eval statistics of the moments_ema variant)."""
        corr = 1.0 - NHWC_BN_DECAY ** self.ema_steps.clamp(min=1.0)
        return self.ema_mean_biased / corr, self.ema_var_biased / corr

    def forward_ref(self, x: torch.Tensor) -> torch.Tensor:
        y = F.conv2d(x, self.weight.to(x.dtype), self.bias.to(x.dtype), stride=self.stride)
        if self.bn == "fused":
            y = F.batch_norm(y, self.running_mean, self.running_var, self.bn_gamma.to(y.dtype),
                             self.bn_beta.to(y.dtype), training=self.training, momentum=0.01,
                             eps=CONV_BN_EPS)
        else:
            if self.training:
                yf = y.float()
                mean = yf.mean(dim=(0, 2, 3))
                var = ((yf - mean.view(1, -1, 1, 1)) ** 2).mean(dim=(0, 2, 3))   # tf.nn.moments (biased)
                self.ema_update(mean, var)
            else:
                mean, var = self.ema_moments()
            inv = torch.rsqrt(var + NHWC_BN_EPS)
            y = ((y - mean.view(1, -1, 1, 1).to(y.dtype)) * (inv * self.bn_gamma).view(1, -1, 1, 1).to(y.dtype)
                 + self.bn_beta.view(1, -1, 1, 1).to(y.dtype))
        return R.clipped_relu(y)


class RecurrentDirection(nn.Module):
    """Parameters of one direction of one recurrent layer.

    rnn_relu: W [H,in], U [H,H], b [H] — names follow CustomRNNCell2 (src/custom_ops.py:56-70).
    gru     : W [3H,in], U [3H,H], b [3H] (input bias, gates r,z,n), b_h [3H] (recurrent bias).
    The sequence-BN moving stats are buffers (non-trainable, like the reference's sbn vars).
    """

    def __init__(self, in_dim: int, hidden: int, cell: str):
        super().__init__()
        G = GATES[cell]
        self.cell = cell
        self.hidden = hidden
        self.W = nn.Parameter(torch.empty(G * hidden, in_dim))
        self.U = nn.Parameter(torch.empty(G * hidden, hidden))
        self.b = nn.Parameter(torch.zeros(G * hidden))
        if cell == "gru":
            self.b_h = nn.Parameter(torch.zeros(G * hidden))
        else:
            self.register_parameter("b_h", None)
        self.register_buffer("sbn_mean", torch.zeros(G * hidden))
        self.register_buffer("sbn_var", torch.ones(G * hidden))
        glorot_uniform_(self.W, [G * hidden, in_dim])
        glorot_uniform_(self.U, [G * hidden, hidden])


class RecurrentLayer(nn.Module):
    def __init__(self, in_dim: int, hidden: int, cell: str, bidirectional: bool, seq_bn: str):
        super().__init__()
        self.cell = cell
        self.hidden = hidden
        self.bidirectional = bidirectional
        self.seq_bn = seq_bn
        self.fw = RecurrentDirection(in_dim, hidden, cell)
        self.bw = RecurrentDirection(in_dim, hidden, cell) if bidirectional else None

    def directions(self) -> List[RecurrentDirection]:
        return [self.fw] + ([self.bw] if self.bw is not None else [])

    def input_projection_ref(self, x: torch.Tensor, d: RecurrentDirection, lens) -> torch.Tensor:
        y = x @ d.W.to(x.dtype).t()
        y = R.seq_batch_norm(y, lens, self.seq_bn, d.sbn_mean, d.sbn_var, self.training)
        return y + d.b.to(y.dtype)

    def forward_ref_split(self, x_f: torch.Tensor, x_b: torch.Tensor, lens: torch.Tensor):
        """Per-direction stacks (NHWC graph): the forward direction reads the forward stack's
        input, the backward direction the backward stack's; outputs are NOT summed."""
        bh = lambda d: None if d.b_h is None else d.b_h.to(x_f.dtype)
        gx_f = self.input_projection_ref(x_f, self.fw, lens)
        y_f, _ = R.recurrent_scan(self.cell, gx_f, self.fw.U.to(x_f.dtype), bh(self.fw), lens)
        gx_b = self.input_projection_ref(x_b, self.bw, lens)
        y_br, _ = R.recurrent_scan(self.cell, R.reverse_sequence(gx_b, lens), self.bw.U.to(x_b.dtype), bh(self.bw),
                                   lens)
        return y_f, R.reverse_sequence(y_br, lens)

    def forward_ref(self, x: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
        gx_f = self.input_projection_ref(x, self.fw, lens)
        gx_b = self.input_projection_ref(x, self.bw, lens) if self.bw is not None else None
        bh = lambda d: None if d is None or d.b_h is None else d.b_h.to(x.dtype)
        return R.birnn_ref(self.cell, gx_f, gx_b, self.fw.U.to(x.dtype),
                           None if self.bw is None else self.bw.U.to(x.dtype),
                           bh(self.fw), bh(self.bw), lens)


class DeepSpeech2(nn.Module):
    def __init__(self, num_filters: int = 32, num_hidden: int = 1024, num_rnn_layers: int = 2,
                 cell: str = "rnn_relu", bidirectional: bool = True, stack_fix: bool = True,
                 seq_bn: str = "frozen", num_classes: int = NUM_CLASSES,
                 freq_bins: int = FREQ_BINS, layout: str = "nchw"):
        """layout 'nchw' = src/deepSpeech_NCHW.py (default, --nchw True); 'nhwc' =
        src/deepSpeech.py (--nchw False): moments+EMA conv BN (eps 1e-5) and, when
        bidirectional, two deep per-direction stacks (bidirectional_dynamic_rnn over a
        MultiRNNCell each, src/deepSpeech.py:165-185) summed only at the top. The NHWC
        graph's channels-last flatten of conv2 (feature f*C + c) is a fixed permutation of
        the first layer's input columns; it is applied at the checkpoint boundary
        (utils/checkpoint.py), the compute layout is shared."""
        super().__init__()
        if cell not in GATES:
            raise ValueError("cell must be one of %s" % list(GATES))
        if layout not in ("nchw", "nhwc"):
            raise ValueError("layout must be nchw or nhwc")
        self.layout = layout
        if layout == "nhwc":
            stack_fix = True          # the NHWC graph's MultiRNNCell stacks correctly (no Q1)
        self.num_filters = num_filters
        self.num_hidden = num_hidden
        self.num_rnn_layers = num_rnn_layers
        self.cell = cell
        self.bidirectional = bidirectional
        self.stack_fix = stack_fix
        self.seq_bn = seq_bn
        self.num_classes = num_classes
        self.freq_bins = freq_bins
        _, f2 = freq_out(freq_bins)
        self.rnn_in = f2 * num_filters                     # 75*C = 2400 for 161 bins
        bn = "fused" if layout == "nchw" else "moments_ema"
        self.conv1 = ConvBlock(1, num_filters, (20, 5), (2, 2), bn=bn)
        self.conv2 = ConvBlock(num_filters, num_filters, (10, 5), (2, 1), bn=bn)
        layers = []
        for i in range(num_rnn_layers):
            # Q1: with stack_fix=False every layer consumes the conv output.
            in_dim = self.rnn_in if (i == 0 or not stack_fix) else num_hidden
            layers.append(RecurrentLayer(in_dim, num_hidden, cell, bidirectional, seq_bn))
        self.rnn = nn.ModuleList(layers)
        self.fc_weight = nn.Parameter(torch.empty(num_classes, num_hidden))
        self.fc_bias = nn.Parameter(torch.zeros(num_classes))
        he_trunc_normal_(self.fc_weight, [num_classes, num_hidden])
        self.engine = "ref"
        self.compute_dtype = torch.float32
        # activation summaries (reference _activation_summary at conv1 / conv2 / rnn / logits,
        # src/deepSpeech_NCHW.py:134,158,183,199): when ``capture`` is set, the next forward
        # keeps detached references to those activations in ``act_taps``
        self.capture = False
        self.act_taps: Dict[str, torch.Tensor] = {}

    # ------------------------------------------------------------------ config
    def set_engine(self, engine: str, compute_dtype: torch.dtype = torch.float32, fp8: bool = False) -> "DeepSpeech2":
        """engine: 'ref' (pure torch) | 'hip' (gfx950 kernels). fp8=True (HIP engine only,
        BASELINE config 5's fp8 mode): the recurrent layers' input projections run as MX-fp8
        e4m3 GEMMs, and where csrc/rnn_fp8.hip covers the GRU geometry (ops/rnn.py
        fp8_recurrence_ok / fp8_bptt_ok: H % 256 == 0, <= 8 rows per group) the forward
        recurrence multiplies an e4m3 U and exchanges e4m3 hidden states, and the BPTT runs on
        an e4m3 U^T with per-(row, 32-unit) E8M0-scaled gate gradients. Weight gradients, the
        conv front-end, the head and the master weights stay bf16 / fp32."""
        if engine not in ("ref", "hip"):
            raise ValueError(engine)
        if fp8 and engine != "hip":
            raise ValueError("fp8 projections need the HIP engine")
        self.engine = engine
        self.compute_dtype = compute_dtype
        self.fp8 = fp8
        if engine == "hip":
            from ..ops.gemm_tuning import enable_tuned_gemms
            # measured hipBLASLt picks for the library GEMMs that remain reachable: DS2_GEMM=torch
            # A/B runs and shapes the hand-written kernels do not cover (every default-path GEMM
            # of the training step runs on csrc/gemm8.hip / gemm.hip)
            enable_tuned_gemms()
        for layer in self.rnn:
            layer.fp8 = fp8
        return self

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def flops_breakdown(self, N: int, T: int) -> Dict[str, float]:
        """Analytic forward FLOPs per layer for a [N, T] batch (the reference's tfprof
        flops.log, src/deepSpeech_train.py:368-372)."""
        t1, t2 = conv_out_len(T)
        f1, f2 = freq_out(self.freq_bins)
        C, H, G = self.num_filters, self.num_hidden, GATES[self.cell]
        dirs = 2 if self.bidirectional else 1
        out = {"conv1": 2.0 * N * t1 * f1 * C * 100, "conv2": 2.0 * N * t2 * f2 * C * C * 50}
        for i, layer in enumerate(self.rnn):
            in_dim = layer.fw.W.shape[1]
            out["rnn_cell_%d" % i] = dirs * 2.0 * N * t2 * G * H * (in_dim + H)
        out["softmax_linear"] = 2.0 * N * t2 * H * self.num_classes
        return out

    def flops_per_step(self, N: int, T: int) -> float:
        """Analytic training FLOPs (fwd + 2x bwd) for a [N, T] batch."""
        return 3.0 * sum(self.flops_breakdown(N, T).values())

    # ------------------------------------------------------------------ forward
    def frontend(self, feats: torch.Tensor) -> torch.Tensor:
        """feats [N, T, F] -> time-major rnn input [T2, N, C*F2]."""
        if self.engine == "hip":
            from ..ops import frontend as FE
            return FE.frontend_hip(self, feats)
        from ..utils import trace as TR
        x = feats.unsqueeze(1)
        with TR.phase(TR.conv(1)):
            x = self.conv1.forward_ref(x)
        self._tap("conv1", x)
        with TR.phase(TR.conv(2)):
            x = self.conv2.forward_ref(x)
        self._tap("conv2", x)
        N, C, T2, F2 = x.shape
        return x.permute(2, 0, 1, 3).reshape(T2, N, C * F2)

    def _tap(self, name: str, t: torch.Tensor) -> None:
        if self.capture:
            self.act_taps[name] = t.detach()

    def direction_stacks(self) -> bool:
        return self.layout == "nhwc" and self.bidirectional

    def recurrent(self, x: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
        if self.direction_stacks():
            x_f = x_b = x
            for i, layer in enumerate(self.rnn):
                if self.engine == "hip":
                    from ..ops import rnn as RNN
                    x_f, x_b = RNN.recurrent_layer_split_hip(layer, x_f, x_b, lens, i)
                else:
                    from ..utils import trace as TR
                    with TR.phase(TR.rnn_cell(i)):
                        x_f, x_b = layer.forward_ref_split(x_f, x_b, lens)
            out = x_f + x_b
            self._tap("rnn", out)
            return out
        inp = x
        out = x
        for i, layer in enumerate(self.rnn):
            if self.engine == "hip":
                from ..ops import rnn as RNN
                # an fp8 layer feeding an fp8 layer hands over its two direction outputs and
                # the upper layer's quantiser sums them (no direction-sum launch)
                pair = self.stack_fix and i + 1 < len(self.rnn) and RNN.pairs_ok(self.rnn[i + 1])
                out = RNN.recurrent_layer_hip(layer, inp, lens, i, pair_out=pair)
            else:
                from ..utils import trace as TR
                with TR.phase(TR.rnn_cell(i)):
                    out = layer.forward_ref(inp, lens)
            inp = out if self.stack_fix else x
        self._tap("rnn", out)
        return out

    def arena_groups(self):
        """Parameter layout for ops.optim.ParamArena: gradient-production order (FC first,
        conv1 last) and, per recurrent layer, [W_fw; W_bw] and [b_fw; b_bw] packed back to
        back so the fused layer reads/writes both directions as one matrix."""
        groups = [[("fc_bias", self.fc_bias)], [("fc_weight", self.fc_weight)]]
        for i in reversed(range(len(self.rnn))):
            layer = self.rnn[i]
            pre = "rnn.%d." % i
            dirs = [("fw", layer.fw)] + ([("bw", layer.bw)] if layer.bw is not None else [])
            groups.append([(pre + n + ".W", d.W) for n, d in dirs])
            groups.append([(pre + n + ".b", d.b) for n, d in dirs])
            groups.append([(pre + n + ".U", d.U) for n, d in dirs])
            if layer.fw.b_h is not None:
                groups.append([(pre + n + ".b_h", d.b_h) for n, d in dirs])
        for cname in ("conv2", "conv1"):
            blk = getattr(self, cname)
            for pn in ("bn_beta", "bn_gamma", "bias", "weight"):
                groups.append([("%s.%s" % (cname, pn), getattr(blk, pn))])
        return groups

    def head(self, h: torch.Tensor) -> torch.Tensor:
        if self.engine == "hip":
            from ..ops.frontend import FusedHead
            from ..utils import trace as TR
            with TR.phase(TR.SOFTMAX_F):
                return FusedHead.apply(h, self.fc_weight, self.fc_bias)
        T, N, H = h.shape
        w = self.fc_weight.to(h.dtype)
        b = self.fc_bias.to(h.dtype)
        return torch.addmm(b, h.reshape(T * N, H), w.t()).view(T, N, -1)

    def _hip_inputs(self, feats: torch.Tensor, seq_lens: torch.Tensor):
        """(features in the compute dtype, rnn lengths int32) of the HIP engine: one fused launch
        (csrc/fill.hip prep_inputs_kernel) for fp32 device features, else the torch ops."""
        seq_lens = seq_lens.to(feats.device)
        if (_PREP_FUSED and feats.is_cuda and feats.dtype == torch.float32 and self.compute_dtype == torch.bfloat16 and
                feats.is_contiguous() and feats.data_ptr() % 16 == 0 and seq_lens.dtype == torch.int32 and
                seq_lens.is_contiguous()):
            from ..ops import _ext
            x = torch.empty(feats.shape, device=feats.device, dtype=torch.bfloat16)
            lens = torch.empty_like(seq_lens)
            _ext.ext().prep_inputs(feats, x, seq_lens, lens)
            return x, lens
        return feats.to(self.compute_dtype), R.get_rnn_seqlen(seq_lens)

    def forward(self, feats: torch.Tensor, seq_lens: torch.Tensor
                ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Returns (logits [T2, N, K] time-major, rnn lengths [N] int32)."""
        if self.engine == "hip":
            feats, lens = self._hip_inputs(feats, seq_lens)
        else:
            lens = R.get_rnn_seqlen(seq_lens.to(feats.device))
        if self.engine == "ref" and feats.device.type == "cuda" and self.compute_dtype != torch.float32:
            with torch.autocast("cuda", dtype=self.compute_dtype):
                x = self.frontend(feats)
                h = self.recurrent(x, lens)
                logits = self.head(h)
            return logits.float(), lens
        x = self.frontend(feats)
        h = self.recurrent(x, lens.to(x.device))
        logits = self.head(h)
        self._tap("softmax_linear", logits)
        return logits, lens

    def forward_loss(self, feats: torch.Tensor, seq_lens: torch.Tensor, targets: torch.Tensor,
                     target_lens: torch.Tensor) -> torch.Tensor:
        """Training forward: mean CTC loss of a batch. On the HIP engine the FC head and the
        CTC loss are one fused op (ops/ctc.py FusedHeadCTC: the logits never reach memory);
        otherwise forward() + loss()."""
        if self.engine == "hip" and self.num_classes <= 32 and self.num_hidden % 32 == 0:
            from ..ops import ctc as CTC
            xin, lens = self._hip_inputs(feats, seq_lens)
            x = self.frontend(xin)
            h = self.recurrent(x, lens.to(x.device))
            from ..ops import rnn as RNN
            RNN.flush_transposes()      # the dx GEMMs' W^T shadows, beside the head + CTC
            if self.capture:
                with torch.no_grad():   # the fused head never materialises the logits
                    self._tap("softmax_linear", self.head(h.detach()))
            return CTC.head_ctc_mean_loss_hip(h, self.fc_weight, self.fc_bias, lens, targets, target_lens)
        logits, lens = self(feats, seq_lens)
        return self.loss(logits, lens, targets, target_lens)

    # ------------------------------------------------------------------ loss
    def loss(self, logits: torch.Tensor, lens: torch.Tensor, targets: torch.Tensor,
             target_lens: torch.Tensor) -> torch.Tensor:
        """Mean CTC loss over the batch (src/deepSpeech_NCHW.py:204-228)."""
        if self.engine == "hip":
            from ..ops import ctc as CTC
            return CTC.ctc_mean_loss_hip(logits, lens, targets, target_lens)
        from ..utils import trace as TR
        with TR.phase(TR.CTC_F):
            return R.ctc_loss_ref(logits, targets, lens, target_lens).mean()


def build_model(**kw) -> DeepSpeech2:
    return DeepSpeech2(**kw)
