"""Autograd wrapper around the persistent bidirectional recurrence kernels.

Forward of one recurrent layer on the HIP engine (reference: src/custom_ops.py:36-96):

    gx = x . [W_fw; W_bw]^T * s + [b_fw; b_bw]      one hipBLASLt GEMM, both directions
    y_fw, y_bw = persistent_recurrence(gx, U, b_h)   csrc/rnn_persistent.hip
    y = y_fw + y_bw                                   directions summed (quirk Q2)

Backward:

    dgx, dgh = persistent_bptt(dy, saved gates / states)   csrc/rnn_persistent.hip
    dU_d = dgh_d^T . h_prev_d     (one GEMM per direction, all steps at once)
    dW   = dgx^T . x,  dx = dgx . W_cat                (autograd of the projection GEMM)

The projection (and its sequence-BN) stays in torch autograd: it is a plain library
GEMM. Only the serial recurrence is a custom autograd.Function.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import List, Optional

import torch

from . import _ext
from . import reference as R

CELL_CODE = {"rnn_relu": 0, "gru": 1}
GATES = {"rnn_relu": 1, "gru": 3}
TIMEOUT_TICKS = int(float(os.environ.get("DS2_RNN_TIMEOUT_S", "20")) * 1e8)   # s_memrealtime = 100 MHz
_pending_errors: List[torch.Tensor] = []
# diagnostic: when set to a list, each kernel launch appends (kind, plan, stamps[grid, 8])
# recorded by the s_memtime build (csrc/rnn_persistent_stamps.hip)
STAMP_LOG: Optional[list] = None


@dataclass(frozen=True)
class RnnPlan:
    N: int
    NP: int
    BG: int
    mt: int
    nw: int
    persistent: bool
    H: int
    S: int
    cell: str
    ndir: int


# Largest KPW (k-steps per wave) that compiles WITHOUT register spills, per
# (cell, direction, waves per workgroup, row tiles) — from hipcc -Rpass-analysis on gfx950.
_MAX_KPW = {
    ("gru", "fwd", 4, 1): 24, ("gru", "fwd", 4, 2): 16, ("gru", "fwd", 8, 1): 8, ("gru", "fwd", 8, 2): 8,
    ("rnn_relu", "fwd", 4, 1): 32, ("rnn_relu", "fwd", 4, 2): 32,
    ("rnn_relu", "fwd", 8, 1): 16, ("rnn_relu", "fwd", 8, 2): 16,
    ("gru", "bwd", 4, 1): 32, ("gru", "bwd", 4, 2): 32, ("gru", "bwd", 8, 1): 16, ("gru", "bwd", 8, 2): 12,
    ("rnn_relu", "bwd", 4, 1): 32, ("rnn_relu", "bwd", 4, 2): 32,
    ("rnn_relu", "bwd", 8, 1): 24, ("rnn_relu", "bwd", 8, 2): 12,
}


def _kpw(H: int, G: int, nw: int, fwd: bool) -> int:
    ks = (H // 32) if fwd else (G * H // 32)
    need = -(-ks // nw)
    for k in (4, 8, 12, 16, 24, 32):
        if k >= need:
            return k
    return -1


def _fits(cell: str, H: int, nw: int, mt: int) -> bool:
    G = GATES[cell]
    kf, kb = _kpw(H, G, nw, True), _kpw(H, G, nw, False)
    return (0 < kf <= _MAX_KPW[(cell, "fwd", nw, mt)]) and (0 < kb <= _MAX_KPW[(cell, "bwd", nw, mt)])


def make_plan(N: int, H: int, cell: str, ndir: int, cus: int, mode: Optional[str] = None) -> RnnPlan:
    """Choose tile geometry: rows per workgroup (16*mt), waves per workgroup (nw), and
    whether the persistent (all workgroups co-resident) schedule fits the chip."""
    if H % 32 != 0:
        raise ValueError("HIP recurrence requires num_hidden % 32 == 0 (got %d)" % H)
    G = GATES[cell]
    S = H // 16
    mode = mode or os.environ.get("DS2_RNN_MODE", "auto")
    force_nw = int(os.environ.get("DS2_RNN_NW", "0"))
    chosen = None
    for mt in (1, 2):
        BG = -(-N // (16 * mt))
        if ndir * BG * S <= cus:
            chosen = (mt, BG, True)
            break
    if chosen is None:
        mt = 2
        chosen = (mt, -(-N // 32), False)
    mt, BG, persistent = chosen
    if mode == "step":
        persistent = False
    nw_opts = [force_nw] if force_nw else [8, 4]
    nw = None
    for cand in nw_opts:
        if _fits(cell, H, cand, mt):
            nw = cand
            break
    if nw is None:
        # no spill-free instantiation: take the 4-wave one (correct, some register spills)
        if _kpw(H, G, 4, True) < 0 or _kpw(H, G, 4, False) < 0:
            raise ValueError("no tile for H=%d cell=%s" % (H, cell))
        nw = 4
    return RnnPlan(N=N, NP=BG * 16 * mt, BG=BG, mt=mt, nw=nw, persistent=persistent, H=H, S=S,
                   cell=cell, ndir=ndir)


def check_errors(clear: bool = True) -> None:
    """Raise if any recurrence kernel since the last check hit its spin timeout.
    Call at a point where the host synchronises anyway (e.g. when logging the loss)."""
    global _pending_errors
    errs = _pending_errors
    if clear:
        _pending_errors = []
    for e in errs:
        if int(e.item()) != 0:
            raise RuntimeError("persistent recurrence kernel timed out waiting for its peers "
                               "(grid not co-resident?) — rerun with DS2_RNN_MODE=step")


def _stamps(kind: str, plan: "RnnPlan", grid: int, dev) -> Optional[torch.Tensor]:
    if STAMP_LOG is None:
        return None
    t = torch.zeros(grid, 8, device=dev, dtype=torch.int64)
    STAMP_LOG.append((kind, plan, t))
    return t


def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    try:
        return torch.mm(a, b, out_dtype=torch.float32)
    except (RuntimeError, TypeError):
        return torch.mm(a, b).float()


class BiRecurrence(torch.autograd.Function):
    """y = sum_d recurrence_d(gx[..., d]) over a [T, N, ndir*G*H] bf16 projection."""

    @staticmethod
    def forward(ctx, gx, lens, U_f, U_b, bh_f, bh_b, plan: RnnPlan):
        C = _ext.ext()
        T, N, gstride = gx.shape
        H, ndir, G = plan.H, plan.ndir, GATES[plan.cell]
        steps = T
        dev = gx.device
        gx = gx.contiguous()
        lens = lens.to(device=dev, dtype=torch.int32).contiguous()
        U_f = U_f.contiguous()
        U_b = U_b.contiguous() if U_b is not None else None
        bf16 = torch.bfloat16
        y2 = torch.empty(ndir, T, N, H, device=dev, dtype=bf16)
        hx = torch.empty(ndir, steps + 1, plan.NP, H, device=dev, dtype=bf16)
        hx[:, 0].zero_()                         # h0
        hs = torch.empty(ndir, steps + 1, plan.NP, H, device=dev, dtype=torch.float32)
        hs[:, 0].zero_()
        gates = (torch.empty(ndir, steps, plan.NP, H, 4, device=dev, dtype=torch.float32)
                 if plan.cell == "gru" else None)
        flags = torch.zeros(ndir * plan.BG * plan.S, device=dev, dtype=torch.int32)
        err = torch.zeros(1, device=dev, dtype=torch.int32)
        d1 = ndir == 2
        C.rnn_fwd(gx, lens, U_f, U_b if d1 else None,
                  bh_f.contiguous().float() if bh_f is not None else None,
                  bh_b.contiguous().float() if (bh_b is not None and d1) else None,
                  y2[0], y2[1] if d1 else None, hx[0], hx[1] if d1 else None,
                  hs[0], hs[1] if d1 else None,
                  gates[0] if gates is not None else None,
                  gates[1] if (gates is not None and d1) else None,
                  flags, err, T, N, plan.NP, H, plan.BG, steps, gstride, ndir,
                  CELL_CODE[plan.cell], plan.nw, plan.mt, plan.persistent, TIMEOUT_TICKS,
                  _stamps("fwd", plan, flags.numel(), dev))
        _pending_errors.append(err)
        y = y2[0] + y2[1] if d1 else y2[0]
        ctx.save_for_backward(lens, U_f, U_b if U_b is not None else torch.empty(0, device=dev),
                              hx, hs, gates if gates is not None else torch.empty(0, device=dev))
        ctx.plan = plan
        ctx.shape = (T, N, gstride, steps)
        ctx.has_bh = (bh_f is not None, bh_b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _ext.ext()
        lens, U_f, U_b, hx, hs, gates = ctx.saved_tensors
        plan: RnnPlan = ctx.plan
        T, N, gstride, steps = ctx.shape
        H, ndir, G = plan.H, plan.ndir, GATES[plan.cell]
        dev = dy.device
        d1 = ndir == 2
        dy = dy.to(torch.bfloat16).contiguous()
        dgh = torch.empty(ndir, steps, plan.NP, G * H, device=dev, dtype=torch.bfloat16)
        dgx = torch.empty(T, N, gstride, device=dev, dtype=torch.bfloat16)
        carry = None if plan.persistent else torch.zeros(ndir, plan.NP, H, device=dev, dtype=torch.float32)
        flags = torch.zeros(ndir * plan.BG * plan.S, device=dev, dtype=torch.int32)
        err = torch.zeros(1, device=dev, dtype=torch.int32)
        has_g = gates.numel() > 0
        C.rnn_bwd(dy, lens, U_f, U_b if d1 else None, hs[0], hs[1] if d1 else None,
                  gates[0] if has_g else None, gates[1] if (has_g and d1) else None,
                  dgh[0], dgh[1] if d1 else None, dgx,
                  carry[0] if carry is not None else None,
                  carry[1] if (carry is not None and d1) else None,
                  flags, err, T, N, plan.NP, H, plan.BG, steps, gstride, ndir,
                  CELL_CODE[plan.cell], plan.nw, plan.mt, plan.persistent, TIMEOUT_TICKS,
                  _stamps("bwd", plan, flags.numel(), dev))
        _pending_errors.append(err)
        grads_U, grads_b = [], []
        for d in range(ndir):
            g2 = dgh[d].view(steps * plan.NP, G * H)
            h2 = hx[d, :steps].reshape(steps * plan.NP, H)
            grads_U.append(_mm_f32(g2.t(), h2))
            grads_b.append(g2.sum(0, dtype=torch.float32) if ctx.has_bh[d] else None)
        dU_f = grads_U[0].to(U_f.dtype)
        dU_b = grads_U[1].to(U_f.dtype) if d1 else None
        return (dgx, None, dU_f, dU_b, grads_b[0], grads_b[1] if d1 else None, None)


_plan_cache = {}


def plan_for(N: int, H: int, cell: str, ndir: int, device: torch.device) -> RnnPlan:
    key = (N, H, cell, ndir, device.index, os.environ.get("DS2_RNN_MODE"), os.environ.get("DS2_RNN_NW"))
    p = _plan_cache.get(key)
    if p is None:
        p = make_plan(N, H, cell, ndir, _ext.num_cus(device.index or 0))
        _plan_cache[key] = p
    return p


def sbn_scale() -> float:
    return 1.0 / math.sqrt(1.0 + R.SBN_EPS)


def input_projection_hip(layer, x: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
    """gx[T, N, ndir*G*H] (bf16) = seq_bn(x W^T) + b for all directions in one GEMM."""
    T, N, D = x.shape
    dirs = layer.directions()
    W = torch.cat([d.W for d in dirs], 0).to(torch.bfloat16)
    b = torch.cat([d.b for d in dirs], 0).to(torch.bfloat16)
    x2 = x.reshape(T * N, D)
    if layer.seq_bn == "frozen":
        # moving stats are constant (mean 0, var 1): SBN is a scalar scale folded into the GEMM
        gx = torch.addmm(b, x2, W.t(), alpha=sbn_scale())
    elif layer.seq_bn == "none":
        gx = torch.addmm(b, x2, W.t())
    else:
        y = (x2 @ W.t()).view(T, N, -1)
        outs = []
        GH = dirs[0].W.shape[0]
        for i, d in enumerate(dirs):
            outs.append(R.seq_batch_norm(y[..., i * GH:(i + 1) * GH], lens, "batch", d.sbn_mean,
                                         d.sbn_var, layer.training))
        gx = (torch.cat(outs, -1) + b).reshape(T * N, -1)
    return gx.view(T, N, -1)


def recurrent_layer_hip(layer, x: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
    x = x.to(torch.bfloat16)
    ndir = 2 if layer.bw is not None else 1
    plan = plan_for(x.shape[1], layer.hidden, layer.cell, ndir, x.device)
    gx = input_projection_hip(layer, x, lens)
    U_f = layer.fw.U.to(torch.bfloat16)
    U_b = layer.bw.U.to(torch.bfloat16) if ndir == 2 else None
    bh_f = layer.fw.b_h if layer.cell == "gru" else None
    bh_b = layer.bw.b_h if (layer.cell == "gru" and ndir == 2) else None
    return BiRecurrence.apply(gx, lens, U_f, U_b, bh_f, bh_b, plan)
