"""Autograd wrapper around the persistent bidirectional recurrence kernels.

Forward of one recurrent layer on the HIP engine (reference: src/custom_ops.py:36-96):

    gx = x . [W_fw; W_bw]^T * s + [b_fw; b_bw]      ONE hand-written GEMM for both directions
                                                     (csrc/gemm8.hip, or gemm.hip where TUNED;
                                                     fp8 e4m3 operands with --fp8)
    y  = recurrence_fw(gx) + recurrence_bw(gx)       ONE persistent launch, direction sum fused
                                                     (csrc/rnn_xcd.hip; rnn_persistent.hip for
                                                     the widths the XCD kernels do not cover)

Backward (FusedBiLayer):

    dgx, dgh, bias partials = persistent BPTT         csrc/rnn_xcd.hip (reduce-scatter exchange)
    dx  = dgx . [W_fw; W_bw]                           gemm on the K-contiguous W^T shadow that the
                                                       forward transposed on a side stream
    dW  = dgx^T . x,  dU_d = dgh_d^T . h_prev_d        column-mode gemm8 into the fp32 arena; on one
                                                       GPU every layer's dW / dU is deferred and run as
                                                       ONE grouped launch after the bottom layer's BPTT
                                                       (WgradScheduler), beside the conv front-end

The sequence-BN scale of the projection is folded into its alpha; everything runs without
torch autograd inside the layer.
"""
from __future__ import annotations

import math
import os
import weakref
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch

from . import _ext
from . import gemm as GM
from . import reference as R
from .optim import arena_of, emit_grad, mm_into
from ..utils import trace as TR

CELL_CODE = {"rnn_relu": 0, "gru": 1}
GATES = {"rnn_relu": 1, "gru": 3}
TIMEOUT_TICKS = int(float(os.environ.get("DS2_RNN_TIMEOUT_S", "20")) * 1e8)   # s_memrealtime = 100 MHz
# One persistent error word per device: every recurrence launch ORs its spin-timeout bits
# into it (atomicOr in the kernels), check_errors() reads and clears it at a point where the
# host synchronises anyway. Nothing accumulates per launch.
_err_words = {}
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
    kind: str = "v1"      # "xcd": csrc/rnn_xcd.hip (gen 2); "v1": csrc/rnn_persistent.hip
    R: int = 0            # xcd: batch rows per group
    xcd_map: int = 0      # xcd: group = blockIdx % 8 (<= 8 groups of <= CUs/8 workgroups)


RNNX_KNOBS = int(os.environ.get("DS2_RNNX_KNOBS", "0"))   # diagnostic timing switches only
# knob bits that skip work (no output stores, no waits, no MFMAs, no publishes: wrong results):
# they reach a kernel only in an explicit timing session (DS2_TIMING_ONLY=1); otherwise a
# training run refuses them (check_knobs) and every launch masks them off (_kernel_knobs). The
# kernels keep their runtime tests: compiling the branches out changed hipcc's schedule of the
# config-5 BPTT (rnnrs_bwd_kernel<1, 12, 6, *>: 70-112 spilled VGPRs folded, +15 % kernel time
# with an opaque zero; round 5, profiles/r5_negative_results.md), so the guard is host-side.
TIMING_ONLY_KNOBS = 2 | 4 | 8 | 32


def _timing_only() -> bool:
    return os.environ.get("DS2_TIMING_ONLY") == "1"


# Poll timing of the persistent recurrences (csrc/rnn_xcd.hip): bits 17-19 = s_sleep units a
# forward wave waits after publishing its h before polling the next step, bits 20-22 the same
# before a BPTT gather. The forward's poll exits drain vmcnt (drain_vm), so its first poll is no
# longer held behind its own store's write acknowledgement; polling right away then measured
# slower (stale reads contend with the producers' stores in the XCD's L2), 4 units faster than
# both (scripts/r6_presleep*.sh, profiles/r6_recurrence_poll.md); BPTT 4 units: 7.301-7.309 vs
# 7.359-7.369 ms/step at 2 (scripts/r6_ab4.sh). Bit 23: take bits 17-22 as given (an explicit
# 0) instead of these defaults.
POLL_DEFAULT = (4 << 17) | (4 << 20)
POLL_EXPLICIT = 1 << 23
POLL_MASK = 0x7f << 17


# GRU layers wider than 1024 (config 5 bf16: rnnq_fwd_kernel, whose groups straddle XCDs and
# exchange write-through) poll later: the forward field counts s_sleep 4 units there (config 5
# bf16 20.74-20.81 vs 21.49-21.51 ms/step, scripts/r6_c5poll3.sh), and bit 29 makes the BPTT's
# field count 4 units too: 3 x 4 = 12, 20.84-20.85 vs 21.03-21.04 (20: 20.89-20.90, 28:
# 20.99-21.06; scripts/r6_c5bwd.sh)
POLL_WIDE = (5 << 17) | (3 << 20) | (1 << 29)


# clipped-ReLU stacks (the reference's 7 x bi-RNN-1760: rnnw kernels, 64-unit workgroups):
# forward sleep 2, 13.561-13.575 vs 13.603-13.659 ms/step at 4 (scripts/r6_relu2.sh)
POLL_RELU = (2 << 17) | (4 << 20)


def poll_default(plan=None) -> int:
    if plan is not None and plan.cell == "gru" and plan.H > 1024:
        return POLL_WIDE
    if plan is not None and plan.cell != "gru":
        return POLL_RELU
    return POLL_DEFAULT


def _kernel_knobs(plan=None) -> int:
    """DS2_RNNX_KNOBS as the kernels of ``plan`` receive it: timing-only bits dropped outside a
    timing session, the plan's default poll timing unless set explicitly."""
    k = RNNX_KNOBS if _timing_only() else RNNX_KNOBS & ~TIMING_ONLY_KNOBS
    if not (k & POLL_MASK):
        k |= poll_default(plan)
    return k


def check_knobs() -> None:
    """Refuse DS2_RNNX_KNOBS bits that skip work unless DS2_TIMING_ONLY=1 (they would silently
    time — and train — a different computation than the caller believes)."""
    bad = RNNX_KNOBS & TIMING_ONLY_KNOBS
    if bad and not _timing_only():
        raise RuntimeError("DS2_RNNX_KNOBS bits 0x%x skip work (timing only, wrong results); set DS2_TIMING_ONLY=1 "
                           "for a timing session (tools/bench_rnn.py --knobs)" % bad)
_FUSE_DIRSUM = True        # module switch: tests compare the fused direction sum with torch.add
# split-K of a dU GEMM issued beside the next layer's BPTT (data-parallel runs, where the
# weight gradients are not deferred): measured 2 (1: 9.21-9.29, 3: 9.09-9.15, 2: 8.98-9.03 ms/step)
_DU_SPLITS = 2


LDS_BYTES = 160 * 1024


def _xcd_kb(H: int, G: int, fwd: bool) -> int:
    """k-steps per MFMA wave of csrc/rnn_xcd.hip (K split over the 7 worker waves; the
    8th is the memory wave). -1 if the tile would not fit."""
    need = -(-((H if fwd else G * H) // 32) // 7)
    opts = (1, 2, 3, 4, 5, 6) if fwd else (2, 4, 6, 8, 11)
    for k in opts:
        if k >= need:
            return k
    return -1


def _rs_ok(H: int) -> bool:
    """The reduce-scatter BPTT (generation 3) serves P = H/32 <= 42 workgroups per group.
    Groups wider than one XCD (P > 32) exchange write-through across XCDs; measured on
    MI355X that still beats the generation-1 kernels for the 3-gate GRU (H=1280: fwd 1.52 vs
    1.93, BPTT 2.05 vs 3.68 ms per layer) but not for the one-gate clipped ReLU (H=1760 with
    8-producer gathers: 1.84 / 2.35 vs 1.26 / 1.41): those layers run the 64-unit wide
    kernels instead (_wide_ok)."""
    return H // 32 <= 42


def _xcd_lds(H: int, G: int, mt: int) -> int:
    """Static LDS bytes of the larger of the two csrc/rnn_xcd.hip kernels (16-row tiles only)."""
    if mt != 1 or _xcd_kb(H, G, True) < 0 or not _rs_ok(H):
        return 1 << 30
    # forward + reduce-scatter BPTT (static, ~61 KB at G = 3)
    return 2 * 7 * 16 * (G * 32 + 1) * 4 + 16 * 32 * 2 + 2 * 16 * G * 32 * 4 + 2 * 2 * 16 * 32 * 4 \
        + (2 * 16 * 32 * 16 if G == 3 else 16) + 16 * 4 + G * 32 * 4 + 64


def _wide_ok(H: int, cell: str) -> bool:
    """One-gate layers wider than an XCD at 32 units per workgroup (32 < H/32, H <= 1792, e.g.
    the reference's ReLU-1760) run the 64-unit wide kernels of csrc/rnn_xcd.hip (rnnw_*):
    P = ceil(H/64) <= 28 workgroups per group, one XCD. (Two 32-unit workgroups per CU also
    kept such a group on one XCD but measured slower: profiles/r3_negative_results.md.)"""
    return cell == "rnn_relu" and H % 32 == 0 and H // 32 > 32 and H <= 1792


def _xcd_p(H: int, cell: str) -> int:
    """Workgroups per group of an XCD-kernel plan."""
    return -(-H // 64) if _wide_ok(H, cell) else H // 32


# geometry experiments (tools/bench_rnn.py): minimum rows per XCD group (0: the plan's choice),
# generation-1 waves per workgroup (0: the plan's choice)
_MIN_ROWS = 0
_FORCE_NW = 0


def make_xcd_plan(N: int, H: int, cell: str, ndir: int, cus: int) -> Optional[RnnPlan]:
    """Generation-2 geometry: groups of R batch rows x all H units (H/32 workgroups of 32
    units). Prefer the most groups that still fit the chip (smaller per-step gathers), at
    most 8 so a group can live on one XCD; rows per group R <= 32."""
    G = GATES[cell]
    P = H // 32
    if _wide_ok(H, cell):
        # 8 groups (one per XCD) of R <= 8 rows: the wide BPTT's two-producers-per-load gather
        Pw = _xcd_p(H, cell)
        BG = 8 // ndir
        R = -(-N // BG)
        if R > 8 or ndir * BG * Pw > cus or Pw > cus // 8:
            return None
        return RnnPlan(N=N, NP=BG * R, BG=BG, mt=1, nw=8, persistent=True, H=H, S=H // 16, cell=cell,
                       ndir=ndir, kind="xcd", R=R, xcd_map=1)
    wide = 42 if (_rs_ok(H) and G == 3) else 32         # see _rs_ok
    if H % 32 != 0 or P > wide:          # larger H: the resident U slice would spill
        return None
    best = None
    # groups wider than an XCD (P > CUs/8) exchange across XCDs (write-through): fewer,
    # taller groups measured faster there (H=1280: R=16 27.9 vs R=11 30.3 ms/step)
    minr = _MIN_ROWS or (min(16, N) if P > cus // 8 else 1)
    for R in range(max(1, minr), 33):
        BG = -(-N // R)
        ngroups = ndir * BG
        if ngroups * P > cus:
            continue
        if ngroups > 8 and R < 16:
            continue                       # many small groups: no XCD locality, keep MFMA rows full
        mt = 1 if R <= 16 else 2
        if _xcd_lds(H, G, mt) > LDS_BYTES:
            continue
        best = (R, BG, mt)
        break
    if best is None:
        return None
    R, BG, mt = best
    xcd_map = int(ndir * BG <= 8 and P <= cus // 8)
    return RnnPlan(N=N, NP=BG * R, BG=BG, mt=mt, nw=8, persistent=True, H=H, S=H // 16, cell=cell,
                   ndir=ndir, kind="xcd", R=R, xcd_map=xcd_map)


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
    if mode == "auto":
        p = make_xcd_plan(N, H, cell, ndir, cus)
        if p is not None:
            return p
    force_nw = _FORCE_NW
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


def error_word(device: torch.device) -> torch.Tensor:
    """The device's persistent recurrence error word (int32, 0 = no timeout so far)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    w = _err_words.get(idx)
    if w is None:
        w = torch.zeros(1, device=torch.device("cuda", idx), dtype=torch.int32)
        _err_words[idx] = w
    return w


def check_errors(clear: bool = True) -> None:
    """Raise if any recurrence kernel since the last check hit its spin timeout.
    Call at a point where the host synchronises anyway (e.g. when logging the loss, once
    per eval batch, after each streaming chunk). Costs one 4-byte read per device."""
    for idx, w in list(_err_words.items()):
        v = int(w.item())
        if v != 0:
            if clear:
                w.zero_()
            raise RuntimeError("persistent recurrence kernel timed out waiting for its peers "
                               "(error bits 0x%x; grid not co-resident?) — rerun with DS2_RNN_MODE=step" % v)


# Side-stream work beside a persistent recurrence waits until that launch's last workgroup is
# resident (csrc/fill.hip wait_resident on its census word) instead of racing it for CUs at
# dispatch; a pure scheduling hint, bounded by _GATE_TICKS (2 ms of s_memrealtime)
_RESIDENCY_GATE = True
_GATE_TICKS = 200000


def _gate(census: Optional[torch.Tensor], plan: Optional["RnnPlan"]) -> None:
    """On the current stream: wait until the persistent XCD launch of ``plan`` that owns
    ``census`` holds its CUs: its last workgroup (group ngroups-1, member P-1) published its
    census word, slot ngroups * P - 1 (the buffer may be longer: wide plans use P = H / 64)."""
    if not (_RESIDENCY_GATE and census is not None and census.is_cuda and plan is not None and plan.kind == "xcd"):
        return
    if torch.cuda.is_current_stream_capturing():
        # a replayed graph orders its nodes itself (one queue, DEBUG_HIP_FORCE_GRAPH_QUEUES):
        # a spin on a launch the replay may issue after it would only wait for its timeout
        return
    last = plan.ndir * plan.BG * _xcd_p(plan.H, plan.cell) - 1
    if 0 <= last < census.numel():
        _ext.ext().wait_resident(census[last:last + 1], _GATE_TICKS)


def _next_bptt(dev: torch.device):
    """(census, plan) of the BPTT launch prefilled for the next (lower) layer, if any."""
    pre = _BWD_PREFILL.get(dev.index)
    return (pre[2][0], pre[0]) if pre is not None else (None, None)


def _stamps(kind: str, plan: "RnnPlan", grid: int, dev) -> Optional[torch.Tensor]:
    if STAMP_LOG is None:
        return None
    t = torch.zeros(grid, 8, device=dev, dtype=torch.int64)
    STAMP_LOG.append((kind, plan, t))
    return t


_PROJ_BESIDE = True   # projection grid = the CUs a carried dU GEMM leaves (see _proj_grid)


def _proj_grid(arena, plan: "RnnPlan", M: int, Nout: int, dev: torch.device) -> int:
    """Grid cap of a projection GEMM (256 x 256 tiles) launched while a carried dU GEMM
    (Trainer defer_update) still holds the CUs the previous recurrence left idle: the other
    CUs, when that costs no extra round of tiles (headline: 589 tiles are 3 rounds on 256 CUs
    and on 200). Uncapped, the projection's workgroups queued behind the dU GEMM finish a
    third of a tile round late (in-step projection ~120 us against ~92 us alone). 0 = no cap."""
    if not (_PROJ_BESIDE and arena is not None and arena.carried_gemm_beside()):
        return 0
    cus, carry = _cus(dev), _idle_cus(plan, dev)
    if carry <= 0 or cus <= carry:
        return 0
    tiles = -(-M // 256) * -(-Nout // 256)
    g = cus - carry
    return g if -(-tiles // g) == -(-tiles // cus) else 0


def _linear(x2: torch.Tensor, W16: torch.Tensor, b16: Optional[torch.Tensor], alpha: float,
            fill=None, max_grid: int = 0) -> torch.Tensor:
    """gx = alpha * x2 W16^T + b16 (bf16): the hand-written MFMA GEMM (csrc/gemm.hip) with the
    sequence-BN scale and the bias fused in its epilogue; library GEMM only for shapes the
    kernel does not cover (K % 32 != 0) or under DS2_GEMM=torch. fill: (regions, patterns) of
    the recurrence that follows, initialised by the GEMM launch (GM.matmul) or after it."""
    M, K = x2.shape
    N = W16.shape[0]
    if GM.enabled("proj") and x2.is_cuda:
        out = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
        if GM.matmul(x2, W16.t(), out, alpha=alpha, bias=b16, fill=fill, max_grid=max_grid):
            return out
    if b16 is None:
        out = torch.mm(x2, W16.t()) * alpha if alpha != 1.0 else torch.mm(x2, W16.t())
    else:
        out = torch.addmm(b16, x2, W16.t(), alpha=alpha)
    if fill is not None:
        _ext.ext().multi_fill(list(fill[0]), list(fill[1]))
    return out


def _stream_wait(dst, src) -> None:
    """dst waits for the work enqueued on src so far: one event record + wait through
    csrc/bindings.cpp stream_wait (a cached device-scope event; no event object created and
    destroyed per call as torch's wait_stream does). Every record or wait still costs its
    queue ~6 us (tools/probe_event_gap.py), so the backward issues as few as it can."""
    if dst == src:
        return
    if src.device.index == torch.cuda.current_device():
        _ext.ext().stream_wait(dst.cuda_stream, src.cuda_stream)
    else:
        dst.wait_stream(src)


class _PendingT:
    """A queued W^T shadow: transposed on the side stream by WgradScheduler.flush_transposes."""
    __slots__ = ("W16", "wT", "side", "event")

    def __init__(self, W16, wT, side):
        self.W16, self.wT, self.side, self.event = W16, wT, side, None


def _transpose_async(W16: torch.Tensor, side, sch=None):
    """W16^T (contiguous bf16) for the input-gradient GEMM, so the backward's dx GEMM reads a
    K-contiguous row-major W^T (csrc/gemm.hip / gemm8 row-row: faster than reading W column-
    major). With a scheduler the transpose is only queued: the model issues every layer's on
    the side stream once the top layer's recurrence has been enqueued (flush_transposes), so
    they run beside the FC head and the CTC instead of beside a latency-bound recurrence (the
    layer-0 one, 26 us, slowed its recurrence by ~55 us). Returns a _PendingT (or, without a
    side stream, the transposed tensor)."""
    wT = torch.empty(W16.shape[1], W16.shape[0], device=W16.device, dtype=torch.bfloat16)
    if side is None or sch is None:
        _ext.ext().transpose_bf16(W16, wT)
        return wT
    job = _PendingT(W16, wT, side)
    sch.transposes.append(job)
    return job


def _mm_bf16(a: torch.Tensor, b: torch.Tensor, fill=None) -> torch.Tensor:
    """a @ b in bf16 through csrc/gemm.hip (library GEMM for uncovered shapes). fill:
    (regions, patterns) for the next kernel, initialised by the GEMM launch or after it."""
    if GM.enabled("dx") and a.is_cuda:
        out = torch.empty(a.shape[0], b.shape[1], device=a.device, dtype=torch.bfloat16)
        if GM.matmul(a, b, out, fill=fill):
            return out
    out = torch.mm(a, b)
    if fill is not None:
        _ext.ext().multi_fill(list(fill[0]), list(fill[1]))
    return out


def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    try:
        return torch.mm(a, b, out_dtype=torch.float32)
    except (RuntimeError, TypeError):
        return torch.mm(a, b).float()


class _FwdBufs:
    """Output / state buffers of one forward recurrence launch, initialised (for the XCD
    kernels: h0 slots zero, exchange slots sentinel 0xFFFF, census words -1, the fused sum
    buffer sentinel) by ONE multi_fill right before the launch. (Initialising them on the side
    stream beside the projection GEMM measured slower: the recurrence then found its
    exchange slots out of L2, +20-40 us per layer.)"""
    __slots__ = ("y2", "ysum", "hx", "hs", "gates", "census", "fuse")


def _alloc_fwd(T: int, N: int, plan: RnnPlan, dev) -> _FwdBufs:
    C = _ext.ext()
    H, ndir = plan.H, plan.ndir
    d1 = ndir == 2
    bf16 = torch.bfloat16
    b = _FwdBufs()
    # generation-4 forward fuses the direction sum into its output stores (sentinel-filled
    # sum buffer, one direction writes through, the other adds): no torch.add launch and no
    # per-direction output round trip
    b.fuse = (plan.kind == "xcd" and d1 and _FUSE_DIRSUM and
              bool(C.rnnx_fwd_fuses_sum(H, CELL_CODE[plan.cell], plan.mt, ndir, _kernel_knobs(plan))))
    b.y2 = None if b.fuse else torch.empty(ndir, T, N, H, device=dev, dtype=bf16)
    b.ysum = torch.empty(T, N, H, device=dev, dtype=bf16) if b.fuse else None
    b.hx = torch.empty(ndir, T + 1, plan.NP, H, device=dev, dtype=bf16)
    b.hs = torch.empty(ndir, T + 1, plan.NP, H, device=dev, dtype=torch.float32)
    b.gates = (torch.empty(ndir, T, plan.NP, H, 4, device=dev, dtype=torch.float32)
               if plan.cell == "gru" else None)
    b.census = torch.empty(ndir * plan.BG * (H // 32), device=dev, dtype=torch.int32) \
        if plan.kind == "xcd" else None
    return b


def _fill_regions(b: _FwdBufs, plan: RnnPlan):
    """(regions, patterns) that an XCD forward launch needs initialised."""
    ndir = plan.ndir
    hx, hs = b.hx, b.hs
    regions = ([hx[d, 0] for d in range(ndir)] + [hx[d, 1:] for d in range(ndir)] +
               [hs[d, 0] for d in range(ndir)] + [b.census] + ([b.ysum] if b.fuse else []))
    return regions, [0] * ndir + [-1] * ndir + [0] * ndir + [-1] + ([-1] if b.fuse else [])


def _fill_fwd(b: _FwdBufs, plan: RnnPlan) -> None:
    _ext.ext().multi_fill(*_fill_regions(b, plan))


def _run_fwd(gx, lens, U, bh, plan: RnnPlan, h0=None, bufs: Optional[_FwdBufs] = None):
    """Launch the persistent forward recurrence over gx [T, N, ndir*G*H] (bf16).
    U / bh: per-direction lists (bf16 [G*H, H] / fp32 [G*H] or None).
    h0: optional initial state [ndir, N, H] (streaming state carry; zeros otherwise).
    bufs: the launch's buffers, already initialised (the projection GEMM that produced gx
    filled them: _alloc_fwd + _fill_regions); allocated and filled here when None.
    Returns (y [T, N, H] bf16 = sum of directions, saved-state tuple)."""
    C = _ext.ext()
    T, N, gstride = gx.shape
    H, ndir = plan.H, plan.ndir
    steps = T
    dev = gx.device
    d1 = ndir == 2
    b = bufs if bufs is not None else _alloc_fwd(T, N, plan, dev)
    fuse, y2, ysum, hx, hs, gates = b.fuse, b.y2, b.ysum, b.hx, b.hs, b.gates
    if plan.kind == "xcd":
        census = b.census
        err = error_word(dev)
        if bufs is None:
            _fill_fwd(b, plan)
        if h0 is not None:
            hs[:, 0, :N].copy_(h0)
            hx[:, 0, :N].copy_(h0)
        yf, yb = (ysum, ysum) if fuse else (y2[0], y2[1] if d1 else None)
        C.rnnx_fwd(gx, lens, U[0], U[1] if d1 else None, bh[0], bh[1] if d1 else None,
                   yf, yb, hx[0], hx[1] if d1 else None,
                   hs[0], hs[1] if d1 else None,
                   gates[0] if gates is not None else None,
                   gates[1] if (gates is not None and d1) else None,
                   census, err, T, N, plan.NP, H, plan.BG, plan.R, steps, gstride, ndir,
                   CELL_CODE[plan.cell], plan.mt, TIMEOUT_TICKS, plan.xcd_map, _kernel_knobs(plan),
                   _stamps("fwd", plan, int(C.rnnx_info(H, GATES[plan.cell], plan.mt, ndir * plan.BG,
                                                         plan.xcd_map)["grid"]), dev), ysum)
        y = ysum if fuse else (torch.add(y2[0], y2[1]) if d1 else y2[0])
        return y, (hx, hs, gates if gates is not None else torch.empty(0, device=dev))
    hx[:, 0].zero_()                         # h0
    hs[:, 0].zero_()
    if h0 is not None:
        hs[:, 0, :N].copy_(h0)
        hx[:, 0, :N].copy_(h0)
    err = error_word(dev)
    flags = torch.zeros(ndir * plan.BG * plan.S, device=dev, dtype=torch.int32)
    C.rnn_fwd(gx, lens, U[0], U[1] if d1 else None,
              bh[0], bh[1] if d1 else None,
              y2[0], y2[1] if d1 else None, hx[0], hx[1] if d1 else None,
              hs[0], hs[1] if d1 else None,
              gates[0] if gates is not None else None,
              gates[1] if (gates is not None and d1) else None,
              flags, err, T, N, plan.NP, H, plan.BG, steps, gstride, ndir,
              CELL_CODE[plan.cell], plan.nw, plan.mt, plan.persistent, TIMEOUT_TICKS,
              _stamps("fwd", plan, flags.numel(), dev))
    y = torch.add(y2[0], y2[1]) if d1 else y2[0]
    return y, (hx, hs, gates if gates is not None else torch.empty(0, device=dev))


_FWD_FAMILY = {6: "rnnw_fwd (wide one-gate)", 5: "rnne_fwd (gen 5)", 4: "rnnq_fwd (gen 4)", 2: "rnnx_fwd (gen 2)"}
_BWD_FAMILY = {6: "rnnw_bwd (wide one-gate)", 3: "rnnrs_bwd (reduce-scatter)"}


def kernel_families(plan: RnnPlan) -> Tuple[str, str]:
    """(forward, BPTT) kernel family a bf16 plan launches: csrc/rnn_xcd.hip's dispatch
    (ds2_rnnx_fwd_family / ds2_rnnx_bwd_family, the functions the launches themselves branch
    on) or generation 1 (csrc/rnn_persistent.hip), persistent or one launch per step. The fp8
    layers (fp8_recurrence_ok) run csrc/rnn_fp8.hip instead. Raises if the xcd dispatch would
    refuse the plan."""
    if plan.kind != "xcd":
        g1 = "rnn_%s (gen 1, " + ("persistent)" if plan.persistent else "step launches)")
        return g1 % "fwd", g1 % "bwd"
    C = _ext.ext()
    f = int(C.rnnx_fwd_family(plan.H, CELL_CODE[plan.cell], plan.mt, _kernel_knobs(plan)))
    b = int(C.rnnx_bwd_family(plan.H, CELL_CODE[plan.cell], plan.mt, plan.R))
    if f not in _FWD_FAMILY or b not in _BWD_FAMILY:
        raise ValueError("xcd plan not covered by csrc/rnn_xcd.hip: %r" % (plan,))
    return _FWD_FAMILY[f], _BWD_FAMILY[b]


def fp8_recurrence_ok(plan: RnnPlan, N: int) -> bool:
    """csrc/rnn_fp8.hip serves this GRU layer (config 5's fp8 mode): H % 256 == 0, H/64 <= 32
    workgroups per group (one XCD), 8 groups of <= 8 rows, and the same padded batch rows as
    the layer's bf16 BPTT plan (which runs on the saved state unchanged)."""
    if plan.cell != "gru" or plan.kind != "xcd" or not _ext.ext().rnnf8_supported(plan.H, N, plan.ndir):
        return False
    BG = 8 // plan.ndir
    return BG * (-(-N // BG)) == plan.NP


def _quant_u(U, plan: RnnPlan, rowmajor: bool = True, transposed: bool = True):
    """(U8 [ndir, 3H, H] | None, U8T [ndir, H, 3H] | None, uexp int32 [ndir]): e4m3 copies of the
    recurrent weights with one power-of-two scale per direction, computed on the device: the
    forward's layout and the BPTT's transposed one from one read of U (csrc/rnn_fp8.hip
    quant_u_kernel; two launches for every direction and layout)."""
    C = _ext.ext()
    H, ndir = plan.H, plan.ndir
    dev = U[0].device
    U8 = torch.empty(ndir, 3 * H, H, device=dev, dtype=torch.uint8) if rowmajor else None
    U8T = torch.empty(ndir, H, 3 * H, device=dev, dtype=torch.uint8) if transposed else None
    words = torch.empty(ndir, device=dev, dtype=torch.int32)
    part = torch.empty(ndir * 256, device=dev, dtype=torch.float32)
    C.fp8_quant_u(U[0].contiguous(), U[1].contiguous() if ndir == 2 else None, U8, U8T, words, part)
    return U8, U8T, words


def _run_fwd_fp8(gx, lens, U, bh, plan: RnnPlan, keep: Optional[dict] = None, pair: bool = False):
    """GRU forward with e4m3 recurrent weights (one power-of-two scale per direction, computed
    on the device) and an e4m3 hidden-state exchange: groups of H/64 workgroups on one XCD
    (csrc/rnn_fp8.hip). Returns (y, (hx, hs, gates)) in the layout of _run_fwd. With keep (a
    dict), the transposed e4m3 U of the same quantisation goes into keep["quant"] for the BPTT.
    pair (two directions): y is the [2, T, N, H] pair of direction outputs, unsummed — the next
    fp8 layer's quantiser sums them (fp8_linear x2b)."""
    C = _ext.ext()
    T, N, gstride = gx.shape
    H, ndir = plan.H, plan.ndir
    BG = 8 // ndir
    R = -(-N // BG)
    NP = BG * R
    dev = gx.device
    U8, U8T, words = _quant_u(U, plan, True, keep is not None)
    if keep is not None:
        keep["quant"] = (U8T, words)
    y2 = torch.empty(ndir, T, N, H, device=dev, dtype=torch.bfloat16)
    hq = torch.empty(ndir, T + 1, NP, H, device=dev, dtype=torch.uint8)
    hx = torch.empty(ndir, T + 1, NP, H, device=dev, dtype=torch.bfloat16)
    hs = torch.empty(ndir, T + 1, NP, H, device=dev, dtype=torch.float32)
    gates = torch.empty(ndir, T, NP, H, 4, device=dev, dtype=torch.float32)
    census = torch.empty(ndir * BG * (H // 64), device=dev, dtype=torch.int32)
    # e4m3 h0 = 0x00, exchange slots 0xFF ("not yet produced"), census -1, bf16 / fp32 h0 = 0
    C.multi_fill([hq[d, 0] for d in range(ndir)] + [hq[d, 1:] for d in range(ndir)] + [census],
                 [0] * ndir + [-1] * ndir + [-1])
    C.multi_fill([hx[d, 0] for d in range(ndir)] + [hs[d, 0] for d in range(ndir)], [0] * (2 * ndir))
    C.rnnf8_fwd(gx.contiguous(), lens, U8, words, bh[0], bh[1] if ndir == 2 else None, y2, hq, hx, hs, gates, census,
                error_word(dev), T, N, NP, H, BG, R, T, gstride, ndir, TIMEOUT_TICKS, 1)
    y = (y2 if pair else torch.add(y2[0], y2[1])) if ndir == 2 else y2[0]
    return y, (hx, hs, gates)


# config 5's fp8 mode: the BPTT too runs on the fp8 geometry (csrc/rnn_fp8.hip rnnf8_bwd_kernel:
# e4m3 U^T and dg operands, one XCD per group) where the fp8 forward ran; False keeps the bf16
# reduce-scatter BPTT on the saved states (tests compare the two)
# (tools/bench_rnn_fp8.py, H = 1280, N = 32: 4.72 vs 5.32 us/step; config 5 fp8 19.58 vs 19.69-19.79
# ms/step, same box)
_FP8_BPTT = True


def fp8_bptt_ok(plan: RnnPlan, N: int) -> bool:
    return _FP8_BPTT and fp8_recurrence_ok(plan, N) and bool(_ext.ext().rnnf8_bwd_supported(plan.H, N, plan.ndir))


def _run_bwd_fp8(dy, lens, U, hs, gates, plan: RnnPlan, gstride: int, dgx_scale: float = 1.0,
                 want_bias: bool = True, quant=None):
    """fp8 GRU BPTT (csrc/rnn_fp8.hip): groups of H/64 workgroups on one XCD, U^T in e4m3 with
    a per-tensor power-of-two scale (the forward's, via quant, or computed here on the device), the
    gate gradients requantised to e4m3 per (row, 32-unit group) each step. Same outputs as _run_bwd: (dgx [T, N, gstride] bf16 x
    dgx_scale, dgh [ndir, steps, NP, 3H] bf16, bias partials [2, ndir, BG, 3H] or None)."""
    C = _ext.ext()
    T, N, H = dy.shape
    ndir = plan.ndir
    BG = 8 // ndir
    R = -(-N // BG)
    NP = BG * R
    assert NP == plan.NP, (NP, plan.NP)
    dev = dy.device
    steps = T
    dy = dy.to(torch.bfloat16).contiguous()
    # quant: (U8T, uexp) of the forward's quantisation of the same U, else quantised here
    U8T, words = quant if quant is not None else _quant_u(U, plan, False, True)[1:]
    dgh = torch.empty(ndir, steps, NP, 3 * H, device=dev, dtype=torch.bfloat16)
    dgx = torch.empty(T, N, gstride, device=dev, dtype=torch.bfloat16)
    census = torch.empty(ndir * BG * (H // 64), device=dev, dtype=torch.int32)
    parts = torch.empty(2, ndir, BG, 3 * H, device=dev, dtype=torch.float32) if want_bias else None
    ring = torch.empty(ndir, int(C.rnnf8_ring_words(H, BG, R)), device=dev, dtype=torch.int32)
    _fill_bwd(census, parts, ring)
    C.rnnf8_bwd(dy, lens, U8T, words, hs, gates, dgh, dgx, parts[0] if parts is not None else None,
                parts[1] if parts is not None else None, float(dgx_scale), census, error_word(dev), ring,
                T, N, NP, H, BG, R, steps, gstride, ndir, TIMEOUT_TICKS, 1)
    return dgx, dgh, parts


def _alloc_bwd(plan: RnnPlan, want_bias: bool, dev) -> tuple:
    """(census, parts, ring) of an XCD BPTT launch and the multi_fill that initialises them:
    census words -1, bias partials 0, the reduce-scatter ring 0xFFFFFFFF (none depends on T)."""
    H, ndir, G = plan.H, plan.ndir, GATES[plan.cell]
    census = torch.empty(ndir * plan.BG * (H // 32), device=dev, dtype=torch.int32)
    parts = torch.empty(2 if plan.cell == "gru" else 1, ndir, plan.BG, G * H, device=dev,
                        dtype=torch.float32) if want_bias else None
    rf = int(_ext.ext().rnnx_ring_floats(H, plan.BG, plan.R))
    ring = torch.empty(ndir, rf, device=dev, dtype=torch.float32)
    return census, parts, ring


def _bwd_fill_regions(census, parts, ring):
    regions, pats = [census], [-1]
    if parts is not None:
        regions.append(parts)
        pats.append(0)
    return regions + [ring], pats + [-1]


def _fill_bwd(census, parts, ring) -> None:
    _ext.ext().multi_fill(*_bwd_fill_regions(census, parts, ring))     # one launch for every init


# device index -> (plan, stream, (census, parts, ring)): the next BPTT's buffers, initialised by
# the input-gradient GEMM of the layer above (FusedBiLayer._backward), so no fill launch sits
# between that GEMM and the BPTT it feeds. Taken (once) by _run_bwd on the same plan and stream.
_BWD_PREFILL = {}


def _prefill_bwd(plan: "RnnPlan", dev):
    """Allocate the next BPTT's buffers; returns the fill for the GEMM that precedes it."""
    bufs = _alloc_bwd(plan, True, dev)
    _BWD_PREFILL[dev.index] = (plan, torch.cuda.current_stream(dev).cuda_stream, bufs)
    return _bwd_fill_regions(*bufs)


def _run_bwd(dy, lens, U, hx, hs, gates, plan: RnnPlan, gstride: int, dgx_scale: float = 1.0,
             want_bias: bool = True):
    """Launch BPTT. Returns (dgx [T, N, gstride] bf16 (x dgx_scale), dgh [ndir, steps, NP, G*H],
    parts [k, ndir, BG, G*H] fp32 in-kernel bias-gradient partials: k=0 input bias, k=1 GRU
    recurrent bias; None if want_bias is False)."""
    C = _ext.ext()
    T, N, H = dy.shape
    ndir, G = plan.ndir, GATES[plan.cell]
    steps = T
    dev = dy.device
    d1 = ndir == 2
    dy = dy.to(torch.bfloat16).contiguous()
    dgh = torch.empty(ndir, steps, plan.NP, G * H, device=dev, dtype=torch.bfloat16)
    dgx = torch.empty(T, N, gstride, device=dev, dtype=torch.bfloat16)
    has_g = gates.numel() > 0
    if plan.kind == "xcd":
        err = error_word(dev)
        # generation-3 BPTT: reduce-scatter of partials through a 3-slot ring (readiness =
        # per-use tag in each word's LSB, ring filled with 0xFFFFFFFF); dgh is a plain output
        pre = _BWD_PREFILL.pop(dev.index, None)
        if (pre is not None and want_bias and pre[0] is plan and
                pre[1] == torch.cuda.current_stream(dev).cuda_stream):
            census, parts, ring = pre[2]
        else:
            census, parts, ring = _alloc_bwd(plan, want_bias, dev)
            _fill_bwd(census, parts, ring)
        C.rnnx_bwd(dy, lens, U[0], U[1] if d1 else None, hs[0], hs[1] if d1 else None,
                   gates[0] if has_g else None, gates[1] if (has_g and d1) else None,
                   dgh[0], dgh[1] if d1 else None, dgx,
                   parts[0] if parts is not None else None,
                   parts[1] if (parts is not None and plan.cell == "gru") else None,
                   float(dgx_scale), census, err, T, N, plan.NP, H, plan.BG, plan.R, steps, gstride, ndir,
                   CELL_CODE[plan.cell], plan.mt, TIMEOUT_TICKS, plan.xcd_map, _kernel_knobs(plan),
                   _stamps("bwd", plan, int(C.rnnx_info(H, G, plan.mt, ndir * plan.BG, plan.xcd_map)["grid"]), dev),
                   ring[0], ring[1] if d1 else None)
        return dgx, dgh, parts
    err = error_word(dev)
    parts = torch.zeros(2 if plan.cell == "gru" else 1, ndir, plan.BG, G * H, device=dev,
                        dtype=torch.float32) if want_bias else None
    carry = None if plan.persistent else torch.zeros(ndir, plan.NP, H, device=dev, dtype=torch.float32)
    flags = torch.zeros(ndir * plan.BG * plan.S, device=dev, dtype=torch.int32)
    C.rnn_bwd(dy, lens, U[0], U[1] if d1 else None, hs[0], hs[1] if d1 else None,
              gates[0] if has_g else None, gates[1] if (has_g and d1) else None,
              dgh[0], dgh[1] if d1 else None, dgx,
              carry[0] if carry is not None else None,
              carry[1] if (carry is not None and d1) else None,
              flags, err, T, N, plan.NP, H, plan.BG, steps, gstride, ndir,
              CELL_CODE[plan.cell], plan.nw, plan.mt, plan.persistent, TIMEOUT_TICKS,
              _stamps("bwd", plan, flags.numel(), dev),
              parts[0] if parts is not None else None,
              parts[1] if (parts is not None and plan.cell == "gru") else None,
              float(dgx_scale))
    return dgx, dgh, parts


def _dU(dgh, hx, d: int, plan: RnnPlan, p_U):
    steps = dgh.shape[1]
    G = GATES[plan.cell]
    g2 = dgh[d].view(steps * plan.NP, G * plan.H)
    h2 = hx[d, :steps].reshape(steps * plan.NP, plan.H)
    return mm_into(p_U, g2.t(), h2)


class BiRecurrence(torch.autograd.Function):
    """y = sum_d recurrence_d(gx[..., d]) over a [T, N, ndir*G*H] bf16 projection.
    Used when the projection needs autograd of its own (sequence-BN in batch mode)."""

    @staticmethod
    def forward(ctx, gx, lens, U_f, U_b, bh_f, bh_b, plan: RnnPlan):
        gx = gx.contiguous()
        lens = lens.to(device=gx.device, dtype=torch.int32).contiguous()
        U = [U_f.contiguous(), U_b.contiguous() if U_b is not None else None]
        bh = [b.contiguous().float() if b is not None else None for b in (bh_f, bh_b)]
        y, (hx, hs, gates) = _run_fwd(gx, lens, U, bh, plan)
        ctx.save_for_backward(lens, U[0], U[1] if U[1] is not None else torch.empty(0, device=gx.device),
                              hx, hs, gates)
        ctx.plan = plan
        ctx.gstride = gx.shape[2]
        ctx.has_bh = (bh_f is not None, bh_b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        lens, U_f, U_b, hx, hs, gates = ctx.saved_tensors
        plan: RnnPlan = ctx.plan
        d1 = plan.ndir == 2
        dgx, dgh, parts = _run_bwd(dy, lens, [U_f, U_b if d1 else None], hx, hs, gates, plan, ctx.gstride,
                                   want_bias=any(ctx.has_bh))
        dbh = parts[1].sum(1) if parts is not None and parts.shape[0] > 1 else None
        dU = [_dU(dgh, hx, d, plan, None) for d in range(plan.ndir)]
        gb = [dbh[d] if (dbh is not None and ctx.has_bh[d]) else None for d in range(plan.ndir)]
        return (dgx, None, dU[0].to(U_f.dtype), dU[1].to(U_f.dtype) if d1 else None,
                gb[0], gb[1] if d1 else None, None)


FP8_MAX = 448.0      # OCP e4m3 (gfx950 MFMA fp8 is OCP e4m3fn, not MI300's fnuz)


def fp8_linear(x2: torch.Tensor, W16: torch.Tensor, b16: torch.Tensor, alpha: float,
               x2b: Optional[torch.Tensor] = None, xsum: Optional[torch.Tensor] = None) -> torch.Tensor:
    """alpha * x2 @ W16^T + b16 with both operands quantised to fp8 e4m3 (per-tensor amax
    scaling, scales kept on the device: no host sync) and multiplied on the CDNA4 fp8 MFMA
    path of the hand-written gemm8 kernel (ops/gemm.py linear_fp8); bf16 output. Forward-only
    precision reduction: the backward GEMMs keep the bf16 copies (fp8 'mixed precision',
    BASELINE config 5). CPU: the same arithmetic in torch (dequantised fp32 product).
    x2b / xsum: the input is the direction sum x2 + x2b, written to xsum by the quantiser."""
    if x2b is not None:
        if x2.is_cuda and not (x2.shape[1] % 8 or W16.shape[0] % 4):
            return GM.linear_fp8(x2, W16, b16, alpha, x2b, xsum)
        torch.add(x2, x2b, out=xsum)
        x2 = xsum
    if x2.is_cuda:
        if x2.shape[1] % 8 or W16.shape[0] % 4:
            return torch.addmm(b16, x2, W16.t(), alpha=alpha)      # outside the kernels' contract
        return GM.linear_fp8(x2, W16, b16, alpha)
    f8 = torch.float8_e4m3fn
    sx = (x2.abs().amax().float() / FP8_MAX).clamp(min=1e-12)
    sw = (W16.abs().amax().float() / FP8_MAX).clamp(min=1e-12)
    xq = (x2.float() / sx).clamp(-FP8_MAX, FP8_MAX).to(f8).float() * sx
    wq = (W16.float() / sw).clamp(-FP8_MAX, FP8_MAX).to(f8).float() * sw
    return (alpha * (xq @ wq.t()) + b16.float()).to(torch.bfloat16)


def _bf16_group(params):
    """bf16 tensor for the row-concatenation of ``params`` (all 2-D with equal columns, or
    all 1-D): a zero-copy view of the arena's bf16 shadow when they are packed there."""
    arena = arena_of(params[0])
    if arena is not None:
        v = arena.group_view(params, "p16")
        if v is not None:
            if params[0].dim() == 1:
                return v
            return v.view(-1, params[0].shape[1])
    return torch.cat([p.to(torch.bfloat16) for p in params], 0)


def _bf16(p):
    return p.bf16 if arena_of(p) is not None else p.to(torch.bfloat16)


def _bias_grads(params, part):
    """Reduce in-kernel partials [ndir, BG, G*H] over batch groups into the bias grads:
    one sum kernel writing straight into the packed arena rows when the direction biases
    are adjacent there; otherwise per-direction (returned for autograd if not arena-managed)."""
    return _bias_grads_multi([(params, part)])[0]


def _bias_grads_multi(jobs):
    """_bias_grads of several (params, partials) pairs (a layer's input bias b and GRU recurrent
    bias b_h): every arena-packed group in ONE csrc/reduce.hip col_sum launch (written, or
    accumulated after an earlier producer) instead of a torch reduce kernel each."""
    res = [[None, None] for _ in jobs]
    fused = []
    for i, (params, part) in enumerate(jobs):
        if params[0] is None:
            continue
        arena = arena_of(params[0])
        grp = arena.group_view(params, "grad") if arena is not None else None
        firsts = [arena.first_write(p) for p in params] if arena is not None else []
        if grp is not None and part.is_cuda and part.is_contiguous() and len(set(firsts)) == 1:
            fused.append((params, part, grp, not firsts[0]))
            continue
        if arena is not None and grp is not None and all(firsts):
            torch.sum(part, dim=1, out=grp.view(len(params), -1))
            arena.grad_done(*params)
            continue
        for d, p in enumerate(params):
            res[i][d] = emit_grad(p, part[d].sum(0))
    if fused:
        _ext.ext().col_sum([f[1] for f in fused], [f[2] for f in fused], [f[3] for f in fused])
        for params, _, _, _ in fused:
            arena_of(params[0]).grad_done(*params)
    return res


class FusedBiLayer(torch.autograd.Function):
    """One whole (bi)directional recurrent layer with manual backward.

    forward:  gx = alpha * x [W_fw; W_bw]^T + [b_fw; b_bw]     (one GEMM, bf16 out)
              y  = sum_d recurrence_d(gx_d)                     (persistent kernel)
    backward: dgx (pre-scaled by alpha), db, db_h               (BPTT kernel, bias sums in-kernel)
              dx = dgx [W_fw; W_bw]                             (critical path: feeds layer below)
              dW = dgx^T x, dU_d = dgh_d^T h_d                  (fp32 straight into main_grad)
    alpha = 1/sqrt(1+eps) folds the reference's frozen sequence-BN (quirk Q3); 1 for 'none'.

    fp8 stacks (config 5): with pair_out an fp8 bidirectional layer returns its two direction
    outputs unsummed, [2, T, N, H], and the next fp8 layer takes that pair as x: its quantiser
    writes the sum (bitwise torch.add) while it takes the amax (fp8_linear x2b), so the
    direction sum costs no launch of its own (the sum fused into an existing pass,
    src/custom_ops.py:94-95). The pair's gradient is the sum's, shared by both halves.
    """

    @staticmethod
    def forward(ctx, x, lens, plan: RnnPlan, alpha: float, idx: int, fp8: bool, W_f, W_b, U_f, U_b, b_f, b_b,
                bh_f, bh_b, pair_out: bool = False):
        pair_in = x.dim() == 4
        T, N, D = x.shape[-3:]
        arena = arena_of(W_f)
        if arena is not None:
            # an optimizer update carried over from the previous step (Trainer defer_update)
            # may still be writing these weights on the side stream
            arena.await_params(W_f, W_b, U_f, U_b, b_f, b_b, bh_f, bh_b)
        dirs_W = [W_f] + ([W_b] if W_b is not None else [])
        dirs_b = [b_f] + ([b_b] if b_b is not None else [])
        W16 = _bf16_group(dirs_W)                     # [ndir*G*H, D]
        b16 = _bf16_group(dirs_b)                     # [ndir*G*H]
        if pair_in:
            if not fp8:
                raise ValueError("a direction pair feeds only an fp8 layer (its quantiser sums it)")
            xa, xb = x[0].to(torch.bfloat16).contiguous(), x[1].to(torch.bfloat16).contiguous()
            x16 = torch.empty(T, N, D, device=x.device, dtype=torch.bfloat16)     # written by the quantiser
        else:
            x16 = x.to(torch.bfloat16).contiguous()
        x2 = x16.view(T * N, D)
        ctx.pair_in = pair_in
        fp8_rec = fp8 and x.is_cuda and fp8_recurrence_ok(plan, N)
        bufs = fill = None
        if x.is_cuda and not fp8_rec and plan.kind == "xcd":
            # the recurrence's buffers are initialised by the projection GEMM's idle workgroups
            # (csrc/gemm8.hip DS2Fill): no separate fill launch between the two
            bufs = _alloc_fwd(T, N, plan, x.device)
            fill = _fill_regions(bufs, plan)
        if pair_in:
            gx = fp8_linear(xa.view(T * N, D), W16, b16, alpha, xb.view(T * N, D), x2).view(T, N, -1)
            if fill is not None:
                _ext.ext().multi_fill(*fill)
        elif fp8:
            gx = fp8_linear(x2, W16, b16, alpha).view(T, N, -1)
            if fill is not None:
                _ext.ext().multi_fill(*fill)
        else:
            pg = _proj_grid(arena, plan, T * N, W16.shape[0], x.device) if x.is_cuda else 0
            gx = _linear(x2, W16, b16, alpha, fill=fill, max_grid=pg).view(T, N, -1)
        if arena is not None and x.is_cuda:
            # the next chunk of the optimizer update carried over from the previous step (the
            # layer above's, or the head's): on the side stream behind this projection, i.e.
            # beside this layer's recurrence on the CUs it leaves idle (gated on its residency)
            census = bufs.census if bufs is not None else None
            arena.issue_pending_update(_idle_cus(plan, x.device), gate=lambda: _gate(census, plan))
        lens = lens.to(device=x.device, dtype=torch.int32).contiguous()
        U = [_bf16(U_f), _bf16(U_b) if U_b is not None else None]
        bh = [b.float() if b is not None else None for b in (bh_f, bh_b)]
        wT = None
        if x.is_cuda and ctx.needs_input_grad[0] and GM.enabled("dx") and W16.shape[1] % 8 == 0 and \
                W16.shape[0] % 8 == 0:
            arena = arena_of(W_f)
            wT = _transpose_async(W16, wgrad_stream(x.device, arena), arena.wgrad if arena is not None else None)
        ctx.fp8_bwd = False
        if fp8_rec:
            # config 5's fp8 mode: the recurrence too (e4m3 U and h exchange), and its BPTT on the
            # same geometry with the same e4m3 U (rnnf8_bwd_kernel; dg requantised per row). The
            # gradient is straight-through with respect to the quantisation of the exchanged h and
            # of dg (no quantisation gradient); tests/test_convergence_gpu.py pins the resulting
            # 300-step loss curve against the bf16 recurrence
            ctx.fp8_bwd = fp8_bptt_ok(plan, N)
            keep = {} if ctx.fp8_bwd else None
            y, (hx, hs, gates) = _run_fwd_fp8(gx, lens, U, bh, plan, keep, pair=pair_out and plan.ndir == 2)
            ctx.fp8_quant = keep["quant"] if keep is not None else None
        else:
            y, (hx, hs, gates) = _run_fwd(gx, lens, U, bh, plan, bufs=bufs)
        dev = x.device
        ctx.save_for_backward(x16, lens, W16, U[0], U[1] if U[1] is not None else torch.empty(0, device=dev),
                              hx, hs, gates)
        ctx.wT = wT
        ctx.params = (W_f, W_b, U_f, U_b, b_f, b_b, bh_f, bh_b)
        ctx.plan = plan
        ctx.alpha = alpha
        ctx.idx = idx
        return y

    @staticmethod
    def backward(ctx, dy):
        if dy.dim() == 4:
            # the pair output's gradient: the next layer's quantiser returns the sum's gradient
            # for both halves (one tensor expanded). A materialised dy means a second consumer
            # (the model only pairs a layer with the fp8 layer above it, deepspeech2.py
            # recurrent): refused without comparing the halves, which would sync the host
            # (and raise inside a step-graph capture)
            if dy.stride(0) != 0:
                raise RuntimeError("direction-pair output consumed other than by the next layer's quantiser")
            dy = dy[0]
        with TR.phase(TR.rnn_cell(ctx.idx, True)):
            return FusedBiLayer._backward(ctx, dy)

    @staticmethod
    def _backward(ctx, dy):
        x16, lens, W16, U_f16, U_b16, hx, hs, gates = ctx.saved_tensors
        plan: RnnPlan = ctx.plan
        W_f, W_b, U_f, U_b, b_f, b_b, bh_f, bh_b = ctx.params
        d1 = plan.ndir == 2
        T, N, D = x16.shape
        GH = GATES[plan.cell] * plan.H
        if getattr(ctx, "fp8_bwd", False):
            dgx, dgh, parts = _run_bwd_fp8(dy, lens, [U_f16, U_b16 if d1 else None], hs, gates, plan,
                                           plan.ndir * GH, dgx_scale=ctx.alpha, quant=ctx.fp8_quant)
            ctx.fp8_quant = None
        else:
            dgx, dgh, parts = _run_bwd(dy, lens, [U_f16, U_b16 if d1 else None], hx, hs, gates, plan,
                                       plan.ndir * GH, dgx_scale=ctx.alpha)
        dgx2 = dgx.view(T * N, plan.ndir * GH)

        def input_grad():
            if not ctx.needs_input_grad[0]:
                return None
            if ctx.wT is not None:
                wT = ctx.wT
                if isinstance(wT, _PendingT):
                    sch_t = arena_of(W_f).wgrad
                    if wT.event is None:                 # not flushed by the model: do it now
                        sch_t.flush_transposes()
                    sch_t.wait_transposes(torch.cuda.current_stream(dgx.device), wT.event)
                    wT = wT.wT
                # the layer below's BPTT buffers ride on this GEMM (same plan in a DS2 stack;
                # an fp8 or differently shaped layer below just leaves them unused)
                fill = (_prefill_bwd(plan, dgx.device) if ctx.idx >= 1 and plan.kind == "xcd" and
                        not getattr(ctx, "fp8_bwd", False) else None)
                dx = _mm_bf16(dgx2, wT.t(), fill=fill).view(T, N, D)
            else:
                dx = _mm_bf16(dgx2, W16).view(T, N, D)
            return dx.unsqueeze(0).expand(2, T, N, D) if ctx.pair_in else dx

        # ---- weight gradients (off the critical path) ----
        # only arena-managed weights (gradients written to main_grad, nothing returned to
        # autograd) may be produced on another stream; the Trainer joins it before Adam
        side = wgrad_stream(x16.device, arena_of(ctx.params[0]))
        sch = arena_of(ctx.params[0]).wgrad if side is not None else None
        if (side is not None and ctx.idx == 0 and _GROUP_BEFORE_DX and ctx.wT is not None and sch.grouped and
                sch.defer_input and _defer_wgrad(plan, x16.device)):
            # bottom layer: the grouped weight-gradient launch (and the optimizer range behind it)
            # goes out before layer 0's dx GEMM, so it starts as the last BPTT ends (the dx GEMM
            # reads the transposed W^T copy, which the optimizer does not write; without that copy
            # dx would read the arena's bf16 shadow that the optimizer range rewrites, so this
            # ordering is taken only when ctx.wT exists)
            _stream_wait(side, torch.cuda.current_stream(x16.device))
            sch.hold(x16, dgx, dgh, hx, parts)
            with torch.cuda.stream(side):
                res = FusedBiLayer._weight_grads(ctx, x16, dgx2, dgh, hx, parts, None)
            dx = input_grad()
            ctx.wT = None
            return (dx,) + tuple(res[1:])
        dx = input_grad()
        ctx.wT = None
        if side is None:
            return FusedBiLayer._weight_grads(ctx, x16, dgx2, dgh, hx, parts, dx)
        # The layer below only needs dx: its BPTT (200 of the 256 CUs, latency-bound) runs
        # while these GEMMs fill the idle CUs. Gradients land in the arena on the side
        # stream, and the bucket hooks fire inside it, so an all-reduce waits for them.
        _stream_wait(side, torch.cuda.current_stream(x16.device))
        sch.hold(x16, dgx, dgh, hx, parts)
        with torch.cuda.stream(side):
            if ctx.idx >= 1 and not (sch.defer_input and _defer_layer(plan, x16.device, ctx.idx, x16.shape[0])):
                _gate(*_next_bptt(x16.device))        # the lower layer's BPTT holds its CUs first
            return FusedBiLayer._weight_grads(ctx, x16, dgx2, dgh, hx, parts, dx)

    @staticmethod
    def _weight_grads(ctx, x16, dgx2, dgh, hx, parts, dx):
        plan: RnnPlan = ctx.plan
        W_f, W_b, U_f, U_b, b_f, b_b, bh_f, bh_b = ctx.params
        d1 = plan.ndir == 2
        T, N, D = x16.shape
        GH = GATES[plan.cell] * plan.H
        x2 = x16.view(T * N, D)
        arena = arena_of(W_f)
        gW = [None, None]
        grp = arena.group_view([W_f, W_b] if d1 else [W_f], "grad") if arena is not None else None
        if grp is not None and arena.first_write(W_f) and (not d1 or arena.first_write(W_b)):
            def dw_done(W_f=W_f, W_b=W_b if d1 else None):
                arena.grad_done(W_f, W_b)

            sch = arena.wgrad
            on_side = x16.is_cuda and sch.on_side(x16.device)
            grouped = sch.grouped and on_side
            defer_w = sch.defer_input and on_side and (ctx.idx >= 1 or grouped) and _defer_layer(plan, x16.device,
                                                                                                  ctx.idx, T)
            fp8b = bool(getattr(ctx, "fp8_bwd", False))
            cap_w = (_beside_grid(plan, x16.device, not sch.defer_input, fp8b)
                     if (on_side and ctx.idx > 0 and not defer_w) else 0)

            def dw(grp=grp, dgx2=dgx2, x2=x2, cap=cap_w):
                mm_into(W_f, dgx2.t(), x2, out=grp.view(plan.ndir * GH, D), max_grid=cap)
                dw_done()
            if defer_w:
                # run after the last recurrent layer's BPTT (grouped: every layer's, in one launch)
                ops = GM.group_operands(dgx2.t(), x2, grp.view(plan.ndir * GH, D)) if grouped else None
                sch.deferred.append(Deferred(dw, (dgx2, x2), [ops + (grp.view(plan.ndir * GH, D),)] if ops else None,
                                             dw_done))
                arena.hold_report(W_f, W_b if d1 else None)
                sch.queue_end_of_backward()
            else:
                dw()
            if ctx.idx == 0 and not grouped:
                sch.flush()
        else:
            for d, p in enumerate([W_f, W_b] if d1 else [W_f]):
                g = mm_into(p, dgx2[:, d * GH:(d + 1) * GH].t(), x2)
                if g is None:
                    arena.grad_done(p)
                gW[d] = g
        gU = [None, None]
        ugrp = arena.group_view([U_f, U_b], "grad") if (arena is not None and d1) else None
        if ugrp is not None and arena.first_write(U_f) and arena.first_write(U_b):
            # both directions' dU_d = dgh_d^T h_d as ONE batched GEMM into the packed slots
            sch = arena.wgrad
            on_side = x16.is_cuda and sch.on_side(x16.device)
            grouped = sch.grouped and on_side
            defer = sch.defer_input and on_side and (ctx.idx >= 1 or grouped) and _defer_layer(plan, x16.device, ctx.idx, T)
            beside = ctx.idx > 0 and not defer            # runs beside the next layer's BPTT
            splits = _DU_SPLITS if beside else None
            cap_u = (_beside_grid(plan, x16.device, not sch.defer_input, bool(getattr(ctx, "fp8_bwd", False)))
                     if (beside and on_side) else 0)
            if cap_u and (_DU_UNCAP == "all" or (_DU_UNCAP == "low" and ctx.idx == (
                    _upper_trigger(plan, x16.device, T) if sch.defer_input else 1))):
                cap_u = 0

            steps = dgh.shape[1]
            g3 = dgh.view(2, steps * plan.NP, GH).transpose(1, 2)
            h3 = hx[:, :steps].reshape(2, steps * plan.NP, plan.H)
            out = ugrp.view(2, GH, plan.H)

            def du_done(U_f=U_f, U_b=U_b):
                arena.grad_done(U_f, U_b)

            def du(g3=g3, h3=h3, out=out, splits=splits, cap=cap_u):
                if not (GM.enabled("wgrad") and GM.matmul(g3, h3, out, splits=splits, max_grid=cap)):
                    try:
                        torch.bmm(g3, h3, out_dtype=torch.float32, out=out)
                    except (RuntimeError, TypeError):
                        out.copy_(torch.bmm(g3, h3))
                du_done()
            carry_from = (_upper_trigger(plan, x16.device, T) + 1) if sch.carry_du else 0
            if beside and on_side and carry_from and ctx.idx >= carry_from and cap_u:
                # carried into the NEXT step's forward (Trainer defer_update): the GEMM runs on
                # the side stream beside a forward recurrence, right before this layer's carried
                # optimizer chunk, so only dW runs beside the next BPTT (dW + dU outlasted it by
                # ~140 us, which landed on the next dx GEMM). The slots count as written now
                # (no zeroing; first write overwrites) and the operands stay referenced.
                arena.mark_written(U_f, U_b)

                def du_carried(grid, g3=g3, h3=h3, out=out, hold=(dgh, hx)):
                    sch.hold(*hold)
                    if not (GM.enabled("wgrad") and GM.matmul(g3, h3, out, splits=_DU_SPLITS, max_grid=grid)):
                        torch.bmm(g3, h3, out_dtype=torch.float32, out=out)
                sch.carried_du[ctx.idx] = du_carried
            elif defer:
                # every weight gradient after the BPTT chain: a GEMM beside the latency-bound
                # persistent BPTT slows it by 27-48 % (its L2 / fabric / clock share), more
                # than the tail gains back (WgradScheduler)
                ops = [GM.group_operands(g3[d], h3[d], out[d]) for d in range(2)] if grouped else None
                members = [o + (out[d],) for d, o in enumerate(ops)] if ops and all(ops) else None
                sch.deferred.append(Deferred(du, (dgh, hx), members, du_done))
                arena.hold_report(U_f, U_b)
                sch.queue_end_of_backward()
            elif sch.defer_input and on_side and ctx.idx == 0 and _defer_wgrad(plan, x16.device):
                # the side stream already carries dW_0 + every deferred dW and ends after the
                # conv front-end's backward on the main stream: balance by issuing the
                # bottom layer's dU on the main stream behind the front-end (WgradScheduler.join)
                sch.main_tail.append(du)
                arena.hold_report(U_f, U_b)
                sch.queue_end_of_backward()
            else:
                du()
        else:
            for d, p in enumerate([U_f, U_b] if d1 else [U_f]):
                g = _dU(dgh, hx, d, plan, p)
                if g is None:
                    arena.grad_done(p)
                gU[d] = g
        tail = ctx.idx == 0 and arena is not None and arena.wgrad.grouped and x16.is_cuda and \
            arena.wgrad.on_side(x16.device)
        if tail:
            arena.wgrad.flush()             # the bottom layer: every deferred GEMM in one group
        jobs = [([b_f, b_b] if d1 else [b_f], parts[0])]
        if parts.shape[0] > 1:
            jobs.append(([bh_f, bh_b] if d1 else [bh_f], parts[1]))
        sums = _bias_grads_multi(jobs)
        gb = sums[0]
        gbh = sums[1] if parts.shape[0] > 1 else [None, None]
        if tail:
            arena.wgrad.run_early_update()  # the recurrent stack's optimizer range, beside the front-end
        elif (ctx.idx >= 1 and ctx.idx == _upper_trigger(plan, x16.device, T) and arena is not None and x16.is_cuda and
              arena.wgrad.defer_input and arena.wgrad.on_side(x16.device)):
            arena.wgrad.run_early_upper(ctx.idx)   # layers >= idx and the head, beside the next BPTT
        return (dx, None, None, None, None, None, gW[0], gW[1], gU[0], gU[1], gb[0], gb[1], gbh[0], gbh[1], None)


# A layer's weight gradients are deferred to the grouped tail launch only when its BPTT leaves
# fewer than this many CUs idle; with more, they run beside the next layer's BPTT on the side
# stream. Measured (same box, bench.py): headline (BPTT 200 of 256 CUs) deferral kept;
# 7 x BiGRU-1280 (160 CUs, 96 idle) 23.10 ms/step beside vs 24.53 deferred; 7 x bi-ReLU-1760
# (generation-1 kernels) 20.95 deferred vs 21.64 beside.
_BESIDE_MIN_IDLE_CUS = 96
# weight-gradient GEMMs issued beside a later layer's BPTT (data parallelism, or wide layers
# that leave >= _BESIDE_MIN_IDLE_CUS idle) run on a grid of at most the CUs the persistent BPTT
# leaves idle, so that they fill the idle CUs instead of queueing workgroups behind the BPTT's:
# with data parallelism and beside the fp8 BPTT (-1, the default), always (-2), at most
# _BESIDE_GRID workgroups (> 0), or never (0). Same box, alternating rounds
# (scripts/ab_dp.sh, scripts/ab_beside.sh):
#   headline, DP machinery at world 1: plain 7.731 / 7.745 / 7.739 ms/step; whole chip 7.821 /
#     7.809 / 7.822 (+1.1 %); idle CUs (56) 7.788 / 7.770 / 7.773 (+0.5 %); 32: 9.13-9.21
#   config 5 fp8: idle CUs (96) 18.13 / 18.14, whole chip 18.50 / 18.29
#   config 5 bf16: idle CUs 23.37 / 23.42, whole chip 23.16 / 23.18 (kept uncapped)
_BESIDE_GRID = -1
_BESIDE_SPARE_PER_XCD = 2


# bottom layer: the grouped launch before layer 0's dx GEMM (same-box A/B, 3 rounds: 8.025 /
# 8.028 / 8.081 vs 8.091 / 8.024 / 8.101 ms/step after it)
_GROUP_BEFORE_DX = True


def _bptt_cus(plan: RnnPlan) -> int:
    """CUs the persistent BPTT of ``plan`` occupies (one workgroup per CU)."""
    if plan.kind == "xcd":
        return plan.ndir * plan.BG * _xcd_p(plan.H, plan.cell)
    return plan.ndir * plan.BG * plan.S if plan.persistent else 1 << 30


# with deferral, only the bottom _defer_layers() layers' weight gradients join the grouped tail
# launch; the layers above run theirs beside the next BPTT, on the CUs it leaves idle
# (_beside_grid), and their optimizer range goes out once the lowest of them has issued its
# gradients. Round 4, beside GEMMs on the whole chip: all deferred 8.101 / 8.076 ms/step, bottom
# 1 8.125 / 8.115 (the BPTT chain grew by what the tail lost: shared L2 / fabric). Round 5, the
# beside GEMMs capped to the BPTT's 56 idle CUs, same box, 3 rounds each on two boxes: all
# deferred 7.696-7.723 / 7.709-7.717, bottom 1 7.652-7.653 / 7.578-7.599, bottom 2 7.627-7.693,
# bottom 0 7.593-7.605; a 48-workgroup cap 8.49-8.54 (the GEMMs outlast the BPTT). Plans whose
# BPTT leaves fewer than _PARTIAL_MIN_IDLE CUs (ReLU-1760: 32) keep everything deferred, and so do
# sequences shorter than _PARTIAL_MIN_T recurrence steps: per-length eager A/B (same box, 2
# rounds, tools/host_overhead.py, ms/step bottom-1 vs all deferred): 400 frames 3.62 vs 3.41,
# 600 4.88 vs 4.79, 800 6.14 vs 6.22, 1000 7.64 vs 7.74, 1500 11.36 vs 11.68; a second box:
# 700 5.67-5.68 vs 5.60-5.64, 800 6.24-6.29 vs 6.30-6.31 -- over a short BPTT the beside GEMMs
# cannot hide and the split tail loses its one-launch efficiency; the cut sits past 800 frames
# (191 steps).
# _DEFER_LAYERS >= 0 forces a count (tests).
_DEFER_LAYERS = -1
_PARTIAL_MIN_IDLE = 56
_PARTIAL_MIN_T = 200


_FULL = 1 << 30            # "every layer" / "no cap" sentinel of the schedule fields


@dataclass(frozen=True)
class StepSchedule:
    """Where and when one recurrent stack's weight-gradient GEMMs and optimizer ranges run in a
    training step, for one recurrence plan on one chip (every threshold below is a measured
    choice; the comments above each constant give the A/B). Produced by :func:`schedule_for`.

    bptt_cus       CUs the persistent BPTT (and forward) recurrence occupies
    idle_cus       CUs it leaves idle (num_cus - bptt_cus)
    defer_wgrad    single device: weight gradients go to the grouped tail launch after the last
                   BPTT (the BPTT leaves < _BESIDE_MIN_IDLE_CUS idle), not beside each BPTT
    defer_layers   bottom layers whose weight gradients join that grouped launch (_FULL: all)
    upper_trigger  layer whose issued weight gradients complete the head + every layer above
                   it (their optimizer range, or the carried update of Trainer defer_update)
    beside_grid    grid cap of weight-gradient GEMMs issued beside a BPTT (0: uncapped)
    carry_grid     block cap of a carried optimizer chunk beside a forward recurrence (0: none)
    group_cap      grid cap of the grouped tail launch
    """
    bptt_cus: int
    idle_cus: int
    defer_wgrad: bool
    defer_layers: int
    upper_trigger: int
    beside_grid: int
    carry_grid: int
    group_cap: int

    def defer_layer(self, idx: int) -> bool:
        return self.defer_wgrad and idx < self.defer_layers


def schedule_for(plan: RnnPlan, T: int, dp: bool, fp8: bool, num_cus: int) -> StepSchedule:
    """The step schedule of a recurrence plan at T recurrence steps: data parallel or not, fp8
    BPTT or not, on a chip of ``num_cus`` CUs (``num_cus`` <= 0: no GPU, everything deferred)."""
    if num_cus <= 0:
        layers = _FULL if _DEFER_LAYERS < 0 else _DEFER_LAYERS
        return StepSchedule(0, 0, True, layers, layers, 0, 0, 0)
    bptt = _bptt_cus(plan)
    idle = num_cus - bptt
    defer = idle < _BESIDE_MIN_IDLE_CUS
    if _DEFER_LAYERS >= 0:
        layers = _DEFER_LAYERS
    else:
        layers = 1 if idle >= _PARTIAL_MIN_IDLE and T >= _PARTIAL_MIN_T else _FULL
    beside = 0
    if _BESIDE_GRID != 0 and (_BESIDE_GRID != -1 or dp or fp8 or defer):
        cap = idle if _BESIDE_GRID < 0 else min(_BESIDE_GRID, idle)
        if (_BESIDE_GRID < 0 and not dp and ((defer and layers == 1) or fp8) and
                cap > 8 * _BESIDE_SPARE_PER_XCD):
            # single device: the GEMMs beside a BPTT leave 2 of each XCD's idle CUs free.
            # Headline (partial deferral: the upper layers' dW, 5 of 7 per XCD): 7.280-7.307 vs
            # 7.315-7.338 ms/step (4 rounds; another box 7.26-7.305 vs 7.296-7.324); 6 of 7
            # measured 7.445-7.459, 4 of 7: 7.318-7.322. Config 5 fp8 (10 of 12): 17.17-17.21 vs
            # 17.30-17.31, 8 of 12: 17.28. Data parallel keeps every idle CU (headline 7.607-7.62
            # at 5 of 7 vs 7.547-7.548) (scripts/r6_beside*.sh)
            cap -= 8 * _BESIDE_SPARE_PER_XCD
        beside = max(8, cap // 8 * 8)
    carry = idle // 8 * 8 if (plan.kind == "xcd" and idle >= 16) else 0
    group = _GROUP_CAP or (3 * num_cus) // 4
    return StepSchedule(bptt, idle, defer, layers, layers if defer else 1, beside, carry, group)


def _cus(device: torch.device) -> int:
    return _ext.num_cus(device.index or 0) if device.type == "cuda" else 0


def _beside_grid(plan: RnnPlan, device: torch.device, dp: bool, fp8: bool) -> int:
    return schedule_for(plan, 0, dp, fp8, _cus(device)).beside_grid


def _idle_cus(plan: RnnPlan, device: torch.device) -> int:
    """Block cap for work beside this plan's persistent recurrence (schedule ``carry_grid``)."""
    return schedule_for(plan, 0, False, False, _cus(device)).carry_grid


def _defer_wgrad(plan: RnnPlan, device: torch.device) -> bool:
    return schedule_for(plan, 0, False, False, _cus(device)).defer_wgrad


def _defer_layers(plan: RnnPlan, device: torch.device, T: int) -> int:
    """How many of the bottom layers defer their weight gradients to the grouped tail launch
    at recurrence length ``T`` (everything deferred: 1 << 30)."""
    return schedule_for(plan, T, False, False, _cus(device)).defer_layers


def _defer_layer(plan: RnnPlan, device: torch.device, idx: int, T: int) -> bool:
    return schedule_for(plan, T, False, False, _cus(device)).defer_layer(idx)


def _upper_trigger(plan: RnnPlan, device: torch.device, T: int) -> int:
    """Layer whose issued weight gradients complete the head + every layer above it."""
    return schedule_for(plan, T, False, False, _cus(device)).upper_trigger


class Deferred:
    """A deferred weight-gradient GEMM: ``fn`` runs it (and reports the gradient) on the
    current stream; ``members`` are its (A, B, out) stored column-mode operands for a grouped
    launch (None: not groupable), after which ``done`` reports the gradient."""
    __slots__ = ("fn", "tensors", "members", "done")

    def __init__(self, fn, tensors, members=None, done=None):
        self.fn, self.tensors, self.members, self.done = fn, tensors, members, done


class WgradScheduler:
    """Where and when one parameter arena's weight-gradient GEMMs run.

    Owned by the :class:`~deepspeech_amd.ops.optim.ParamArena` whose gradients it produces
    (``arena.wgrad``), so two trainers / models in one process (training beside eval or
    streaming, two Trainers in a test) never share a side stream, a deferral switch or a
    queue of pending GEMMs (this state used to be module-global).

    * ``stream(device)``: side stream for the recurrent layers' (and head's / front-end's)
      weight-gradient GEMMs (``single_stream`` keeps them on the current stream). The
      Trainer joins it (:meth:`join`) before the optimizer reads the gradients.
    * Single device (``set_deferral``): every recurrent layer's weight gradients (dW = dgx^T x
      and both directions' dU = dgh^T h) are deferred until the bottom layer's BPTT has been
      issued, and then run as one grouped gemm8 launch on the side stream, beside the conv
      front-end's backward. A GEMM beside the latency-bound persistent BPTT slowed it by
      27-48 % (its L2 / fabric / clock share), more than the overlap gained back. With data
      parallelism deferral would hold every recurrent gradient bucket back to the end of
      backward, so the Trainer enables it for world_size == 1 only (DS2_DEFER_DW=0/1
      overrides); the GEMMs then run per layer on the side stream as each BPTT finishes.
    * ``set_early_update``: the optimizer range of the parameters that are final once the
      grouped launch is issued runs on the side stream right behind it.
    * ``set_fused_update``: the grouped launch applies Adam + EMA to its members' elements in
      its epilogue (csrc/gemm8.hip) instead of storing their gradients; ``fused_ranges`` then
      lists the arena element ranges already updated this step, which every later optimizer
      range of the step skips.
    """

    def __init__(self):
        self.streams = {}
        self.defer_input = False
        # every deferred weight gradient of the backward (all layers' dW and dU) as ONE grouped
        # gemm8 launch after the bottom layer's BPTT (GM.gemm8_group): one grid over all their
        # tiles (measured tail, tools/bench_gemm8.py: 0.84 / 1.96 / 1.32 ms for the headline /
        # config 5 / 7 x ReLU-1760 vs 1.42 / 2.94 / 2.32 as one hipBLASLt call each); without
        # it (DS2_GEMM=torch) the GEMMs of layers >= 1 are issued one by one after that BPTT
        self.grouped = GM.enabled("wgrad")
        self.deferred = []
        self.main_tail = []        # GEMMs issued on the main stream once the whole backward is queued
        self._eob_queued = False
        self._early = None         # (fn, params, main stream): set_early_update
        self.early_done = False
        self._early_upper = None   # (ranger, fn, main stream, grid): the layers run beside the BPTT
        self.early_upper_done = False
        self.early_upper_hi = 0
        self.transposes = []       # queued W^T shadows of this forward (_transpose_async)
        self._t_events = {}        # device -> event of the last transposes flush
        self._t_waited = set()     # streams that waited for it
        self._hold = []            # tensors read on the side stream, released by join()
        self._fused = None         # (arena, tensors, constants, store_g): set_fused_update
        self.fused_ranges = []     # arena element ranges the grouped epilogue updated this step
        # Trainer defer_update (carry_du): the recurrent layers above the upper trigger hand their
        # beside dU GEMM to the next step's forward (carried_du: layer -> fn(grid), taken by the
        # Trainer with take_carried_du; whatever is not taken runs before this step's optimizer)
        self.carry_du = False
        self.carried_du = {}
        # every weight gradient on the current stream (a captured step graph: ROCm replays a
        # graph's cross-stream edges as barrier packets between its queues)
        self.single_stream = False
        _schedulers.add(self)

    def stream(self, device: torch.device) -> Optional["torch.cuda.Stream"]:
        if device.type != "cuda" or self.single_stream:
            return None
        idx = device.index if device.index is not None else torch.cuda.current_device()
        s = self.streams.get(idx)
        if s is None:
            s = torch.cuda.Stream(device=torch.device("cuda", idx))
            self.streams[idx] = s
        return s

    def on_side(self, device: torch.device) -> bool:
        """True when the current stream is this arena's weight-gradient side stream (the step
        itself may run on a non-default, high-priority main stream)."""
        idx = device.index if device.index is not None else torch.cuda.current_device()
        s = self.streams.get(idx)
        return s is not None and torch.cuda.current_stream(idx) == s

    def set_deferral(self, on: bool) -> None:
        env = os.environ.get("DS2_DEFER_DW")
        self.defer_input = (env == "1") if env in ("0", "1") else bool(on)

    def discard(self) -> None:
        """Drop deferred GEMMs of an aborted backward (called at the start of a step)."""
        if self._hold:
            if not self.single_stream:
                for idx, s in self.streams.items():
                    _stream_wait(torch.cuda.current_stream(idx), s)
            self._hold.clear()
        self.deferred.clear()
        self.main_tail.clear()
        self._eob_queued = False
        self._early = None
        self.early_done = False
        self._early_upper = None
        self.early_upper_done = False
        self.early_upper_hi = 0
        self.transposes.clear()
        self._fused = None
        self.fused_ranges = []
        self.carried_du = {}

    def flush_transposes(self) -> None:
        """Issue the queued W^T transposes on the side stream behind everything the current
        stream has enqueued (the recurrences whose weights they read were issued before)."""
        if not self.transposes:
            return
        jobs, self.transposes = self.transposes, []
        C = _ext.ext()
        cur = torch.cuda.current_stream(jobs[0].W16.device)
        side = jobs[0].side
        _stream_wait(side, cur)
        with torch.cuda.stream(side):
            for j in jobs:
                self.hold(j.W16, j.wT)
                C.transpose_bf16(j.W16, j.wT)
        # one event for the whole flush, waited once per consumer stream (wait_transposes)
        idx = side.device.index
        ev = self._t_events.get(idx)
        if ev is None:
            ev = self._t_events[idx] = int(C.event_new(0))
        C.event_record(ev, side.cuda_stream)
        self._t_waited = set()
        for j in jobs:
            j.event = ev

    def wait_transposes(self, stream, ev) -> None:
        """Make ``stream`` wait for the flushed W^T transposes (once per flush and stream)."""
        if stream.cuda_stream in self._t_waited:
            return
        _ext.ext().event_wait(stream.cuda_stream, ev)
        self._t_waited.add(stream.cuda_stream)

    def hold(self, *tensors) -> None:
        """Keep tensors that side-stream work reads alive until join() has made the current
        stream wait for the side stream, instead of record_stream: the caching allocator
        records an event on the side stream for every such tensor it frees, and three of
        those landing behind the grouped weight-gradient launch held the optimizer range
        back by 80-85 us per step (tools/probe_event_gap.py: ~6 us per record alone)."""
        if len(self._hold) > 512 and all(torch.cuda.current_stream(i) != st for i, st in self.streams.items()):
            # a loop that never joins (bare loss.backward() without join_wgrad_streams): bound
            # what is held by ordering the current stream after the side stream and letting go
            for idx, st in self.streams.items():
                _stream_wait(torch.cuda.current_stream(idx), st)
            self._hold.clear()
        self._hold.extend(t for t in tensors if t is not None)

    def set_early_upper(self, ranger, fn, grid: int = 0) -> None:
        """For THIS backward: once the lowest layer b whose weight gradients run beside the
        BPTT (not deferred to the grouped tail launch) has issued them, every parameter of the
        head and of layers >= b is final: ``ranger(b)`` gives that arena range as (end, params)
        and ``fn(end, grid)`` runs its optimizer update on the side stream, beside layer b-1's
        BPTT on the CUs it leaves idle. The lower range (set_early_update) then starts at
        ``early_upper_hi``."""
        self._early_upper = (ranger, fn, torch.cuda.current_stream(), grid)
        self.early_upper_done = False

    def run_early_upper(self, b: int) -> None:
        if self._early_upper is None:
            return
        ranger, fn, main, grid = self._early_upper
        r = ranger(b)
        if r is None:
            return
        self._early_upper = None
        hi, params = r
        arena = arena_of(params[0]) if params else None
        if arena is None or any(arena.first_write(p) for p in params):
            return
        _stream_wait(torch.cuda.current_stream(), main)   # readers of the weights issued so far
        fn(hi, grid)
        self.early_upper_hi = hi
        self.early_upper_done = True

    def set_early_update(self, fn, params) -> None:
        """For THIS backward: once the bottom recurrent layer has issued its weight gradients
        (the grouped tail launch and its bias sums, on the side stream), run ``fn()`` — the
        optimizer update of the parameters whose gradients are then final (FC head and the
        recurrent stack) — on that side stream, behind the main stream's work issued so far,
        so it runs beside the conv front-end's backward instead of after it. Skipped (the
        caller updates everything afterwards; ``early_done`` stays False) if any of ``params``
        has not been written by then. Call on the stream that runs the backward."""
        self._early = (fn, params, torch.cuda.current_stream())
        self.early_done = False

    def run_early_update(self) -> None:
        if self._early is None:
            return
        fn, params, main = self._early
        self._early = None
        arena = arena_of(params[0]) if params else None
        if arena is None or any(arena.first_write(p) for p in params):
            return
        _stream_wait(torch.cuda.current_stream(), main)   # readers of the weights issued so far
        self._run_carried()                # dU GEMMs nobody carried: before their optimizer range
        fn()
        self.early_done = True

    def _run_carried(self) -> None:
        for k in sorted(self.carried_du, reverse=True):
            self.carried_du[k](0)
        self.carried_du = {}

    def set_fused_update(self, arena, tensors, constants, store_g: bool = False) -> None:
        """For THIS backward: the grouped tail launch applies the optimizer to its members'
        elements in its epilogue (tensors / constants as gemm.gemm8_group's ``opt``)."""
        self._fused = (arena, list(tensors), list(constants), bool(store_g))
        self.fused_ranges = []

    def _fused_opt(self, members):
        """gemm8_group ``opt`` for these members, or None when the epilogue cannot take them
        (not all contiguous, 16-B aligned first-write views of this arena's gradient buffer)."""
        if self._fused is None:
            return None
        arena, tensors, constants, store_g = self._fused
        g = arena.grad
        base, n = g.data_ptr(), g.numel()
        ranges = []
        for _, _, out in members:
            e0 = (out.data_ptr() - base) // 4
            if (out.dtype != torch.float32 or not out.is_contiguous() or (out.data_ptr() - base) % 16 or
                    e0 < 0 or e0 + out.numel() > n or out.shape[-1] % 4):
                return None
            ranges.append((e0, e0 + out.numel()))
        return (tensors, constants, store_g), ranges

    def flush(self) -> None:
        """Issue every deferred weight-gradient GEMM on the current stream: one grouped launch
        when every one of them can join it, else one call each."""
        if self.deferred and self.grouped and all(isinstance(d, Deferred) and d.members for d in self.deferred):
            items, self.deferred = self.deferred, []
            members = [m for d in items for m in d.members]
            fused = self._fused_opt(members)
            # the grouped launch on 3/4 of the CUs: the conv front-end's backward beside it
            # (LDS-bound kernels that cannot share a CU with a group workgroup's 128 KB) gets
            # the rest; headline, same box: 7.83-7.87 ms/step vs 7.89-7.90 on every CU, 7.94
            # at 176, 7.84-7.92 at 208, 8.03 at 128
            cap = _GROUP_CAP or (3 * _ext.num_cus(torch.cuda.current_device())) // 4   # schedule group_cap
            if fused is not None:
                GM.gemm8_group(members, opt=fused[0], max_grid=cap)
                self.fused_ranges.extend(fused[1])
            else:
                GM.gemm8_group(members, max_grid=cap)
            for d in items:
                d.done()
            return
        while self.deferred:
            item = self.deferred.pop(0)
            (item.fn if isinstance(item, Deferred) else item)()

    def take_carried_du(self) -> dict:
        """The carried dU GEMMs of this backward (layer -> fn(grid)); the caller runs each before
        that layer's optimizer update."""
        c, self.carried_du = self.carried_du, {}
        return c

    def drain(self) -> None:
        """Issue every deferred weight-gradient GEMM: leftover input-weight GEMMs (a backward
        that never reached layer 0) on the side stream, then the main-stream tail (the bottom
        layer's dU behind the front-end backward). Carried dU GEMMs nobody took run here."""
        if self.carried_du:
            for idx, s in self.streams.items():
                _stream_wait(s, torch.cuda.current_stream(idx))
                with torch.cuda.stream(s):
                    self._run_carried()
            self._run_carried()
        if self.deferred:
            for idx, s in self.streams.items():
                _stream_wait(s, torch.cuda.current_stream(idx))
                with torch.cuda.stream(s):
                    self.flush()
            self.flush()
        while self.main_tail:
            self.main_tail.pop(0)()

    def queue_end_of_backward(self) -> None:
        """Drain the deferred GEMMs when the running backward finishes, whoever drives it
        (Trainer.step, a bare loss.backward(), the --debug profiler): autograd runs final
        callbacks on the caller's current streams once the whole graph has been executed,
        so no gradient is left unwritten (lazy zeroing would otherwise keep a stale value)."""
        if self._eob_queued:
            return
        self._eob_queued = True

        def cb():
            self._eob_queued = False
            self.drain()
        try:
            torch.autograd.Variable._execution_engine.queue_callback(cb)
        except RuntimeError:              # not inside a backward: drained by join()
            self._eob_queued = False

    def pending(self) -> int:
        """Number of weight-gradient GEMMs still waiting to be issued (0 after a backward)."""
        return len(self.deferred) + len(self.main_tail)

    def join(self) -> None:
        """Make the current stream wait for every pending side-stream weight gradient."""
        self.drain()
        if not self.single_stream:
            for idx, s in self.streams.items():
                _stream_wait(torch.cuda.current_stream(idx), s)
        self._hold.clear()           # frees on the current stream, ordered after the side work


_schedulers = weakref.WeakSet()


def wgrad_stream(device: torch.device, arena=None) -> Optional["torch.cuda.Stream"]:
    """The weight-gradient side stream of ``arena`` (None without an arena: plain autograd
    gradients are returned to autograd on the current stream)."""
    return arena.wgrad.stream(device) if arena is not None else None


def flush_transposes() -> None:
    """Issue every live arena's queued W^T transposes (the model calls this after its
    recurrent stack, before the head and the loss)."""
    for sch in list(_schedulers):
        sch.flush_transposes()


def join_wgrad_streams(arena=None) -> None:
    """Join ``arena``'s weight-gradient work (every live arena's when None: tests and tools
    that drive a bare ``loss.backward()``)."""
    for sch in ([arena.wgrad] if arena is not None else list(_schedulers)):
        sch.join()


def pending_deferred(arena=None) -> int:
    return sum(sch.pending() for sch in ([arena.wgrad] if arena is not None else list(_schedulers)))


_plan_cache = {}


def plan_for(N: int, H: int, cell: str, ndir: int, device: torch.device) -> RnnPlan:
    key = (N, H, cell, ndir, device.index, os.environ.get("DS2_RNN_MODE"), _FORCE_NW, _MIN_ROWS)
    p = _plan_cache.get(key)
    if p is None:
        check_knobs()
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
        gx = _linear(x2, W, b, sbn_scale())
    elif layer.seq_bn == "none":
        gx = _linear(x2, W, b, 1.0)
    else:
        y = _linear(x2, W, None, 1.0).view(T, N, -1)
        outs = []
        GH = dirs[0].W.shape[0]
        for i, d in enumerate(dirs):
            outs.append(R.seq_batch_norm(y[..., i * GH:(i + 1) * GH], lens, "batch", d.sbn_mean,
                                         d.sbn_var, layer.training))
        gx = (torch.cat(outs, -1) + b).reshape(T * N, -1)
    return gx.view(T, N, -1)


@torch.no_grad()
def recurrent_layer_infer(layer, x: torch.Tensor, lens: torch.Tensor, h0: Optional[torch.Tensor] = None,
                          h_out: Optional[torch.Tensor] = None):
    """Inference-only layer with state carry: returns (y [T, N, H], h_last [ndir, N, H] fp32).
    h_last holds each row's state after its last valid step (the kernels freeze the state
    past an utterance's length), which is what a streaming caller carries to the next chunk;
    with h_out ([ndir, N, H] fp32) it is written there (one copy) and h_out is returned."""
    ndir = 2 if layer.bw is not None else 1
    T, N, _ = x.shape
    plan = plan_for(N, layer.hidden, layer.cell, ndir, x.device)
    dirs = layer.directions()
    # bf16 operand copies are cached per layer and rebuilt only when a parameter changed
    # (its version counter moves with every in-place update): a streaming chunk no longer
    # re-casts W and U on every call
    params = [p for d in dirs for p in (d.W, d.b, d.U, d.b_h) if p is not None]
    key = (x.device, tuple(p._version for p in params), tuple(p.data_ptr() for p in params))
    cache = getattr(layer, "_infer_cache", None)
    if cache is None or cache[0] != key:
        with torch.no_grad():
            cache = (key,
                     torch.cat([d.W for d in dirs], 0).to(torch.bfloat16),
                     torch.cat([d.b for d in dirs], 0).to(torch.bfloat16),
                     [d.U.to(torch.bfloat16).contiguous() for d in dirs] + ([None] if ndir == 1 else []),
                     [d.b_h.float().contiguous() if d.b_h is not None else None for d in dirs]
                     + ([None] if ndir == 1 else []))
        layer._infer_cache = cache
    _, W16, b16, U, bh = cache
    alpha = sbn_scale() if layer.seq_bn == "frozen" else 1.0
    if layer.seq_bn == "batch":
        gx = input_projection_hip(layer, x.to(torch.bfloat16), lens)
    else:
        gx = _linear(x.to(torch.bfloat16).reshape(T * N, -1), W16, b16, alpha).view(T, N, -1)
    lens = lens.to(device=x.device, dtype=torch.int32).contiguous()
    y, (hx, hs, gates) = _run_fwd(gx.contiguous(), lens, U, bh, plan, h0=h0)
    if h_out is not None:
        h_out.copy_(hs[:, T, :N])
        return y, h_out
    return y, hs[:, T, :N].clone()


def recurrent_layer_hip(layer, x: torch.Tensor, lens: torch.Tensor, idx: int = 0,
                        pair_out: bool = False) -> torch.Tensor:
    """One recurrent layer on the HIP engine. x: [T, N, D], or the [2, T, N, D] direction pair
    of an fp8 layer below (pairs_ok). pair_out: return this layer's fp8 direction outputs as
    such a pair when it has them (the caller feeds them to an fp8 layer), else the sum."""
    with TR.phase(TR.rnn_cell(idx)):
        return _recurrent_layer_hip(layer, x, lens, idx, pair_out)


# grid cap of the grouped tail launch (0: 3/4 of the CUs)
_GROUP_CAP = 0
# The lowest beside layer's dU is issued behind its dW and mostly runs after the last BPTT has
# ended: on the whole chip, not the BPTT's idle CUs (capped it took 381 us on 56 CUs while the
# tail's side stream waited for it). Same box, 3 rounds: 7.560 / 7.583 / 7.595 vs capped 7.609 /
# 7.601 / 7.609 ms/step (an uncapped grouped tail launch on top: no further gain).
# "none": capped; "all": every beside layer's dU uncapped (A/B: 7.639 / 7.695 / 7.690 vs 7.535 /
# 7.554 / 7.563 ms/step for "low": an upper layer's dU then waits for the BPTT's CUs and lands
# on the next dx GEMM and BPTT)
_DU_UNCAP = "low"

# False: every fp8 layer sums its directions with torch.add (A/B timing)
_FP8_PAIRS = True


def pairs_ok(layer) -> bool:
    """layer takes the unsummed direction pair of the layer below (FusedBiLayer's fp8 form)."""
    return _FP8_PAIRS and bool(getattr(layer, "fp8", False)) and layer.seq_bn in ("frozen", "none")


def _recurrent_layer_hip(layer, x: torch.Tensor, lens: torch.Tensor, idx: int, pair_out: bool = False) -> torch.Tensor:
    ndir = 2 if layer.bw is not None else 1
    plan = plan_for(x.shape[-2], layer.hidden, layer.cell, ndir, x.device)
    fw, bw = layer.fw, layer.bw
    if layer.seq_bn in ("frozen", "none"):
        alpha = sbn_scale() if layer.seq_bn == "frozen" else 1.0
        return FusedBiLayer.apply(x, lens, plan, alpha, idx, bool(getattr(layer, "fp8", False)),
                                  fw.W, bw.W if bw is not None else None,
                                  fw.U, bw.U if bw is not None else None,
                                  fw.b, bw.b if bw is not None else None,
                                  fw.b_h, bw.b_h if bw is not None else None, pair_out)
    if x.dim() == 4:
        x = x[0] + x[1]
    x = x.to(torch.bfloat16)
    gx = input_projection_hip(layer, x, lens)
    U_f = fw.U.to(torch.bfloat16)
    U_b = bw.U.to(torch.bfloat16) if ndir == 2 else None
    bh_f = fw.b_h if layer.cell == "gru" else None
    bh_b = bw.b_h if (layer.cell == "gru" and ndir == 2) else None
    return BiRecurrence.apply(gx, lens, U_f, U_b, bh_f, bh_b, plan)


def _uni_layer_hip(layer, d, x: torch.Tensor, lens: torch.Tensor, idx: int) -> torch.Tensor:
    """One direction of a layer as a one-direction fused layer over x (forward in time)."""
    plan = plan_for(x.shape[1], layer.hidden, layer.cell, 1, x.device)
    if layer.seq_bn in ("frozen", "none"):
        alpha = sbn_scale() if layer.seq_bn == "frozen" else 1.0
        return FusedBiLayer.apply(x, lens, plan, alpha, idx, bool(getattr(layer, "fp8", False)),
                                  d.W, None, d.U, None, d.b, None, d.b_h, None)
    gx = layer.input_projection_ref(x.to(torch.bfloat16), d, lens).to(torch.bfloat16)
    bh = d.b_h if layer.cell == "gru" else None
    return BiRecurrence.apply(gx, lens, d.U.to(torch.bfloat16), None, bh, None, plan)


def recurrent_layer_split_hip(layer, x_f: torch.Tensor, x_b: torch.Tensor, lens: torch.Tensor, idx: int = 0):
    """Per-direction stacks of the NHWC graph (src/deepSpeech.py:165-185, two MultiRNNCells
    under bidirectional_dynamic_rnn): the forward direction of layer idx reads the forward
    stack, the backward direction the backward stack, and the outputs stay separate. The
    backward direction runs as a forward recurrence over the length-aware reversal of its
    input (TF ReverseSequence semantics, ops/reference.py reverse_sequence)."""
    with TR.phase(TR.rnn_cell(idx)):
        lens = lens.to(device=x_f.device, dtype=torch.int32)
        y_f = _uni_layer_hip(layer, layer.fw, x_f, lens, idx)
        xr = R.reverse_sequence(x_b, lens)
        y_b = R.reverse_sequence(_uni_layer_hip(layer, layer.bw, xr, lens, idx), lens)
        return y_f, y_b
