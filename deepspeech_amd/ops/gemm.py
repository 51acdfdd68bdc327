"""Python front for the hand-written MFMA GEMM family (csrc/gemm.hip).

Every GEMM of a recurrent layer runs here on the HIP engine (reference call sites
src/custom_ops.py:59-67 for W.x / U.h, src/deepSpeech_NCHW.py:188-198 for the FC):

  linear(x, W, b, alpha)   gx = alpha * x W^T + b            bf16 out (forward projection)
  mm_nn(a, b)              a [M,K] . b [K,N]                  bf16 out (input gradient dx = dgx W)
  mm_tn(a, b, out, acc)    a^T . b, a [K,M], b [K,N]          fp32 into ``out`` (weight gradients),
                           batched over a leading dim          ``acc`` adds instead of overwriting

Tile choice: per (shape, layout) from a small table measured on MI355X
(tools/bench_gemm_ours.py), else a model that minimises the padded work of the last
dispatch round. gemm._FORCE = <0..5> forces one tile for every call (tuning only).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch

from . import _ext

# cfg -> (BM, BN, workgroups per CU); LDS = 2 stages x (BM + BN) x 64 x 2 B
_TILES = {0: (256, 256, 1), 1: (128, 256, 1), 2: (256, 128, 1), 3: (128, 128, 2), 4: (128, 128, 1),
          5: (128, 128, 1)}
# 6/7/8: persistent versions of 0/1/2 (one workgroup per CU striding over tiles, the next
# tile's loads under this tile's stores); explicit TUNED picks only (no read-modify-write)
_PERSISTENT = {6: 0, 7: 1, 8: 2}
# measured picks: (M, N, K, a_col, b_col, batch) -> cfg
TUNED: Dict[Tuple[int, int, int, bool, bool, int], int] = {
    # headline shapes (T2=241, N=32, H=800), tools/bench_gemm8.py on MI355X
    # projection, layers 1-4: on gemm8 (not listed). Alone it ties the persistent 128x256 tile
    # (82.4 vs 82.5 us); in the step, same box: 7.80-7.83 vs 7.84-7.85 ms/step (round 4)
    # dx = dgx W on the K-contiguous W^T shadow (ops/rnn.py _transpose_async), persistent
    # 128x256: 67 / 197 us vs gemm8 82 / 203 (tools/bench_gemm8.py); in the step gemm8 loses
    # too (7.90-7.94 vs 7.84-7.85 ms/step, round 4)
    (7712, 800, 4800, False, False, 1): 7,
    # layer 0's dx (7712, 2400, 4800) runs on gemm8 (non-persistent): it shares the chip with
    # the grouped weight-gradient launch, and a persistent grid's statically assigned tiles
    # then finish with its most-delayed workgroup (858-1042 us beside the group vs 234 us as
    # gemm8; 197 us alone; round 4 timeline, profiles/r4_headline.md)
    (7712, 800, 32, False, True, 1): 3,        # FC head dh (K = 32 padded classes)
}
# one csrc/gemm.hip configuration for every call (tile tuning tools set it; None in training)
_FORCE = None
# DS2_GEMM selects which engine GEMM classes run on the hand-written kernels: "hip" (all, the
# default), "torch" (none: library GEMMs, A/B timing only) or a comma list of {proj, dx, wgrad}.
_SPEC = os.environ.get("DS2_GEMM", "hip")
_CLASSES = ({"proj", "dx", "wgrad"} if _SPEC == "hip" else set() if _SPEC == "torch"
            else {c.strip() for c in _SPEC.split(",") if c.strip()})


def enabled(cls: str = "wgrad") -> bool:
    return cls in _CLASSES


def _cdiv(a: int, b: int) -> int:
    return -(-a // b)


def choose_cfg(M: int, N: int, K: int, a_col: bool, b_col: bool, batch: int = 1, cus: int = 256) -> int:
    if _FORCE is not None:
        return int(_FORCE)
    key = (M, N, K, a_col, b_col, batch)
    if key in TUNED:
        return TUNED[key]
    best, best_cost = 0, None
    for cfg, (bm, bn, per_cu) in _TILES.items():
        if (a_col and bm < 128) or (b_col and bn < 128):
            continue
        tiles = _cdiv(M, bm) * _cdiv(N, bn) * batch
        slots = cus * per_cu
        rounds = _cdiv(tiles, slots)
        # time ~ rounds x per-tile time; a tile of BMxBN on 1/per_cu of a CU takes
        # bm*bn*per_cu "units"; smaller tiles pay a staging-efficiency penalty
        eff = {0: 1.0, 1: 0.93, 2: 0.93, 3: 0.85, 4: 0.8, 5: 0.85}[cfg]
        cost = rounds * bm * bn * per_cu / eff
        if best_cost is None or cost < best_cost:
            best, best_cost = cfg, cost
    return best


def _dev_cus(t: torch.Tensor) -> int:
    return _ext.num_cus(t.device.index or 0)


def gemm(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, M: int, N: int, K: int, a_col: bool, b_col: bool,
         epi: int, alpha: float = 1.0, bias: Optional[torch.Tensor] = None, cfg: Optional[int] = None,
         alpha_dev: Optional[torch.Tensor] = None, Ml: int = 0, Nl: int = 0, Kl: int = 0, fill=None) -> torch.Tensor:
    """Raw launch. A/B are the STORED matrices (unit-stride last dim): A [M,K] (row) or
    [K,M] (col), B [N,K] (row) or [K,N] (col). alpha_dev: fp32 device scalar multiplied into
    alpha. Ml/Nl: a col-mode operand padded in memory to Ml/Nl columns; Kl: a col-mode
    operand holding only Kl k-rows (the rest must meet zeros in the other operand)."""
    batch = A.shape[0] if A.dim() == 3 else 1
    if cfg is None:
        cfg = choose_cfg(M, N, K, a_col, b_col, batch, _dev_cus(A))
        if epi != 2 and cfg in (1, 2) and _FORCE is None:
            cfg += 6        # the persistent twin: same tile, next tile's loads under the stores
    regions, pats = (list(fill[0]), list(fill[1])) if fill is not None else ([], [])
    _ext.ext().gemm(A, B, C, bias, M, N, K, a_col, b_col, epi, float(alpha), cfg, alpha_dev, Ml, Nl, Kl, regions, pats)
    return C


def supported(M: int, N: int, K: int, a_col: bool = False, b_col: bool = False) -> bool:
    return ((a_col and b_col) or K % 8 == 0) and N % 4 == 0 and (not a_col or M % 8 == 0) and \
        (not b_col or N % 8 == 0)


def linear(x2: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor] = None, alpha: float = 1.0,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """alpha * x2 @ W^T + bias; x2 [M, K], W [N, K] (bf16, unit-stride rows); bf16 [M, N]."""
    M, K = x2.shape
    N = W.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    return gemm(x2, W, out, M, N, K, False, False, 0, alpha, bias)


def mm_nn(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """a [M, K] @ b [K, N] -> bf16 [M, N]."""
    M, K = a.shape
    N = b.shape[1]
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=torch.bfloat16)
    return gemm(a, b, out, M, N, K, False, True, 0)


def _operand(t: torch.Tensor, row_if_unit_last: bool):
    """(stored matrix with a unit-stride last dim, col flag) for a logical 2-D operand, or
    None if neither dimension is unit-stride."""
    if t.stride(-1) == 1:
        return t, not row_if_unit_last
    if t.stride(-2) == 1:
        return t.transpose(-1, -2), row_if_unit_last
    return None


def matmul(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, accumulate: bool = False,
           alpha: float = 1.0, bias: Optional[torch.Tensor] = None, max_grid: int = 0,
           splits: Optional[int] = None, fill=None) -> bool:
    """out (=|+=) alpha * a @ b (+ bias) for 2-D (or batched 3-D) bf16 views of any unit-stride
    orientation: a [M, K], b [K, N]; out fp32 (store / accumulate) or bf16 (store, optional
    bias). Returns False (nothing launched) when the shape or strides are not covered.

    Routing (tools/bench_gemm8.py, MI355X): the headline's dx GEMMs keep their measured
    csrc/gemm.hip persistent tile (TUNED); every other covered shape runs on csrc/gemm8.hip —
    row-row projections, dx = dgx W with W read as stored (column-mode B), and the
    column-column weight gradients with split-K sized to the CU count.

    fill = (regions, patterns): buffers the next kernel needs initialised (multi_fill
    semantics), written by the gemm8 launch's idle workgroups, or by a multi_fill after the
    GEMM on the other paths (done whenever True is returned)."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16):
        return False
    M, K = a.shape[-2], a.shape[-1]
    N = b.shape[-1]
    oa, ob = _operand(a, True), _operand(b, False)
    if oa is None or ob is None or out.stride(-1) != 1:
        return False
    A, a_col = oa          # a [M,K] unit-stride K -> row mode (A(m,k) = A[m*lda+k])
    B, b_col = ob          # b [K,N] unit-stride N -> col mode (B(n,k) = B[k*ldb+n])
    for t in (A, B, out):
        if t.data_ptr() % 16 or (t.dim() >= 2 and t.stride(-2) % 8):
            return False
    if out.dtype == torch.bfloat16:
        if accumulate:
            return False
        epi = 0
    else:
        epi = 2 if accumulate else 1
        if bias is not None:
            return False
    batch = A.shape[0] if A.dim() == 3 else 1
    key = (M, N, K, a_col, b_col, batch)
    if _FORCE is None and key not in TUNED and _small_rowrow(M, N, K, a_col, b_col, batch, epi, a):
        gemm(A, B, out, M, N, K, a_col, b_col, epi, alpha, bias, fill=fill)
        return True
    if _FORCE is None and key not in TUNED and gemm8_supported(M, N, K, False, a_col, b_col):
        gemm8(A, B, out, epi, alpha, bias, a_col=a_col, b_col=b_col, max_grid=max_grid, splits=splits, fill=fill)
        return True
    if not supported(M, N, K, a_col, b_col):
        return False
    gemm(A, B, out, M, N, K, a_col, b_col, epi, alpha, bias, fill=fill)
    return True


# False keeps every covered shape on gemm8 (A/B timing of _small_rowrow)
_SMALL_M = True


def _small_rowrow(M: int, N: int, K: int, a_col: bool, b_col: bool, batch: int, epi: int,
                  a: torch.Tensor) -> bool:
    """Row-row bf16 GEMMs of few output tiles and short K (the projections of the short
    SortaGrad buckets) run on csrc/gemm.hip's cost-model tile: with at most cus/2 256^2 tiles
    gemm8 leaves half the chip idle, and at K <= 2400 its split-K plan does not recover that,
    while 128-row tiles fill it. tools/bench_gemm_small_m.py, MI355X (profiles/r5_gemm.md):
    projection (N 4800, K 800) at M 672: 12.8 vs 27.0 us, at 1312: 20.2 vs 28.5; (4800, 2400):
    27.3 vs 36.9 and 42.3 vs 49.7; at M 2432 (190 tiles) gemm8 wins again (30.3 vs 32.6).
    The input-gradient shapes (K 4800) keep gemm8's split-K, which wins there at every M."""
    if not _SMALL_M or a_col or b_col or epi != 0 or batch != 1 or K > 2400 or not supported(M, N, K, a_col, b_col):
        return False
    return _cdiv(M, 256) * _cdiv(N, 256) * 2 <= _dev_cus(a)


def mm_tn(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False,
          alpha: float = 1.0) -> torch.Tensor:
    """a^T @ b in fp32: a [(batch,) K, M], b [(batch,) K, N] -> out [(batch,) M, N] (written, or
    added to when ``accumulate``)."""
    K, M = a.shape[-2], a.shape[-1]
    N = b.shape[-1]
    if out is None:
        shp = (a.shape[0], M, N) if a.dim() == 3 else (M, N)
        out = torch.empty(shp, device=a.device, dtype=torch.float32)
    return gemm(a, b, out, M, N, K, True, True, 2 if accumulate else 1, alpha)


# ---------------------------------------------------------------------------------------
# csrc/gemm8.hip: 256x256-tile 8-phase MFMA GEMM on the STORED operands, C = epi(alpha * s1 * s2
# * A B^T): A [M, K] row-major or (a_col) [K, M]; B [N, K] or (b_col) [K, N]; bf16 (a row-mode
# operand needs K % 32 == 0) or fp8 e4m3fn (row mode, K % 128 == 0). Persistent grid of one
# 8-wave workgroup per CU; split-K (deterministic slice-order reduce) for grids of few tiles.

def gemm8_supported(M: int, N: int, K: int, fp8: bool = False, a_col: bool = False, b_col: bool = False) -> bool:
    if M <= 0 or N <= 0 or N % 4 or (a_col and M % 8) or (b_col and N % 8):
        return False
    if fp8:
        return not (a_col or b_col) and K % 128 == 0
    return (a_col and b_col) or K % 32 == 0


_MAX_SPLITS = 8


def gemm8_splits(M: int, N: int, K: int, batch: int = 1, cus: int = 256, min_slice: int = 1024,
                 tiles: Optional[int] = None) -> int:
    """k-slices for a grid of few 256^2 tiles (dx at D = 800: 124 tiles, dW / dU: 76-80),
    which would leave CUs idle: the split count that minimises the dispatch rounds per unit
    of work, ceil(tiles * S / cus) / S, with a small per-slice cost for the reduction, each
    slice >= min_slice of K (measured on the full chip: dW / dU 3 slices 93 / 98 us, 4 slices
    — a second round — 137 / 141 us). cus: the CUs the launch may use (a capped grid beside
    the persistent BPTT: 48 -> 5 rounds of 3 slices for 80 tiles)."""
    if tiles is None:
        tiles = _cdiv(M, 256) * _cdiv(N, 256) * batch
    if cus >= 128 and 2 * tiles > cus:
        return 1        # full chip, measured: dx D = 2400 (310 tiles) and dW D = 2400 (190) lose with any split
    best, best_cost = 1, None
    for s in range(1, _MAX_SPLITS + 1):
        if s > 1 and K // s < min_slice:
            break
        cost = _cdiv(tiles * s, cus) / s * (1.0 + 0.05 * (s - 1))
        if best_cost is None or cost < best_cost - 1e-9:
            best, best_cost = s, cost
    return best


# Parallel split-K reduction (csrc/gemm8.hip ds2_gemm8 ext_red): a launch of few tiles that the
# plain policy would already split (>= 2 k-slices, reduced by each tile's last-arriving slice
# reading the S slabs alone) is cut into k-slices of >= _EXT_MIN_KT k-tiles until the units fill
# the chip, and g8_reduce_kernel sums the partials on every CU. Measured (tools/bench_gemm8_plan.py,
# profiles/r5_gemm.md): the dx GEMMs of the short SortaGrad buckets 68-109 -> 28-43 us, the 100-frame
# layer-0 projection 56 -> 37 us; a K = 800 projection that the plain policy leaves unsplit lost
# with any split (28 -> 31-34 us), and a row-split of an under-full last dispatch round (its rows as
# k-sliced units taken round-robin by every workgroup) lost at every shape tried (54 -> 89 us at
# M = 3712), so neither is planned. False keeps the plain policy (A/B timing).
_PLAN = True
_EXT_MIN_KT = 3


def gemm8_plan(M: int, N: int, K: int, batch: int, cus: int, fp8: bool = False):
    """(S, ext_red) of a gemm8 launch, or None when the plain gemm8_splits policy applies."""
    if not _PLAN or batch != 1:
        return None
    tiles = _cdiv(M, 256) * _cdiv(N, 256)
    if gemm8_splits(M, N, K, batch, cus) < 2:
        return None
    nkt = _cdiv(K * (1 if fp8 else 2), 128)
    S = min(cus // tiles, nkt // _EXT_MIN_KT, 32)
    return (S, True) if S >= 2 else None


def gemm8(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor, epi: int = 0, alpha: float = 1.0,
          bias: Optional[torch.Tensor] = None, alpha_dev: Optional[torch.Tensor] = None,
          alpha_dev2: Optional[torch.Tensor] = None, a_col: bool = False, b_col: bool = False,
          splits: Optional[int] = None, max_grid: int = 0, fill=None, plan=None) -> torch.Tensor:
    """out (=, or += for epi 2) alpha * alpha_dev * alpha_dev2 * A @ B^T (+ bias) on the stored
    operands (see the section comment); out bf16 (epi 0) or fp32 (epi 1 / 2). splits=None picks
    the launch plan from the shape (gemm8_plan, else gemm8_splits); plan=(S, ext_red) forces
    one. max_grid > 0 caps the persistent grid (workgroups loop over the units): a launch
    beside the persistent BPTT."""
    batch = A.shape[0] if A.dim() == 3 else 1
    M = A.shape[-1] if a_col else A.shape[-2]
    K = A.shape[-2] if a_col else A.shape[-1]
    N = B.shape[-1] if b_col else B.shape[-2]
    fp8 = A.dtype == torch.float8_e4m3fn
    cus = _dev_cus(A)
    if max_grid > 0:
        cus = min(cus, max_grid)
    ext_red = False
    if plan is None:
        plan = gemm8_plan(M, N, K, batch, cus, fp8) if splits is None else None
    if plan is not None:
        splits, ext_red = plan
    elif splits is None:
        splits = gemm8_splits(M, N, K, batch, cus)
    C = _ext.ext()
    S = int(C.gemm8_splits(K, fp8, splits)) if splits > 1 else 1
    ws = cnt = None
    if S > 1:
        ws = torch.empty(S * batch * M * N, device=A.device, dtype=torch.float32)
        cnt = _tile_counters(A.device, _cdiv(M, 256) * _cdiv(N, 256) * batch)
    regions, pats = (list(fill[0]), list(fill[1])) if fill is not None else ([], [])
    C.gemm8(A, B, out, bias, epi, float(alpha), alpha_dev, alpha_dev2, a_col, b_col, S, ws, cnt, max_grid,
            regions, pats, ext_red and S > 1)
    return out


_GROUP_MAX = 24      # members of one csrc/gemm8.hip group launch (G8_MAXP)


def group_operands(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor):
    """(A, B) stored column-mode operands of a 2-D weight-gradient product out = a @ b (a [M, K]
    with unit-stride M, b [K, N] with unit-stride N, out fp32 [M, N]) that gemm8_group takes, or
    None when the product is not of that form."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and out.dtype == torch.float32):
        return None
    if a.dim() != 2 or b.dim() != 2 or out.dim() != 2 or out.stride(-1) != 1:
        return None
    oa, ob = _operand(a, True), _operand(b, False)
    if oa is None or ob is None or not (oa[1] and ob[1]):
        return None
    A, B = oa[0], ob[0]
    for t in (A, B, out):
        if t.data_ptr() % 16 or t.stride(-2) % 8:
            return None
    M, K, N = a.shape[0], a.shape[1], b.shape[1]
    if not gemm8_supported(M, N, K, False, True, True):
        return None
    return A, B


def gemm8_group(members, accumulate: bool = False, max_grid: int = 0, opt=None) -> None:
    """out_i (=, or += with ``accumulate``) A_i @ B_i^T for a list of (A, B, out) stored
    column-mode operands (:func:`group_operands`), as few launches as the group limit allows:
    one grid over every member's 256^2 tiles, so a set of small weight-gradient GEMMs fills the
    chip where each alone would leave CUs idle. Split-K only when even the whole group has too
    few tiles (gemm8_splits on the summed tile count).

    ``opt`` = (tensors, constants, store_g): instead of storing each out_i, the epilogue applies
    Adam + weight EMA to the same arena elements (csrc/gemm8.hip "Fused optimizer epilogue");
    tensors = [p, m, v, ema | None, p16 | None, grad arena], constants = [lr_t, b1, b2, eps,
    gscale, keep]; the outs must be aligned views of the grad arena (first writes)."""
    if opt is not None and accumulate:
        raise ValueError("the fused optimizer epilogue needs first-write members")
    C = _ext.ext()
    epi = 2 if accumulate else 1
    for lo in range(0, len(members), _GROUP_MAX):
        chunk = members[lo:lo + _GROUP_MAX]
        dev = chunk[0][0].device
        cus = _dev_cus(chunk[0][0])
        if max_grid > 0:
            cus = min(cus, max_grid)
        tiles = sum(_cdiv(A.shape[1], 256) * _cdiv(B.shape[1], 256) for A, B, _ in chunk)
        kmin = min(A.shape[0] for A, _, _ in chunk)
        S = gemm8_splits(0, 0, kmin, cus=cus, tiles=tiles)
        sp = [int(C.gemm8_splits(A.shape[0], False, S)) if S > 1 else 1 for A, _, _ in chunk]
        # the fewest workgroups that still finish in the same number of rounds: CUs the
        # quantisation would leave idle in the last round stay free from the start for the
        # kernels of other streams (the conv front-end's backward beside the tail group)
        units = tiles * max(sp)
        rounds = _cdiv(units, cus)
        grid = min(cus, 8 * _cdiv(_cdiv(units, rounds), 8))
        ws = cnt = None
        if max(sp) > 1:
            ws = torch.empty(sum(s * A.shape[1] * B.shape[1] for (A, B, _), s in zip(chunk, sp) if s > 1),
                             device=dev, dtype=torch.float32)
            cnt = _tile_counters(dev, tiles)
        if opt is None:
            C.gemm8_group([m[0] for m in chunk], [m[1] for m in chunk], [m[2] for m in chunk], [epi] * len(chunk),
                          sp, True, True, ws, cnt, grid)
        else:
            C.gemm8_group([m[0] for m in chunk], [m[1] for m in chunk], [m[2] for m in chunk], [epi] * len(chunk),
                          sp, True, True, ws, cnt, grid, list(opt[0]), [float(x) for x in opt[1]], bool(opt[2]))


_counters: Dict[Tuple[int, int], torch.Tensor] = {}
# replaced counter buffers stay allocated: a captured step graph (Trainer step graphs) keeps
# the address it was captured with, so a buffer must never be freed and handed to another use
_retired: List[torch.Tensor] = []


def _tile_counters(dev: torch.device, n: int) -> torch.Tensor:
    """Split-K arrival counters of the current stream (zero between launches: each launch's
    last-arriving slices reset theirs). One buffer per stream, since launches on different
    streams may run at the same time; a larger grid gets a fresh zeroed buffer."""
    key = (dev.index or 0, torch.cuda.current_stream(dev).cuda_stream)
    buf = _counters.get(key)
    if buf is None or buf.numel() < n:
        if buf is not None:
            _retired.append(buf)
        buf = torch.zeros(max(n, 4096), device=dev, dtype=torch.int32)
        _counters[key] = buf
    return buf


def linear8(x2: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor] = None, alpha: float = 1.0,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """alpha * x2 @ W^T + bias in bf16 through gemm8 (x2 [M, K], W [N, K])."""
    if out is None:
        out = torch.empty(x2.shape[0], W.shape[0], device=x2.device, dtype=torch.bfloat16)
    return gemm8(x2, W, out, 0, alpha, bias, splits=1)


def fp8_pad(K: int) -> int:
    """Reduction length of an fp8 gemm8 operand: K rounded up to the 128-deep k-tile."""
    return -(-K // 128) * 128


def linear_fp8(x2: torch.Tensor, W16: torch.Tensor, b16: Optional[torch.Tensor], alpha: float,
               x2b: Optional[torch.Tensor] = None, xsum: Optional[torch.Tensor] = None) -> torch.Tensor:
    """alpha * x2 @ W16^T + b16 with both operands quantised per tensor to OCP fp8 e4m3
    (csrc/quant.hip: amax, scale, saturating cast into K-padded copies, scales on the device)
    and multiplied by gemm8's fp8 path (v_mfma_scale_f32_16x16x128_f8f6f4: twice the bf16
    MFMA rate); the two scales and alpha are applied in the epilogue. bf16 output.
    x2b / xsum: the input is x2 + x2b (a bidirectional layer's direction outputs), summed by
    the quantiser's first pass into xsum (bf16, x2's shape; bitwise torch.add)."""
    C = _ext.ext()
    x2 = x2.contiguous()
    W16 = W16.contiguous()
    M, K = x2.shape
    N = W16.shape[0]
    Kp = fp8_pad(K)
    f8 = torch.float8_e4m3fn
    x8 = torch.empty(M, Kp, device=x2.device, dtype=f8)
    w8 = torch.empty(N, Kp, device=x2.device, dtype=f8)
    nb = int(C.fp8_quant_blocks(M * Kp, N * Kp))
    ws = torch.empty(2 * nb + 2, device=x2.device, dtype=torch.float32)
    C.fp8_quant2(x2, W16, float(alpha), x8, w8, ws[:2 * nb], ws[2 * nb:], x2b, xsum)
    out = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    return gemm8(x8, w8, out, 0, 1.0, b16, ws[2 * nb:2 * nb + 1], ws[2 * nb + 1:2 * nb + 2], splits=1)
