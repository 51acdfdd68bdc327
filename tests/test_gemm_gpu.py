"""Hand-written MFMA GEMM family (csrc/gemm.hip) against fp32 PyTorch references.

Every operand layout (row/col) and epilogue (bf16 + alpha + bias, fp32 store, fp32
accumulate), every tile configuration, ragged M/N tails, a K that ends in half a k-tile
(K % 64 == 32) and a batched call. Operands are asymmetric random data so a transposed
or swapped store cannot pass.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from deepspeech_amd.ops import gemm as G  # noqa: E402

DEV = torch.device("cuda:0")
BF = torch.bfloat16


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("M,N,K", [(7712, 800, 800), (300, 328, 96), (517, 1040, 2400), (390, 192, 72)])
def test_linear_bias_alpha(cfg, M, N, K):
    torch.manual_seed(cfg * 7 + M)
    x = torch.randn(M, K, device=DEV).to(BF)
    W = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = torch.randn(N, device=DEV).to(BF)
    out = G.gemm(x, W, torch.empty(M, N, device=DEV, dtype=BF), M, N, K, False, False, 0, 0.75, b, cfg=cfg)
    ref = 0.75 * (x.float() @ W.float().t()) + b.float()
    assert _rel(out, ref) < 6e-3


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("M,N,K", [(7712, 800, 4800), (200, 256, 160), (333, 2400, 4800), (390, 192, 200)])
def test_mm_nn(cfg, M, N, K):
    torch.manual_seed(cfg + N)
    a = torch.randn(M, K, device=DEV).to(BF)
    b = (torch.randn(K, N, device=DEV) * 0.05).to(BF)
    out = G.gemm(a, b, torch.empty(M, N, device=DEV, dtype=BF), M, N, K, False, True, 0, 1.0, None, cfg=cfg)
    ref = a.float() @ b.float()
    assert _rel(out, ref) < 6e-3


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("M,N,K", [(4800, 800, 7712), (2400, 800, 7712), (136, 264, 96), (192, 64 * 4, 390),
                                   (136, 128, 8)])
def test_mm_tn_store_and_accumulate(cfg, M, N, K):
    torch.manual_seed(cfg + K)
    a = torch.randn(K, M, device=DEV).to(BF)
    b = torch.randn(K, N, device=DEV).to(BF)
    ref = a.float().t() @ b.float()
    out = torch.full((M, N), float("nan"), device=DEV)
    G.gemm(a, b, out, M, N, K, True, True, 1, 1.0, None, cfg=cfg)
    assert _rel(out, ref) < 2e-5 * K ** 0.5 + 1e-4
    if cfg >= 6:
        return          # persistent configurations: no read-modify-write epilogue
    G.gemm(a, b, out, M, N, K, True, True, 2, 0.5, None, cfg=cfg)
    assert _rel(out, 1.5 * ref) < 2e-5 * K ** 0.5 + 1e-4


def test_mm_tn_batched_strided_output():
    """Both directions' dU in one launch, written into a strided slice of a bigger buffer."""
    torch.manual_seed(3)
    K, M, N = 7712, 2400, 800
    a = torch.randn(2, K, M, device=DEV).to(BF)
    b = torch.randn(2, K, N, device=DEV).to(BF)
    big = torch.zeros(2, M, N + 64, device=DEV)
    out = big[:, :, 32:32 + N]
    G.mm_tn(a, b, out)
    ref = torch.bmm(a.float().transpose(1, 2), b.float())
    assert _rel(out, ref) < 2e-3
    assert float(big[:, :, :32].abs().max()) == 0.0 and float(big[:, :, 32 + N:].abs().max()) == 0.0


def test_row_stride_views():
    """Operands given as column slices of wider matrices (leading dimension > K)."""
    torch.manual_seed(5)
    M, K, N = 1000, 800, 2400
    xw = torch.randn(M, K + 64, device=DEV).to(BF)
    x = xw[:, 64:]
    W = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    out = G.linear(x, W)
    assert _rel(out, x.float() @ W.float().t()) < 6e-3


# ------------------------------------------------------------------ csrc/gemm8.hip (8-phase 256^2)
@pytest.mark.parametrize("M,N,K", [(7712, 4800, 800), (7712, 800, 4800), (300, 328, 96), (517, 1040, 2400),
                                   (256, 256, 64), (255, 260, 32), (33, 4, 160), (7712, 7680, 1280)])
def test_gemm8_bf16_bias_alpha(M, N, K):
    """bf16 A B^T with the bf16 epilogue: ragged M / N tiles, odd k-tile counts, a last
    k-tile of 32 (K % 64 == 32), a single k-tile, and more tiles than CUs."""
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=DEV).to(BF)
    W = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = torch.randn(N, device=DEV).to(BF)
    out = G.linear8(x, W, b, alpha=0.75)
    ref = 0.75 * (x.float() @ W.float().t()) + b.float()
    assert _rel(out, ref) < 6e-3


@pytest.mark.parametrize("M,N,K", [(4800, 800, 7712), (136, 264, 96), (1000, 2400, 4800)])
def test_gemm8_fp32_store_accumulate_batched(M, N, K):
    """fp32 epilogues (store, then accumulate) on row-stride views and a batch of 2, with an
    asymmetric operand pair so a swapped / transposed store cannot pass."""
    torch.manual_seed(K)
    a = torch.randn(2, M, K, device=DEV).to(BF)
    b = (torch.randn(2, N, K, device=DEV) + 0.1).to(BF)
    ref = a.float() @ b.float().transpose(1, 2)
    out = torch.full((2, M, N), float("nan"), device=DEV)
    G.gemm8(a, b, out, 1, 0.5, splits=1)
    assert _rel(out, 0.5 * ref) < 2e-5 * K ** 0.5 + 1e-4
    G.gemm8(a, b, out, 2, 1.0, splits=1)
    assert _rel(out, 1.5 * ref) < 2e-5 * K ** 0.5 + 1e-4
    # a row-strided operand view (every other row of a taller matrix)
    big = torch.randn(2 * M, K, device=DEV).to(BF)
    o2 = torch.empty(M, N, device=DEV)
    G.gemm8(big[::2], b[0], o2, 1, splits=1)
    assert _rel(o2, big[::2].float() @ b[0].float().t()) < 2e-5 * K ** 0.5 + 1e-4


@pytest.mark.parametrize("M,N,K", [(7712, 4800, 800), (7712, 7680, 2400), (300, 328, 96), (64, 256, 1280)])
def test_gemm8_fp8_projection(M, N, K):
    """fp8 e4m3 per-tensor quantised projection (K padded to the 128-deep k-tile): equals
    the fp32 product of the DEQUANTISED operands to fp32 accumulation error, and the bf16
    product to fp8 rounding error."""
    torch.manual_seed(M + K)
    x = torch.randn(M, K, device=DEV).to(BF)
    W = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = torch.randn(N, device=DEV).to(BF)
    out = G.linear_fp8(x, W, b, 0.9)
    sx = x.float().abs().max() / 448.0
    sw = W.float().abs().max() / 448.0
    xq = (x.float() / sx).to(torch.float8_e4m3fn).float() * sx
    wq = (W.float() / sw).to(torch.float8_e4m3fn).float() * sw
    ref_q = 0.9 * (xq @ wq.t()) + b.float()
    # bf16 output rounding, and e4m3 ties the HIP cast and torch's round differently
    assert _rel(out, ref_q) < 1.5e-2
    ref = 0.9 * (x.float() @ W.float().t()) + b.float()
    assert _rel(out, ref) < 6e-2                         # e4m3: 3 mantissa bits


def test_gemm8_rejects_unsupported_k():
    a = torch.randn(64, 48, device=DEV).to(BF)
    with pytest.raises(RuntimeError):
        G.gemm8(a, a, torch.empty(64, 64, device=DEV, dtype=BF), 0)


@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("M,N,K", [(7712, 800, 4800), (7712, 2400, 4800), (300, 328, 96), (136, 264, 7712)])
def test_gemm8_dx_col_b(splits, M, N, K):
    """dx = dgx W with W read as stored ([K][N], N contiguous: column mode, transposed LDS
    reads), bf16 output, optionally split over k-slices (deterministic reduce)."""
    torch.manual_seed(N + K + splits)
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(K, N, device=DEV) * 0.05 + 0.01).to(BF)
    out = G.gemm8(a, w, torch.empty(M, N, device=DEV, dtype=BF), 0, 1.0, b_col=True, splits=splits)
    assert _rel(out, a.float() @ w.float()) < 6e-3


@pytest.mark.parametrize("splits", [1, 2, 5])
@pytest.mark.parametrize("M,N,K", [(4800, 800, 7712), (2400, 800, 7712), (136, 264, 96), (192, 256, 390),
                                   (136, 128, 8), (800, 32, 300)])
def test_gemm8_wgrad_col_col(splits, M, N, K):
    """Weight gradients a^T b with both operands stored [K][M] / [K][N] (column mode), fp32
    store then accumulate, any K (k-rows past K load as zeros), split-K."""
    torch.manual_seed(M + K + splits)
    a = torch.randn(K, M, device=DEV).to(BF)
    b = (torch.randn(K, N, device=DEV) + 0.1).to(BF)
    ref = a.float().t() @ b.float()
    out = torch.full((M, N), float("nan"), device=DEV)
    G.gemm8(a, b, out, 1, 1.0, a_col=True, b_col=True, splits=splits)
    assert _rel(out, ref) < 2e-5 * K ** 0.5 + 1e-4
    G.gemm8(a, b, out, 2, 0.5, a_col=True, b_col=True, splits=splits)
    assert _rel(out, 1.5 * ref) < 2e-5 * K ** 0.5 + 1e-4


def test_gemm8_wgrad_batched_directions():
    """dU of both directions as one batched call (batch stride over the directions)."""
    torch.manual_seed(3)
    K, M, N = 7712, 2400, 800
    a = torch.randn(2, K, M, device=DEV).to(BF)
    b = torch.randn(2, K, N, device=DEV).to(BF)
    out = torch.empty(2, M, N, device=DEV)
    G.gemm8(a, b, out, 1, 1.0, a_col=True, b_col=True)
    ref = a.float().transpose(1, 2) @ b.float()
    assert _rel(out, ref) < 2e-5 * K ** 0.5 + 1e-4


def test_gemm8_row_a_col_b_ragged_k():
    """A row-mode operand with K % 64 == 32 beside a column-mode one: the last k-tile's
    second k-substep is skipped (its row-mode chunks hold the next row's data)."""
    torch.manual_seed(4)
    M, N, K = 520, 264, 800
    a = torch.randn(M, K, device=DEV).to(BF)
    w = torch.randn(K, N, device=DEV).to(BF)
    out = G.gemm8(a, w, torch.empty(M, N, device=DEV, dtype=BF), 0, 1.0, b_col=True, splits=1)
    assert _rel(out, a.float() @ w.float()) < 6e-3


def test_gemm8_split_reproducible():
    """Split-K is bitwise reproducible (slice-order reduce, no atomics)."""
    torch.manual_seed(5)
    a = torch.randn(7712, 4800, device=DEV).to(BF)
    b = torch.randn(7712, 800, device=DEV).to(BF)
    o1 = G.gemm8(a, b, torch.empty(4800, 800, device=DEV), 1, 1.0, a_col=True, b_col=True, splits=4)
    o2 = G.gemm8(a, b, torch.empty(4800, 800, device=DEV), 1, 1.0, a_col=True, b_col=True, splits=4)
    assert torch.equal(o1, o2)


@pytest.mark.parametrize("R,C", [(4800, 800), (4800, 2400), (72, 136), (8, 8), (1000, 24)])
def test_transpose_bf16(R, C):
    """csrc/fill.hip transpose (the dx GEMM's K-contiguous W^T shadow): exact, ragged tiles."""
    from deepspeech_amd.ops import _ext
    torch.manual_seed(R + C)
    w = torch.randn(R, C, device=DEV).to(BF)
    out = torch.full((C, R), float("nan"), device=DEV, dtype=BF)
    _ext.ext().transpose_bf16(w, out)
    assert torch.equal(out, w.t())


def test_gemm8_split_counters_reset_and_streams():
    """Split-K tile counters are left at zero by every launch (a second launch on the same
    buffer is correct), and launches on two streams use separate counter buffers."""
    torch.manual_seed(6)
    a = torch.randn(7712, 2400, device=DEV).to(BF)
    b = torch.randn(7712, 800, device=DEV).to(BF)
    ref = a.float().t() @ b.float()
    s2 = torch.cuda.Stream()
    outs = []
    for i in range(3):
        st = s2 if i == 1 else torch.cuda.current_stream()
        with torch.cuda.stream(st):
            outs.append(G.gemm8(a, b, torch.empty(2400, 800, device=DEV), 1, 1.0, a_col=True, b_col=True,
                                splits=3))
    torch.cuda.synchronize()
    for o in outs:
        assert _rel(o, ref) < 2e-5 * 7712 ** 0.5 + 1e-4
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[0], outs[1])
    for buf in G._counters.values():
        assert int(buf.abs().sum()) == 0


@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm8_group_weight_gradients(accumulate):
    """A grouped launch of unrelated column-column weight-gradient GEMMs (csrc/gemm8.hip
    problem table): shapes of the deferred dW / dU of a wide layer, a ragged tiny one and the
    two directions of a batched dU read through strided views; each member equals its fp32
    product, stored or accumulated."""
    torch.manual_seed(7)
    K = 7712
    dgh = torch.randn(2, K, 1760, device=DEV).to(BF)
    h = torch.randn(2, K, 1760, device=DEV).to(BF)
    dgx = torch.randn(K, 3520, device=DEV).to(BF)
    x = torch.randn(K, 2400, device=DEV).to(BF)
    sa = torch.randn(390, 136, device=DEV).to(BF)
    sb = torch.randn(390, 264, device=DEV).to(BF)
    ops = [(dgh[0], h[0]), (dgh[1], h[1]), (dgx, x), (sa, sb), (dgx[:, 1760:], h[1])]
    outs = [torch.randn(a.shape[1], b.shape[1], device=DEV) for a, b in ops]
    base = [o.clone() for o in outs]
    members = []
    for (a, b), o in zip(ops, outs):
        A, B = G.group_operands(a.t(), b, o)
        members.append((A, B, o))
    G.gemm8_group(members, accumulate=accumulate)
    for (a, b), o, o0 in zip(ops, outs, base):
        ref = a.float().t() @ b.float() + (o0 if accumulate else 0)
        assert _rel(o, ref) < 2e-5 * a.shape[0] ** 0.5 + 1e-4


def test_gemm8_group_split_and_chunks():
    """A group with few tiles takes split-K (workspace ranges per member, counters left at
    zero), and more members than one launch holds run as several launches."""
    torch.manual_seed(8)
    ops = [(torch.randn(4000, 256, device=DEV).to(BF), torch.randn(4000, 264, device=DEV).to(BF))
           for _ in range(3)]
    outs = [torch.empty(256, 264, device=DEV) for _ in ops]
    G.gemm8_group([(a, b, o) for (a, b), o in zip(ops, outs)])
    for (a, b), o in zip(ops, outs):
        assert _rel(o, a.float().t() @ b.float()) < 2e-5 * 4000 ** 0.5 + 1e-4
    torch.cuda.synchronize()
    for buf in G._counters.values():
        assert int(buf.abs().sum()) == 0
    many = [(torch.randn(96, 8 * (i % 5 + 1), device=DEV).to(BF), torch.randn(96, 16, device=DEV).to(BF))
            for i in range(30)]
    outs = [torch.empty(a.shape[1], 16, device=DEV) for a, _ in many]
    G.gemm8_group([(a, b, o) for (a, b), o in zip(many, outs)])
    for (a, b), o in zip(many, outs):
        assert _rel(o, a.float().t() @ b.float()) < 1e-4


@pytest.mark.parametrize("split_case", [False, True])
def test_gemm8_group_fused_adam_epilogue_bitwise(split_case):
    """The grouped weight-gradient launch with the fused optimizer epilogue (csrc/gemm8.hip):
    Adam + EMA + bf16 shadow of every member's arena elements equal BITWISE the plain launch
    (gradients stored) followed by the streaming optimizer (csrc/optim.hip), members at
    offsets inside one arena with untouched gaps between them; store_g also leaves the
    gradients bitwise as the plain launch stores them. split_case: few tiles -> split-K, the
    last-arriving slice applies the update."""
    from deepspeech_amd.ops import _ext
    torch.manual_seed(21)
    C = _ext.ext()
    if split_case:
        shapes = [(4000, 256, 264), (4000, 128, 96)]
    else:
        shapes = [(7712, 4800, 800), (7712, 2400, 800), (7712, 800, 800), (7712, 96, 264)]   # 134 tiles: no split
    ops = [(torch.randn(K, M, device=DEV).to(BF), torch.randn(K, N, device=DEV).to(BF)) for K, M, N in shapes]
    offs, pos = [], 128
    for K, M, N in shapes:
        offs.append(pos)
        pos += M * N + 64                     # a 64-element gap no member owns
    n = pos + 256
    p0 = torch.randn(n, device=DEV)
    m0 = torch.randn(n, device=DEV) * 1e-3
    v0 = torch.rand(n, device=DEV) * 1e-4
    e0 = torch.randn(n, device=DEV)
    lr_t, b1, b2, eps, gscale, keep = 3e-4, 0.9, 0.999, 1e-8, 0.5, 0.99

    def arena():
        return dict(p=p0.clone(), m=m0.clone(), v=v0.clone(), e=e0.clone(), g=torch.zeros(n, device=DEV),
                    p16=torch.zeros(n, device=DEV, dtype=BF))

    def members(a):
        out = []
        for (A, B), o, (K, M, N) in zip(ops, offs, shapes):
            view = a["g"][o:o + M * N].view(M, N)
            oa, ob = G.group_operands(A.t(), B, view)
            out.append((oa, ob, view))
        return out
    ref = arena()
    G.gemm8_group(members(ref))
    ranges = [(o, o + M * N) for o, (K, M, N) in zip(offs, shapes)]
    for lo, hi in ranges:
        C.adam_ema(ref["p"][lo:hi], ref["g"][lo:hi], ref["m"][lo:hi], ref["v"][lo:hi], ref["e"][lo:hi],
                   ref["p16"][lo:hi], lr_t, b1, b2, eps, gscale, keep, None, 0)
    for store_g in (False, True):
        got = arena()
        G.gemm8_group(members(got), opt=([got["p"], got["m"], got["v"], got["e"], got["p16"], got["g"]],
                                         [lr_t, b1, b2, eps, gscale, keep], store_g))
        torch.cuda.synchronize()
        for k in ("p", "m", "v", "e", "p16"):
            assert torch.equal(got[k], ref[k]), (k, store_g)
        if store_g:
            assert torch.equal(got["g"], ref["g"])
        else:
            assert int((got["g"] != 0).sum()) == 0          # no gradient written
    for buf in G._counters.values():
        assert int(buf.abs().sum()) == 0


def test_adam_ema_ranges_bitwise():
    """One launch over several arena ranges (csrc/optim.hip adam_ema_ranges) equals one
    adam_ema launch per range, bitwise, and leaves the elements between ranges untouched."""
    from deepspeech_amd.ops import _ext
    torch.manual_seed(22)
    C = _ext.ext()
    n = 50000
    bufs = [torch.randn(n, device=DEV), torch.randn(n, device=DEV), torch.randn(n, device=DEV) * 1e-3,
            torch.rand(n, device=DEV) * 1e-4, torch.randn(n, device=DEV)]
    ranges = [(0, 1000), (1024, 1028), (4096, 40000), (40064, 49996)]
    a = [t.clone() for t in bufs] + [torch.zeros(n, device=DEV, dtype=BF)]
    b = [t.clone() for t in bufs] + [torch.zeros(n, device=DEV, dtype=BF)]
    for lo, hi in ranges:
        C.adam_ema(a[0][lo:hi], a[1][lo:hi], a[2][lo:hi], a[3][lo:hi], a[4][lo:hi], a[5][lo:hi], 1e-3, 0.9, 0.999,
                   1e-8, 1.0, 0.9, None, 0)
    C.adam_ema_ranges(b[0], b[1], b[2], b[3], b[4], b[5], [x for r in ranges for x in r], 1e-3, 0.9, 0.999, 1e-8,
                      1.0, 0.9)
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert torch.equal(b[0][1000:1024], bufs[0][1000:1024])


@pytest.mark.parametrize("M,N,K", [(7712, 4800, 800), (4096, 4096, 256), (300, 328, 96)])
def test_gemm8_idle_workgroup_fill(M, N, K):
    """csrc/gemm8.hip DS2Fill: regions initialised by the launch's lighter workgroups — the GEMM
    output bitwise that of a launch without fill, every region word its pattern (aligned,
    unaligned-tail and 4-B-aligned regions), for uneven (589 tiles), even (256) and tiny grids."""
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = torch.randn(N, device=DEV).to(BF)
    ref = torch.empty(M, N, device=DEV, dtype=BF)
    G.gemm8(x, w, ref, epi=0, alpha=0.5, bias=b)
    big = torch.zeros(3 * 1024 * 1024 + 7, device=DEV, dtype=torch.int32)
    odd = torch.zeros(1001, device=DEV, dtype=torch.int32)[1:]          # 4-B aligned, not 16-B
    hb = torch.full((2, 242, 32, 800), 1.0, device=DEV, dtype=BF)
    regions = [big, odd, hb[0, 0], hb[0, 1:], hb[1, 1:]]
    pats = [-1, 0x12345678, 0, -1, -1]
    out = torch.empty(M, N, device=DEV, dtype=BF)
    G.gemm8(x, w, out, epi=0, alpha=0.5, bias=b, fill=(regions, pats))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert bool((big == -1).all()) and bool((odd == 0x12345678).all())
    assert bool((hb[0, 0] == 0).all()) and bool((hb[1, 0] == 1.0).all())
    assert bool((hb[:, 1:].view(torch.int16) == -1).all())


def test_gemm8_fill_only_on_row_row():
    a = torch.randn(256, 256, device=DEV).to(BF)
    o = torch.empty(256, 256, device=DEV, dtype=torch.float32)
    r = torch.zeros(64, device=DEV, dtype=torch.int32)
    with pytest.raises(RuntimeError):
        G.gemm8(a, a, o, epi=1, a_col=True, b_col=True, fill=([r], [-1]))


@pytest.mark.parametrize("cfg", [7, 3])
def test_gemm_fill_persistent_and_fallback(cfg):
    """csrc/gemm.hip with a DS2Fill: the persistent configuration fills from its lighter
    workgroups (the dx GEMM feeding the next BPTT: 244 tiles on 248 workgroups), any other runs
    the fill kernel after; output bitwise that of a launch without fill."""
    M, N, K = 7712, 800, 4800
    torch.manual_seed(cfg)
    a = torch.randn(M, K, device=DEV).to(BF)
    wt = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    ref = torch.empty(M, N, device=DEV, dtype=BF)
    G.gemm(a, wt, ref, M, N, K, False, False, 0, 1.0, None, cfg=cfg)
    census = torch.zeros(400, device=DEV, dtype=torch.int32)
    parts = torch.full((2, 2, 4, 2400), 3.0, device=DEV)
    ring = torch.zeros(2, 30001, device=DEV)
    out = torch.empty(M, N, device=DEV, dtype=BF)
    G.gemm(a, wt, out, M, N, K, False, False, 0, 1.0, None, cfg=cfg, fill=([census, parts, ring], [-1, 0, -1]))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert bool((census == -1).all()) and bool((parts == 0).all())
    assert bool((ring.view(torch.int32) == -1).all())


# ------------------------------------------------ gemm8 launch plans (ops/gemm.py gemm8_plan)
@pytest.mark.parametrize("M,N,K,a_col,b_col", [(672, 800, 4800, False, False), (672, 4800, 800, False, False),
                                                (1312, 2400, 4800, False, True), (300, 328, 960, False, False),
                                                (2400, 800, 672, True, True)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm8_parallel_reduce_bitwise_in_launch_reduce(M, N, K, a_col, b_col, epi):
    """ext_red: the k-slices only store their partials and g8_reduce_kernel sums them on the
    whole chip — bitwise the in-launch last-arriver reduction of the same slices (same order,
    same epilogue), and close to the fp32 reference; bf16 (+ bias, alpha) and fp32 store /
    accumulate epilogues, row- and column-mode operands."""
    if epi == 0 and (a_col and b_col):
        pytest.skip("column-column is the fp32 weight-gradient variant")
    torch.manual_seed(M + N + K + epi)
    A = torch.randn((K, M) if a_col else (M, K), device=DEV).to(BF)
    B = (torch.randn((K, N) if b_col else (N, K), device=DEV) * 0.05 + 0.01).to(BF)
    b = torch.randn(N, device=DEV).to(BF) if epi == 0 else None
    dt = BF if epi == 0 else torch.float32
    init = torch.randn(M, N, device=DEV).to(dt)
    S = 6
    o_in, o_ext = init.clone(), init.clone()
    G.gemm8(A, B, o_in, epi, 0.75, b, a_col=a_col, b_col=b_col, plan=(S, False))
    G.gemm8(A, B, o_ext, epi, 0.75, b, a_col=a_col, b_col=b_col, plan=(S, True))
    torch.cuda.synchronize()
    assert torch.equal(o_in, o_ext)
    Af = A.float().t() if a_col else A.float()
    Bf = B.float() if b_col else B.float().t()
    ref = 0.75 * (Af @ Bf) + (b.float() if b is not None else 0.0) + (init.float() if epi == 2 else 0.0)
    assert _rel(o_ext, ref) < (6e-3 if epi == 0 else 2e-5 * K ** 0.5 + 1e-4)


def test_gemm8_plan_policy():
    """The planner's choices at the DS2 shapes (256 CUs): parallel-reduce split-K where the plain
    policy splits (a few tiles), nothing where it does not (full chip, K = 800 projections)."""
    assert G.gemm8_plan(672, 800, 4800, 1, 256) == (21, True)
    assert G.gemm8_plan(672, 4800, 2400, 1, 256) == (4, True)
    assert G.gemm8_plan(672, 4800, 800, 1, 256) is None
    assert G.gemm8_plan(7712, 4800, 800, 1, 256) is None
    assert G.gemm8_plan(7712, 800, 4800, 2, 256) is None            # batched launches: plain policy


@pytest.mark.parametrize("M,N,K", [(672, 4800, 800), (672, 4800, 2400), (1312, 4800, 800), (672, 7680, 1280),
                                   (2432, 4800, 800)])
def test_short_bucket_projection_routing(cuda, M, N, K):
    """matmul's short-bucket rule (ops/gemm.py _small_rowrow): row-row bf16 projections of few
    256^2 tiles and K <= 2400 run on csrc/gemm.hip's cost-model tile, the rest on gemm8; either
    way alpha * x W^T + bias within bf16 rounding of the fp32 product."""
    torch.manual_seed(M + K)
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    W = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    small = G._small_rowrow(M, N, K, False, False, 1, 0, x)
    assert small == (M <= 1312 and (K <= 2400) and (-(-M // 256)) * (-(-N // 256)) * 2 <= G._dev_cus(x))
    assert G.matmul(x, W.t(), out, alpha=0.5, bias=b)
    torch.cuda.synchronize()
    ref = 0.5 * (x.float() @ W.float().t()) + b.float()
    assert _rel(out, ref) < 6e-3
