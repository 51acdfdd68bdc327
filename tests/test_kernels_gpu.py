"""Numerics of every gfx950 kernel against a plain-PyTorch fp32 reference of the same op."""
import math

import pytest
import torch
import torch.nn.functional as F

from deepspeech_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


# --------------------------------------------------------------------------- recurrence
def _rnn_case(cuda, cell, N, H, T, ndir, mode, seed=0, din=None, kernel="xcd"):
    import os
    from deepspeech_amd.ops import rnn as RNN
    torch.manual_seed(seed)
    G = RNN.GATES[cell]
    lens = torch.randint(max(1, T // 2), T + 1, (N,), dtype=torch.int32)
    lens[0] = T
    scale = 0.5 if cell == "gru" else 0.2
    gx = (torch.randn(T, N, ndir * G * H) * scale).bfloat16().to(cuda)
    for b in range(N):
        gx[int(lens[b]):, b] = 0
    Us = [(torch.randn(G * H, H) / math.sqrt(H)).bfloat16().to(cuda) for _ in range(ndir)]
    bhs = [(torch.randn(G * H) * 0.1).to(cuda) if cell == "gru" else None for _ in range(ndir)]
    old = os.environ.get("DS2_RNN_MODE")
    # generation 1 (kernel "v1") is DS2_RNN_MODE=v1; "auto" takes the XCD kernels where they fit
    os.environ["DS2_RNN_MODE"] = "v1" if (kernel == "v1" and mode == "auto") else mode
    try:
        RNN._plan_cache.clear()
        plan = RNN.plan_for(N, H, cell, ndir, cuda)
    finally:
        if old is None:
            os.environ.pop("DS2_RNN_MODE")
        else:
            os.environ["DS2_RNN_MODE"] = old
        RNN._plan_cache.clear()
    if mode == "auto" and kernel == "xcd" and RNN.make_xcd_plan(N, H, cell, ndir, 256) is not None:
        assert plan.kind == "xcd", plan
    # HIP
    gx_h = gx.clone().requires_grad_(True)
    U_h = [u.clone().requires_grad_(True) for u in Us]
    b_h = [b.clone().requires_grad_(True) if b is not None else None for b in bhs]
    y = RNN.BiRecurrence.apply(gx_h, lens.to(cuda), U_h[0], U_h[1] if ndir == 2 else None,
                               b_h[0], b_h[1] if ndir == 2 else None, plan)
    dy = torch.randn(T, N, H, device=cuda).bfloat16()
    for b in range(N):
        dy[int(lens[b]):, b] = 0
    y.backward(dy)
    torch.cuda.synchronize()
    RNN.check_errors()
    # fp32 reference
    gx_r = gx.float().clone().requires_grad_(True)
    U_r = [u.float().clone().requires_grad_(True) for u in Us]
    b_r = [b.clone().requires_grad_(True) if b is not None else None for b in bhs]
    GH = G * H
    yr = R.birnn_ref(cell, gx_r[..., :GH], gx_r[..., GH:] if ndir == 2 else None, U_r[0],
                     U_r[1] if ndir == 2 else None, b_r[0], b_r[1] if ndir == 2 else None,
                     lens.to(cuda), mm_dtype=torch.bfloat16)
    yr.backward(dy.float())
    # wide clipped-ReLU layers: bf16 state exchange flips near-zero ReLU masks against the
    # reference; both kernel generations sit at ~3 % there (measured: v1 3.2 %, xcd 3.1 %)
    gtol = 5e-2 if (cell == "rnn_relu" and H > 1024) else 3e-2
    assert _rel(y, yr) < 2e-2, ("y", _rel(y, yr))
    assert _rel(gx_h.grad, gx_r.grad) < gtol, ("dgx", _rel(gx_h.grad, gx_r.grad))
    for d in range(ndir):
        assert _rel(U_h[d].grad, U_r[d].grad) < gtol, ("dU", d, _rel(U_h[d].grad, U_r[d].grad))
        if cell == "gru":
            assert _rel(b_h[d].grad, b_r[d].grad) < 3e-2, ("dbh", d)
    # padding positions must be exactly zero
    for b in range(N):
        L = int(lens[b])
        assert float(y[L:, b].abs().max() if L < T else 0) == 0.0
        assert float(gx_h.grad[L:, b].abs().max() if L < T else 0) == 0.0


@pytest.mark.parametrize("cell", ["rnn_relu", "gru"])
@pytest.mark.parametrize("mode", ["auto", "step"])
def test_birnn_small(cuda, cell, mode):
    _rnn_case(cuda, cell, N=5, H=64, T=23, ndir=2, mode=mode)


@pytest.mark.parametrize("cell", ["rnn_relu", "gru"])
@pytest.mark.parametrize("kernel", ["xcd", "v1"])
def test_birnn_ds2_shape(cuda, cell, kernel):
    # the flagship geometry: batch 32, H=800 (xcd: 8 groups of 8 rows x 25 workgroups;
    # v1: two batch groups, 50 slices per direction)
    _rnn_case(cuda, cell, N=32, H=800, T=61, ndir=2, mode="auto", seed=3, kernel=kernel)


@pytest.mark.parametrize("N,H", [(16, 1280), (48, 512), (3, 96)])
def test_birnn_xcd_geometries(cuda, N, H):
    # spread groups (H=1280: 40 workgroups > one XCD), 16-row groups, tiny batch
    _rnn_case(cuda, "gru", N=N, H=H, T=33, ndir=2, mode="auto", seed=9)


@pytest.mark.parametrize("cell,N,H", [("gru", 32, 800), ("rnn_relu", 32, 800), ("gru", 40, 256), ("gru", 7, 96), ("gru", 32, 1280), ("rnn_relu", 32, 1760)])
def test_bptt_exchanges(cuda, cell, N, H):
    # the BPTT kernel each geometry's plan selects (reduce-scatter generation 3, or the
    # generation-1 kernels past 42 workgroups per group) against the reference
    _rnn_case(cuda, cell, N=N, H=H, T=45, ndir=2, mode="auto", seed=21)


@pytest.mark.parametrize("N,H,ndir", [(32, 1760, 2), (20, 1440, 2), (32, 1088, 2), (13, 1760, 1)])
def test_wide_relu_kernels(cuda, N, H, ndir):
    # one-gate layers wider than an XCD at 32 units per workgroup run the 64-unit wide kernels
    # (rnnw_fwd_kernel / rnnw_bwd_kernel): full and half-empty last workgroups (H % 64 == 32),
    # every LDS/register split of the U slice in use, one direction
    from deepspeech_amd.ops import rnn as RNN
    assert RNN._wide_ok(H, "rnn_relu")
    p = RNN.make_xcd_plan(N, H, "rnn_relu", ndir, 256)
    assert p is not None and p.kind == "xcd" and p.xcd_map == 1 and p.R <= 8
    _rnn_case(cuda, "rnn_relu", N=N, H=H, T=37, ndir=ndir, mode="auto", seed=31)


def test_unirnn_gru(cuda):
    _rnn_case(cuda, "gru", N=17, H=256, T=40, ndir=1, mode="auto", seed=5)


def test_birnn_mt2(cuda):
    # batch 96 with H=1280 forces two 16-row tiles per workgroup
    _rnn_case(cuda, "gru", N=96, H=1280, T=12, ndir=2, mode="auto", seed=7)


# --------------------------------------------------------------------------- CTC
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ctc_fused(cuda, dtype):
    from deepspeech_amd.ops import ctc as CTC
    torch.manual_seed(0)
    T, N, K = 50, 6, 29
    logits = (torch.randn(T, N, K) * 2).to(dtype).to(cuda)
    lens = torch.tensor([50, 45, 30, 50, 12, 40], dtype=torch.int32)
    Ls = [20, 10, 14, 1, 5, 19]
    labels = torch.zeros(N, max(Ls), dtype=torch.int32)
    for b, L in enumerate(Ls):
        labels[b, :L] = torch.randint(0, K - 1, (L,))
    labels[0, 3] = labels[0, 4]          # a repeat (needs a blank between)
    lab_lens = torch.tensor(Ls, dtype=torch.int32)
    x = logits.clone().requires_grad_(True)
    loss = CTC.ctc_loss_hip(x, lens.to(cuda), labels.to(cuda), lab_lens.to(cuda))
    loss.mean().backward()
    xr = logits.float().clone().requires_grad_(True)
    lr = R.ctc_loss_ref(xr, labels.to(cuda), lens.to(cuda), lab_lens.to(cuda))
    lr.mean().backward()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert torch.allclose(loss, lr, rtol=tol, atol=tol), (loss, lr)
    assert _rel(x.grad, xr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("Lmax,T", [(60, 150), (150, 241), (180, 400), (240, 500), (300, 700)])
def test_ctc_long_labels(cuda, Lmax, T):
    """Lattices of 121..601 states: every register-tile width of the one-wave recursion."""
    from deepspeech_amd.ops import ctc as CTC
    torch.manual_seed(1)
    N, K = 5, 29
    logits = (torch.randn(T, N, K) * 1.5).bfloat16().to(cuda)
    lens = torch.tensor([T, T - 7, T - 30, T, T - 1], dtype=torch.int32)
    Ls = [Lmax, Lmax - 3, Lmax // 2, 1, Lmax - 1]
    labels = torch.zeros(N, Lmax, dtype=torch.int32)
    for b, L in enumerate(Ls):
        labels[b, :L] = torch.randint(0, K - 1, (L,))
    lab_lens = torch.tensor(Ls, dtype=torch.int32)
    x = logits.clone().requires_grad_(True)
    loss = CTC.ctc_loss_hip(x, lens.to(cuda), labels.to(cuda), lab_lens.to(cuda))
    loss.mean().backward()
    xr = logits.float().clone().requires_grad_(True)
    lr = R.ctc_loss_ref(xr, labels.to(cuda), lens.to(cuda), lab_lens.to(cuda))
    lr.mean().backward()
    assert torch.allclose(loss, lr, rtol=1e-3, atol=1e-2), (loss, lr)
    assert _rel(x.grad, xr.grad) < 2e-2


def test_ctc_peaked_distributions(cuda):
    """Confident (peaked) frames, log-probs down to ~-100 nats. The kernel runs the alpha/beta
    recursion in log2 units: the staged log-prob rows are scaled by LOG2E, each lattice state
    takes a branch-free 3-way log-sum-exp (lse3_rec: max3/med3/min3, two exp2 + one log2, -1e30 as log 0), and
    the stored alpha/beta rows are rescaled by LN2 back to nats for the gradient. Large
    log-prob gaps stress exactly that lse (exp2 underflow of the two smaller terms) and the
    unit conversion; the result must track the natural-log reference."""
    from deepspeech_amd.ops import ctc as CTC
    torch.manual_seed(3)
    T, N, K = 120, 4, 29
    logits = (torch.randn(T, N, K) * 12).to(cuda)
    lens = torch.tensor([120, 100, 77, 120], dtype=torch.int32)
    Ls = [40, 30, 20, 55]
    labels = torch.zeros(N, max(Ls), dtype=torch.int32)
    for b, L in enumerate(Ls):
        labels[b, :L] = torch.randint(0, K - 1, (L,))
    lab_lens = torch.tensor(Ls, dtype=torch.int32)
    x = logits.clone().requires_grad_(True)
    loss = CTC.ctc_loss_hip(x, lens.to(cuda), labels.to(cuda), lab_lens.to(cuda))
    loss.mean().backward()
    xr = logits.clone().requires_grad_(True)
    lr = R.ctc_loss_ref(xr, labels.to(cuda), lens.to(cuda), lab_lens.to(cuda))
    lr.mean().backward()
    assert torch.isfinite(loss).all() and float(loss.min()) > 100.0, loss
    assert torch.allclose(loss, lr, rtol=1e-4, atol=1e-2), (loss, lr)
    assert _rel(x.grad, xr.grad) < 1e-3


def test_ctc_infeasible_zero(cuda):
    from deepspeech_amd.ops import ctc as CTC
    T, N, K = 4, 1, 29
    logits = torch.randn(T, N, K, device=cuda, requires_grad=True)
    labels = torch.tensor([[1, 1, 1, 1]], dtype=torch.int32, device=cuda)
    loss = CTC.ctc_loss_hip(logits, torch.tensor([4], dtype=torch.int32, device=cuda), labels,
                            torch.tensor([4], dtype=torch.int32, device=cuda))
    loss.sum().backward()
    assert float(loss) == 0.0 and float(logits.grad.abs().sum()) == 0.0


# --------------------------------------------------------------------------- BN + clip
@pytest.mark.parametrize("layout", [0, 1])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_clip(cuda, layout, dtype):
    from deepspeech_amd.ops.frontend import BNClip, BN_EPS
    torch.manual_seed(0)
    N, C, T, Fd = 3, 8, 37, 11
    y = (torch.randn(N, C, T, Fd) * 3 + 1).to(dtype).to(cuda)
    gamma = (torch.rand(C) + 0.5).to(cuda)
    beta = (torch.randn(C) * 0.5).to(cuda)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    yh = y.clone().requires_grad_(True)
    gh, bh = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    out = BNClip.apply(yh, gh, bh, rm, rv, True, layout, dtype, 1)
    yr = y.float().clone().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    ref = R.clipped_relu(F.batch_norm(yr, None, None, gr, br, training=True, eps=BN_EPS))
    if layout == 1:
        ref = ref.permute(2, 0, 1, 3).reshape(T, N, C * Fd)
    dout = torch.randn_like(ref)
    out.backward(dout.to(dtype))
    ref.backward(dout)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert _rel(out, ref) < tol
    assert _rel(yh.grad, yr.grad) < tol * 3
    assert _rel(gh.grad, gr.grad) < tol * 3
    assert _rel(bh.grad, br.grad) < tol * 3
    # running stats updated with unbiased variance
    m = y.float().mean(dim=(0, 2, 3))
    assert torch.allclose(rm, 0.01 * m, atol=1e-3)


# --------------------------------------------------------------------------- optimizer
def test_adam_ema_matches_torch(cuda):
    from deepspeech_amd.ops.optim import ParamArena, FusedAdamEMA
    torch.manual_seed(0)

    def make(dev):
        torch.manual_seed(1)
        return torch.nn.Sequential(torch.nn.Linear(13, 7), torch.nn.Linear(7, 3)).to(dev)

    outs = []
    for dev in (torch.device("cpu"), cuda):
        m = make(dev)
        arena = ParamArena(m)
        opt = FusedAdamEMA(arena, ema_decay=0.99)
        g = torch.Generator().manual_seed(2)
        for step in range(5):
            arena.zero_grad()
            x = torch.randn(4, 13, generator=g).to(dev)
            m(x).pow(2).sum().backward()
            opt.step(lr=1e-2, global_step=step)
        outs.append((arena.flat.cpu(), opt.ema.cpu()))
    assert torch.allclose(outs[0][0], outs[1][0], atol=1e-5)
    assert torch.allclose(outs[0][1], outs[1][1], atol=1e-5)


@pytest.mark.parametrize("n", [1000003, 4096 * 37 + 3])
def test_adam_ema_launch_variants_bitwise(cuda, n):
    """The grid-strided and the block-contiguous Adam + EMA launches (csrc/optim.hip; the
    latter serves arenas past 120 M parameters) give bitwise the same p, m, v, ema and bf16
    copy, ragged tails included."""
    from deepspeech_amd.ops import _ext
    C = _ext.ext()
    torch.manual_seed(9)
    base = [torch.randn(n, device=cuda) for _ in range(5)]
    base[3].abs_()
    outs = []
    for grid in (0, 333, -7, -2048):
        p, g, m, v, e = (t.clone() for t in base)
        p16 = torch.empty(n, device=cuda, dtype=torch.bfloat16)
        C.adam_ema(p, g, m, v, e, p16, 1e-3, 0.9, 0.999, 1e-8, 0.5, 0.99, None, grid)
        outs.append((p, m, v, e, p16))
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert torch.equal(x, y)


def test_grad_norm(cuda):
    from deepspeech_amd.ops.optim import ParamArena, FusedAdamEMA
    m = torch.nn.Linear(100, 50).to(cuda)
    arena = ParamArena(m)
    arena.grad.normal_()
    opt = FusedAdamEMA(arena)
    n, bad = opt.grad_norm_and_finite(0.5)
    assert abs(float(n) - float(arena.grad.norm() * 0.5)) < 1e-3
    assert int(bad) == 0
    arena.grad[3] = float("nan")
    n, bad = opt.grad_norm_and_finite(1.0)
    assert int(bad) == 1


# --------------------------------------------------------------------------- greedy decode
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("T", [7, 300, 700])
def test_ctc_greedy_kernel(cuda, dtype, T):
    from deepspeech_amd.ops import decode as D
    torch.manual_seed(T)
    N, K = 9, 29
    logits = torch.randn(T, N, K, device=cuda) * 2
    # long runs of blanks / repeats so merging is exercised across 256-frame blocks
    logits[T // 3: T // 3 + 40, :, 28] += 10
    logits[T // 2: T // 2 + 300, :, 5] += 10
    logits = logits.to(dtype)
    lens = torch.randint(1, T + 1, (N,), dtype=torch.int32)
    lens[0] = T
    got, score = D.greedy_decode(logits, lens.to(cuda), with_scores=True)
    lp = torch.log_softmax(logits.float(), -1).cpu()
    want = R.greedy_decode(lp, lens)
    assert got == want
    ref_score = torch.stack([lp[: int(lens[n]), n].max(-1).values.sum() for n in range(N)])
    assert torch.allclose(score, ref_score, atol=1e-2, rtol=1e-4)


# --------------------------------------------------------------------------- fp8 quantisation
def test_fp8_quant2_matches_torch(cuda):
    """csrc/quant.hip per-tensor e4m3fn quantisation == the torch formulation (amax/448
    scale, saturating cast); x * (1/s) vs x / s may round a handful of values one fp8 step
    apart."""
    from deepspeech_amd.ops import _ext
    C = _ext.ext()
    torch.manual_seed(0)
    a = (torch.randn(1000, 136) * 3).bfloat16().to(cuda)
    b = (torch.randn(512, 136) * 0.02).bfloat16().to(cuda)
    b[3, 7] = 5.0                                   # an outlier sets b's scale
    f8 = torch.float8_e4m3fn
    a8 = torch.empty(a.shape, device=cuda, dtype=f8)
    b8 = torch.empty(b.shape, device=cuda, dtype=f8)
    nb = int(C.fp8_quant_blocks(a.numel(), b.numel()))
    ws = torch.empty(2 * nb + 2, device=cuda, dtype=torch.float32)
    C.fp8_quant2(a, b, 0.5, a8, b8, ws[:2 * nb], ws[2 * nb:])
    for x, x8, s_got, mul in ((a, a8, ws[2 * nb], 1.0), (b, b8, ws[2 * nb + 1], 0.5)):
        s = (x.float().abs().amax() / 448.0).clamp(min=1e-12)
        assert abs(float(s_got) - float(s) * mul) <= 1e-6 * float(s) * mul
        ref = (x.float() / s).clamp(-448, 448).to(f8).float()
        got = x8.float()
        bad = (got != ref)
        assert bad.float().mean().item() < 1e-3
        assert ((got - ref).abs()[bad] <= ref.abs()[bad] * 0.125 + 1e-6).all()


def test_fp8_quant2_direction_sum_is_torch_add_then_quant(cuda):
    """The quantiser's direction-sum form (operand a given as a + a2, an fp8 layer's two
    direction outputs): the bf16 sum it writes is bitwise torch.add, and the scales and e4m3
    copies are bitwise those of quantising that sum (ragged element count included)."""
    from deepspeech_amd.ops import _ext
    C = _ext.ext()
    torch.manual_seed(1)
    f8 = torch.float8_e4m3fn
    for rows, K, Kp in ((1000, 136, 256), (77, 1280, 1280)):
        ya = (torch.randn(rows, K) * 2).bfloat16().to(cuda)
        yb = (torch.randn(rows, K) * 2).bfloat16().to(cuda)
        w = (torch.randn(384, K) * 0.05).bfloat16().to(cuda)
        nb = int(C.fp8_quant_blocks(rows * Kp, 384 * Kp))
        outs = []
        for fused in (False, True):
            a8 = torch.empty(rows, Kp, device=cuda, dtype=f8)
            w8 = torch.empty(384, Kp, device=cuda, dtype=f8)
            ws = torch.empty(2 * nb + 2, device=cuda, dtype=torch.float32)
            if fused:
                s = torch.full((rows, K), float("nan"), device=cuda).bfloat16()
                C.fp8_quant2(ya, w, 0.5, a8, w8, ws[:2 * nb], ws[2 * nb:], yb, s)
            else:
                s = torch.add(ya, yb)
                C.fp8_quant2(s, w, 0.5, a8, w8, ws[:2 * nb], ws[2 * nb:])
            outs.append((s, a8.view(torch.uint8), w8.view(torch.uint8), ws[2 * nb:]))
        torch.cuda.synchronize()
        for x, y in zip(outs[0], outs[1]):
            assert torch.equal(x, y)


@pytest.mark.parametrize("cell", ["gru", "rnn_relu"])
def test_fused_direction_sum_bitwise(cuda, cell):
    """The gen-4 forward's in-kernel direction sum (one direction writes its bf16 value, the
    other adds) is bit-identical to y_fw + y_bw in bf16 via torch, variable lengths included."""
    from deepspeech_amd.ops import rnn as RNN
    torch.manual_seed(7)
    N, H, T = 32, 800, 57
    G = RNN.GATES[cell]
    lens = torch.randint(T // 3, T + 1, (N,), dtype=torch.int32)
    lens[0] = T
    gx = (torch.randn(T, N, 2 * G * H) * 0.5).bfloat16().to(cuda)
    Us = [(torch.randn(G * H, H) / math.sqrt(H)).bfloat16().to(cuda) for _ in range(2)]
    bh = [(torch.randn(G * H) * 0.1).to(cuda) if cell == "gru" else None for _ in range(2)]
    RNN._plan_cache.clear()
    plan = RNN.plan_for(N, H, cell, 2, cuda)
    assert plan.kind == "xcd"
    C = _ext_mod().ext()
    assert C.rnnx_fwd_fuses_sum(H, RNN.CELL_CODE[cell], plan.mt, 2, RNN.RNNX_KNOBS)
    old = RNN._FUSE_DIRSUM
    try:
        ys = []
        for fuse in (True, False):
            RNN._FUSE_DIRSUM = fuse
            y, _ = RNN._run_fwd(gx, lens.to(cuda), Us, bh, plan)
            torch.cuda.synchronize()
            RNN.check_errors()
            ys.append(y.clone())
    finally:
        RNN._FUSE_DIRSUM = old
    assert torch.equal(ys[0], ys[1])


def _ext_mod():
    from deepspeech_amd.ops import _ext
    return _ext


# --------------------------------------------------------------------------- fp8 recurrence
def test_fp8_quant_pow2(cuda):
    """csrc/rnn_fp8.hip per-tensor power-of-two e4m3 quantiser: the smallest 2^e with
    amax / 2^e <= 448, and every element the OCP e4m3 rounding of x / 2^e."""
    from deepspeech_amd.ops import _ext
    C = _ext.ext()
    torch.manual_seed(11)
    for scale in (0.02, 3.0, 900.0):
        x = (torch.randn(3 * 256, 256, device=cuda) * scale).to(torch.bfloat16)
        q = torch.empty(x.shape, device=cuda, dtype=torch.uint8)
        w = torch.empty(2, device=cuda, dtype=torch.int32)
        C.fp8_quant_pow2(x, q, w[0:1], w[1:2])
        e = int(w[0]) - 127
        amax = float(x.float().abs().max())
        assert amax / 2.0 ** e <= 448.0 and amax / 2.0 ** (e - 1) > 448.0
        want = (x.float() / 2.0 ** e).to(torch.float8_e4m3fn).view(torch.uint8)
        assert float((q != want).float().mean()) == 0.0


@pytest.mark.parametrize("H,ndir", [(256, 2), (1280, 2), (1280, 1)])
def test_fp8_quant_u_both_layouts(cuda, H, ndir):
    """csrc/rnn_fp8.hip quant_u_kernel (the fp8 layers' U, both directions, one read): the
    row-major and transposed e4m3 copies and each direction's exponent equal the per-tensor
    quantiser's, bitwise; either layout alone gives the same bytes."""
    from deepspeech_amd.ops import _ext
    C = _ext.ext()
    torch.manual_seed(H + ndir)
    U = [(torch.randn(3 * H, H, device=cuda) * s).to(torch.bfloat16) for s in (0.05, 7.0)[:ndir]]
    q = torch.empty(ndir, 3 * H, H, device=cuda, dtype=torch.uint8)
    qt = torch.empty(ndir, H, 3 * H, device=cuda, dtype=torch.uint8)
    uexp = torch.empty(ndir, device=cuda, dtype=torch.int32)
    part = torch.empty(ndir * 256, device=cuda)
    C.fp8_quant_u(U[0], U[1] if ndir == 2 else None, q, qt, uexp, part)
    q2 = torch.empty_like(q)
    C.fp8_quant_u(U[0], U[1] if ndir == 2 else None, q2, None, uexp, part)
    assert torch.equal(q, q2)
    for d in range(ndir):
        ref = torch.empty(3 * H, H, device=cuda, dtype=torch.uint8)
        w = torch.empty(2, device=cuda, dtype=torch.int32)
        C.fp8_quant_pow2(U[d], ref, w[0:1], w[1:2])
        assert int(uexp[d]) == int(w[0])
        assert torch.equal(q[d], ref)
        assert torch.equal(qt[d], ref.t().contiguous())


def _gru_fp8_emulation(gx, lens, U, bh, H):
    """fp32 model of csrc/rnn_fp8.hip: U quantised to e4m3 with a power-of-two scale, h_{t-1}
    requantised to e4m3 every step for the recurrent product, the cell in fp32."""
    T, N, _ = gx.shape
    ndir = len(U)
    ys, hss = [], []
    for d in range(ndir):
        u = U[d].float()
        e = math.ceil(math.log2(float(u.abs().max()) / 448.0))
        if float(u.abs().max()) / 2.0 ** e > 448.0:
            e += 1
        uq = (u / 2.0 ** e).to(torch.float8_e4m3fn).float() * 2.0 ** e
        h = torch.zeros(N, H, device=gx.device)
        y = torch.zeros(T, N, H, device=gx.device)
        hs = []
        for s in range(T):
            t = torch.tensor([s if d == 0 else max(int(lens[b]) - 1 - s, 0) for b in range(N)], device=gx.device)
            act = torch.tensor([s < int(lens[b]) for b in range(N)], device=gx.device)
            g = gx[t, torch.arange(N, device=gx.device), d * 3 * H:(d + 1) * 3 * H].float()
            gh = h.to(torch.float8_e4m3fn).float() @ uq.t() + bh[d].float()
            r = torch.sigmoid(g[:, :H] + gh[:, :H])
            z = torch.sigmoid(g[:, H:2 * H] + gh[:, H:2 * H])
            n = torch.tanh(g[:, 2 * H:] + r * gh[:, 2 * H:])
            hn = (1 - z) * n + z * h
            h = torch.where(act[:, None], hn, h)
            tt = torch.where(act, t, torch.full_like(t, s))
            y[tt, torch.arange(N, device=gx.device)] = torch.where(act[:, None], hn, torch.zeros_like(hn))
            hs.append(h.clone())
        ys.append(y)
        hss.append(torch.stack(hs))
    return sum(ys), hss


@pytest.mark.parametrize("N,H,ndir", [(8, 1280, 2), (20, 1024, 2), (8, 1280, 1), (32, 1280, 2)])
def test_fp8_recurrence_matches_emulation(cuda, N, H, ndir):
    """The fp8 GRU forward (e4m3 U and h exchange, 8 groups of H/64 workgroups) against an
    fp32 emulation of the same quantisation: outputs and saved states within 2 %, padding
    positions exactly zero, bf16 h copy = the fp32 state rounded."""
    from deepspeech_amd.ops import rnn as RNN
    torch.manual_seed(N + H)
    T = 19
    plan = RNN.plan_for(N, H, "gru", ndir, cuda)
    if not RNN.fp8_recurrence_ok(plan, N):
        # (32, 1280, 2) is config 5's production geometry (8 rows per group): it must run
        assert (N, H) != (32, 1280), "config 5 geometry not served by the fp8 recurrence"
        pytest.skip("geometry not served by the fp8 recurrence (plan rows)")
    gx = (torch.randn(T, N, ndir * 3 * H, device=cuda) * 0.5).to(torch.bfloat16)
    lens = torch.randint(T // 2, T + 1, (N,), device=cuda, dtype=torch.int32)
    lens[0] = T
    U = [(torch.randn(3 * H, H, device=cuda) * (1.5 / H ** 0.5)).to(torch.bfloat16) for _ in range(ndir)]
    bh = [torch.randn(3 * H, device=cuda) * 0.1 for _ in range(ndir)]
    y, (hx, hs, gates) = RNN._run_fwd_fp8(gx, lens, U, bh + [None] * (2 - ndir), plan)
    torch.cuda.synchronize()
    RNN.check_errors()
    yr, hsr = _gru_fp8_emulation(gx, lens, U, bh, H)
    assert _rel(y.float(), yr) < 2e-2, _rel(y.float(), yr)
    for d in range(ndir):
        assert _rel(hs[d, 1:, :N], hsr[d]) < 2e-2
        assert torch.equal(hx[d, 1:, :N], hs[d, 1:, :N].to(torch.bfloat16))
    for b in range(N):
        L = int(lens[b])
        if L < T:
            assert float(y[L:, b].abs().max()) == 0.0


def _e4m3_pow2(x, amax):
    """x / 2^e rounded to e4m3, times 2^e, with the smallest e such that amax / 2^e <= 448
    (per-element amax tensor broadcast against x; amax 0 -> e = 0)."""
    am = amax.clamp_min(1e-30)
    e = torch.ceil(torch.log2(am / 448.0))
    e = torch.where(am / torch.exp2(e) > 448.0, e + 1, e)
    e = torch.where(am / torch.exp2(e - 1) <= 448.0, e - 1, e)
    e = torch.where(amax > 0, e, torch.zeros_like(e))
    return (x / torch.exp2(e)).to(torch.float8_e4m3fn).float() * torch.exp2(e)


def _gru_bptt_fp8_emulation(dy, lens, U, hs, gates, H, ndir):
    """fp32 model of csrc/rnn_fp8.hip rnnf8_bwd_kernel on the forward's saved states: U^T in
    e4m3 with the per-tensor power-of-two scale, the gate gradients requantised to e4m3 every
    step with one power-of-two scale per (row, 32-unit group) shared by the three gates; dgh /
    dgx exact."""
    T, N, _ = dy.shape
    P = H // 64
    dgx = torch.zeros(T, N, ndir * 3 * H, device=dy.device)
    dghs = []
    ar = torch.arange(N, device=dy.device)
    for d in range(ndir):
        u = U[d].float()
        uq = _e4m3_pow2(u, u.abs().max())
        carry = torch.zeros(N, H, device=dy.device)
        dhrec = torch.zeros(N, H, device=dy.device)
        dgh = torch.zeros(T, N, 3 * H, device=dy.device)
        for s in range(T - 1, -1, -1):
            act = torch.tensor([s < int(lens[b]) for b in range(N)], device=dy.device)
            t = torch.tensor([s if d == 0 else max(int(lens[b]) - 1 - s, 0) for b in range(N)], device=dy.device)
            dh = torch.where(act[:, None], dy[t, ar].float(), 0.0) + carry + dhrec
            g = gates[d, s, :N].float()
            r, z, n, ghn = g[..., 0], g[..., 1], g[..., 2], g[..., 3]
            hp = hs[d, s, :N].float()
            dn = dh * (1 - z)
            dz = dh * (hp - n)
            dan = dn * (1 - n * n)
            dr = dan * ghn
            ghv = torch.cat([dr * r * (1 - r), dz * z * (1 - z), dan * r], 1) * act[:, None]
            gxs = torch.cat([ghv[:, :2 * H], dan * act[:, None]], 1)
            carry = torch.where(act[:, None], dh * z, 0.0)
            dgh[s] = ghv
            tt = torch.where(act, t, torch.full_like(t, s))
            dgx[tt, ar, d * 3 * H:(d + 1) * 3 * H] = gxs
            blk = ghv.abs().view(N, 3, H // 32, 32).amax(dim=(1, 3), keepdim=True)
            am = blk.expand(N, 3, H // 32, 32).reshape(N, 3 * H)
            dhrec = _e4m3_pow2(ghv, am) @ uq
        dghs.append(dgh)
    return dgx, dghs


@pytest.mark.parametrize("N,H,ndir", [(8, 256, 2), (32, 1280, 2), (20, 1024, 2), (8, 1280, 1)])
def test_fp8_bptt_matches_emulation(cuda, N, H, ndir):
    """The fp8 GRU BPTT (csrc/rnn_fp8.hip rnnf8_bwd_kernel: groups of H/64 workgroups on one XCD,
    e4m3 U^T, per-(row, workgroup) e4m3 gate gradients, tagged-bf16 reduce-scatter) on the saved
    states of the fp8 forward, against an fp32 emulation of the same quantisation: dgx, dgh and
    the bias partials within 3 %, padding exactly zero. (32, 1280, 2) is config 5's production
    geometry."""
    from deepspeech_amd.ops import rnn as RNN
    torch.manual_seed(7 * N + H)
    T = 19
    plan = RNN.plan_for(N, H, "gru", ndir, cuda)
    ok = RNN.fp8_bptt_ok(plan, N)
    if (N, H, ndir) == (32, 1280, 2):
        assert ok, "config 5 geometry not served by the fp8 BPTT"
    if not ok:
        pytest.skip("geometry not served by the fp8 BPTT")
    gx = (torch.randn(T, N, ndir * 3 * H, device=cuda) * 0.5).to(torch.bfloat16)
    lens = torch.randint(T // 2, T + 1, (N,), device=cuda, dtype=torch.int32)
    lens[0] = T
    U = [(torch.randn(3 * H, H, device=cuda) * (1.5 / H ** 0.5)).to(torch.bfloat16) for _ in range(ndir)]
    bh = [torch.randn(3 * H, device=cuda) * 0.1 for _ in range(ndir)]
    y, (hx, hs, gates) = RNN._run_fwd_fp8(gx, lens, U, bh + [None] * (2 - ndir), plan)
    dy = torch.randn(T, N, H, device=cuda).to(torch.bfloat16)
    for b in range(N):
        dy[int(lens[b]):, b] = 0
    dgx, dgh, parts = RNN._run_bwd_fp8(dy, lens, U + [None] * (2 - ndir), hs, gates, plan, ndir * 3 * H)
    torch.cuda.synchronize()
    RNN.check_errors()
    dgx_r, dgh_r = _gru_bptt_fp8_emulation(dy, lens, U, hs, gates, H, ndir)
    assert _rel(dgx.float(), dgx_r) < 3e-2, _rel(dgx.float(), dgx_r)
    for d in range(ndir):
        assert _rel(dgh[d, :, :N].float(), dgh_r[d]) < 3e-2, (d, _rel(dgh[d, :, :N].float(), dgh_r[d]))
        assert float(dgh[d, :, N:].float().abs().max() if dgh.shape[2] > N else 0) == 0.0
        db = parts[0, d].sum(0)
        assert _rel(db, dgx_r[..., d * 3 * H:(d + 1) * 3 * H].sum((0, 1))) < 3e-2
    for b in range(N):
        L = int(lens[b])
        if L < T:
            assert float(dgx[L:, b].abs().max()) == 0.0
    # and close to the bf16 reduce-scatter BPTT on the same states (quantisation only)
    if plan.kind == "xcd":
        dgx16, _, _ = RNN._run_bwd(dy, lens, U + [None] * (2 - ndir), hx, hs, gates, plan, ndir * 3 * H)
        torch.cuda.synchronize()
        assert _rel(dgx.float(), dgx16.float()) < 8e-2, _rel(dgx.float(), dgx16.float())


def test_multi_copy_rows_padding_and_scalars(cuda):
    """csrc/fill.hip multi_copy: row copies into wider rows (rest of each row zeroed), 1-D
    copies of several dtypes and the fp32 scalar slot, all in one launch (graph-replay inputs)."""
    from deepspeech_amd.ops import _ext
    C = _ext.ext()
    torch.manual_seed(2)
    f_src = torch.randn(3 * 7 * 5, device=cuda)
    f_dst = torch.full_like(f_src, float("nan"))
    lab_src = torch.randint(1, 28, (6, 9), device=cuda, dtype=torch.int32)
    lab_dst = torch.full((6, 16), -1, device=cuda, dtype=torch.int32)
    l_src = torch.randint(0, 100, (6,), device=cuda, dtype=torch.int32)
    l_dst = torch.zeros_like(l_src)
    h_src = torch.randn(40, device=cuda).bfloat16()
    h_dst = torch.zeros_like(h_src)
    hyper = torch.zeros(2, device=cuda)
    C.multi_copy([f_dst, lab_dst, l_dst, h_dst], [f_src, lab_src, l_src, h_src], hyper, [1e-3 / 3, 0.9999])
    torch.cuda.synchronize()
    assert torch.equal(f_dst, f_src) and torch.equal(l_dst, l_src) and torch.equal(h_dst, h_src)
    assert torch.equal(lab_dst[:, :9], lab_src) and bool((lab_dst[:, 9:] == 0).all())
    assert torch.equal(hyper.cpu(), torch.tensor([1e-3 / 3, 0.9999], dtype=torch.float32))


def test_prep_inputs_matches_torch(cuda):
    """csrc/fill.hip prep_inputs: fp32 -> bf16 features bitwise torch's cast (ragged tail
    included) and the recurrence lengths bitwise ops/reference.py get_rnn_seqlen (negative
    and non-multiple-of-4 lengths included)."""
    from deepspeech_amd.ops import _ext
    from deepspeech_amd.ops import reference as R
    torch.manual_seed(3)
    x = torch.randn(3, 101, 161, device=cuda) * 7
    y = torch.empty(x.shape, device=cuda, dtype=torch.bfloat16)
    lens = torch.tensor([0, 1, 33, 34, 35, 37, 38, 1000, 999], device=cuda, dtype=torch.int32)
    out = torch.empty_like(lens)
    _ext.ext().prep_inputs(x, y, lens, out)
    torch.cuda.synchronize()
    assert torch.equal(y, x.to(torch.bfloat16))
    assert torch.equal(out, R.get_rnn_seqlen(lens))
