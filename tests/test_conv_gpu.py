"""Conv front-end MFMA kernels (csrc/conv_frontend.hip) against plain-PyTorch fp32 references.

Each kernel is checked on its own (conv1/conv2 forward, conv2 data gradient, conv1/conv2
weight gradients, channels-last BatchNorm statistics/apply/backward), then the whole
FrontendCL autograd function against the reference engine's front-end
(src/deepSpeech_NCHW.py:110-168 semantics: conv + bias + train-mode BN + clip(0, 20),
time-major [T2, N, C*F2] output).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _geom(T, F0=161):
    T1, F1 = (T - 20) // 2 + 1, (F0 - 5) // 2 + 1
    return T1, F1, (T1 - 10) // 2 + 1, F1 - 4


@pytest.mark.parametrize("N,T", [(2, 137), (3, 100), (1, 61)])
def test_conv1_fwd_and_stats(cuda, N, T):
    from deepspeech_amd.ops import _ext
    C_ = _ext.ext()
    torch.manual_seed(N * 1000 + T)
    T1, F1, _, _ = _geom(T)
    x = torch.randn(N, T, 161, device=cuda).bfloat16()
    w = (torch.randn(32, 1, 20, 5, device=cuda) * 0.1).bfloat16()
    b = torch.randn(32, device=cuda) * 0.1
    y = torch.empty(N, T1, F1, 32, device=cuda, dtype=torch.bfloat16)
    nb = int(C_.conv1_fwd_grid(N, T1))
    part = torch.empty(nb * 64, device=cuda)
    C_.conv1_fwd(x, w, b, y, part)
    ref = F.conv2d(x.float().unsqueeze(1), w.float(), b, stride=(2, 2)).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2, _rel(y, ref)
    mean = torch.empty(32, device=cuda)
    inv = torch.empty(32, device=cuda)
    C_.bn_cl_finalize(part, nb, float(N * T1 * F1), 1e-3, mean, inv, None, None, 0.0)
    yf = y.float().reshape(-1, 32)
    assert torch.allclose(mean, yf.mean(0), atol=1e-3, rtol=1e-3)
    assert torch.allclose(inv, torch.rsqrt(yf.var(0, unbiased=False) + 1e-3), atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("N,T", [(2, 137), (3, 100), (1, 61)])
def test_conv2_fwd_and_stats(cuda, N, T):
    from deepspeech_amd.ops import _ext
    C_ = _ext.ext()
    torch.manual_seed(7 + N * T)
    T1, F1, T2, F2 = _geom(T)
    x = torch.rand(N, T1, F1, 32, device=cuda).bfloat16()
    w = (torch.randn(32, 32, 10, 5, device=cuda) * 0.05).bfloat16()
    b = torch.randn(32, device=cuda) * 0.1
    y = torch.empty(N, T2, F2, 32, device=cuda, dtype=torch.bfloat16)
    for grid in (7, 64):
        part = torch.empty(grid * 64, device=cuda)
        y.zero_()
        C_.conv2_fwd(x, w, b, y, part, grid)
        ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), b, stride=(2, 1)).permute(0, 2, 3, 1)
        assert _rel(y, ref) < 1e-2, (grid, _rel(y, ref))
        mean = torch.empty(32, device=cuda)
        inv = torch.empty(32, device=cuda)
        C_.bn_cl_finalize(part, grid, float(N * T2 * F2), 1e-3, mean, inv, None, None, 0.0)
        yf = y.float().reshape(-1, 32)
        assert torch.allclose(mean, yf.mean(0), atol=1e-3, rtol=1e-3)
        assert torch.allclose(inv, torch.rsqrt(yf.var(0, unbiased=False) + 1e-3), atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("N,T", [(2, 137), (1, 61), (2, 62)])
def test_conv2_dgrad_wgrad(cuda, N, T):
    from deepspeech_amd.ops import _ext
    C_ = _ext.ext()
    torch.manual_seed(11 + T)
    T1, F1, T2, F2 = _geom(T)
    x = torch.rand(N, T1, F1, 32, device=cuda).bfloat16()
    w = (torch.randn(32, 32, 10, 5, device=cuda) * 0.05).bfloat16()
    dy = torch.randn(N, T2, F2, 32, device=cuda).bfloat16()
    xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    wr = w.float().clone().requires_grad_(True)
    out = F.conv2d(xr, wr, None, stride=(2, 1))
    out.backward(dy.float().permute(0, 3, 1, 2))
    # conv1's BN state for the fused BN-backward sums of the dgrad epilogue
    y1 = (torch.randn(N, T1, F1, 32, device=cuda) * 2).bfloat16()
    mean, inv = torch.randn(32, device=cuda) * 0.3, torch.rand(32, device=cuda) + 0.5
    gamma, beta = torch.randn(32, device=cuda), torch.randn(32, device=cuda)
    for grid in (5, 64, 512):
        dx = torch.full((N, T1, F1, 32), float("nan"), device=cuda).bfloat16()
        C_.conv2_dgrad(dy, w, dx, grid)
        assert _rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2, ("dx", grid)
        part = torch.full((grid * 64,), float("nan"), device=cuda)
        dx2 = torch.empty_like(dx)
        C_.conv2_dgrad(dy, w, dx2, grid, y1, mean, inv, gamma, beta, part)
        assert torch.equal(dx2, dx)
        outs = []
        for ready in (True, False):
            dg, db = torch.empty(32, device=cuda), torch.empty(32, device=cuda)
            dyb = torch.empty_like(dx)
            p2 = part.clone() if ready else torch.empty(1024 * 64, device=cuda)
            C_.bn_cl_bwd(dx, y1, mean, inv, gamma, beta, p2, grid if ready else 64, dg, db, dyb, False,
                         part_ready=ready)
            outs.append((dg, db, dyb))
        for a_, b_ in zip(outs[0], outs[1]):
            assert _rel(a_, b_) < 1e-4, ("fused BN sums", grid, _rel(a_, b_))
        part = torch.empty(int(C_.conv2_wgrad_part_floats(grid)), device=cuda)
        dw = torch.full((32, 32, 10, 5), float("nan"), device=cuda)
        C_.conv2_wgrad(dy, x, part, dw, grid)
        assert _rel(dw, wr.grad) < 1e-2, ("dw", grid, _rel(dw, wr.grad))


@pytest.mark.parametrize("N,T", [(2, 137), (1, 61)])
def test_conv1_wgrad(cuda, N, T):
    from deepspeech_amd.ops import _ext
    C_ = _ext.ext()
    torch.manual_seed(5 + T)
    T1, F1, _, _ = _geom(T)
    x = torch.randn(N, T, 161, device=cuda).bfloat16()
    dy = torch.randn(N, T1, F1, 32, device=cuda).bfloat16()
    wr = torch.zeros(32, 1, 20, 5, device=cuda, requires_grad=True)
    F.conv2d(x.float().unsqueeze(1), wr, None, stride=(2, 2)).backward(dy.float().permute(0, 3, 1, 2))
    for grid in (3, 64):
        part = torch.empty(int(C_.conv1_wgrad_part_floats(grid)), device=cuda)
        dw = torch.full((32, 1, 20, 5), float("nan"), device=cuda)
        C_.conv1_wgrad(dy, x, part, dw, grid)
        assert _rel(dw, wr.grad) < 1e-2, ("dw1", grid, _rel(dw, wr.grad))
    # the BatchNorm backward applied inside the staging: bitwise the weight gradient of the
    # apply pass's dy (dz and y1 as conv1's BN sees them; sums from the reduce pass)
    y1 = (torch.randn(N, T1, F1, 32, device=cuda) * 3 + 1).bfloat16()
    dz = dy
    yf = y1.float().reshape(-1, 32)
    mean = yf.mean(0).contiguous()
    inv = torch.rsqrt(yf.var(0, unbiased=False) + 1e-3).contiguous()
    gamma, beta = torch.rand(32, device=cuda) + 0.5, torch.randn(32, device=cuda) * 0.3
    bpart = torch.empty(64 * 64, device=cuda)
    dg, db = torch.empty(32, device=cuda), torch.empty(32, device=cuda)
    dy_bn = torch.empty_like(dz)
    C_.bn_cl_bwd(dz, y1, mean, inv, gamma, beta, bpart, 64, dg, db, dy_bn, False)
    dg2, db2 = torch.empty(32, device=cuda), torch.empty(32, device=cuda)
    C_.bn_cl_bwd(dz, y1, mean, inv, gamma, beta, bpart, 64, dg2, db2, dz, False, part_ready=2)
    assert torch.equal(dg, dg2) and torch.equal(db, db2)
    for grid in (3, 64):
        part = torch.empty(int(C_.conv1_wgrad_part_floats(grid)), device=cuda)
        dw_a = torch.full((32, 1, 20, 5), float("nan"), device=cuda)
        dw_b = torch.full((32, 1, 20, 5), float("nan"), device=cuda)
        C_.conv1_wgrad(dy_bn, x, part, dw_a, grid)
        C_.conv1_wgrad(dz, x, part, dw_b, grid, y1, mean, inv, gamma, beta, db, dg)
        assert torch.equal(dw_a, dw_b), ("fused BN backward", grid, (dw_a - dw_b).abs().max())


@pytest.mark.parametrize("tmaj", [False, True])
def test_bn_cl_apply_bwd(cuda, tmaj):
    from deepspeech_amd.ops import _ext
    C_ = _ext.ext()
    torch.manual_seed(3)
    N, T, Fd = 3, 17, 75 if tmaj else 79
    y = (torch.randn(N, T, Fd, 32, device=cuda) * 3 + 1).bfloat16()
    gamma = torch.rand(32, device=cuda) + 0.5
    beta = torch.randn(32, device=cuda) * 0.3
    yf = y.float().reshape(-1, 32)
    mean = yf.mean(0).contiguous()
    inv = torch.rsqrt(yf.var(0, unbiased=False) + 1e-3).contiguous()
    out = torch.empty(T, N, 32 * Fd, device=cuda, dtype=torch.bfloat16) if tmaj else torch.empty_like(y)
    C_.bn_cl_apply(y, mean, inv, gamma, beta, out, tmaj)
    # reference in NCHW
    yr = y.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    g_r = gamma.clone().requires_grad_(True)
    b_r = beta.clone().requires_grad_(True)
    z = F.batch_norm(yr, None, None, g_r, b_r, training=True, eps=1e-3).clamp(0, 20)
    zr = z.permute(2, 0, 1, 3).reshape(T, N, -1) if tmaj else z.permute(0, 2, 3, 1)
    assert _rel(out, zr) < 1e-2
    dz = torch.randn_like(zr).bfloat16()
    zr.backward(dz.float())
    nb = 13
    part = torch.empty(nb * 64, device=cuda)
    dg = torch.empty(32, device=cuda)
    db = torch.empty(32, device=cuda)
    dy = torch.empty_like(y)
    C_.bn_cl_bwd(dz.contiguous(), y, mean, inv, gamma, beta, part, nb, dg, db, dy, tmaj)
    assert _rel(db, b_r.grad) < 1e-2, "dbeta"
    assert _rel(dg, g_r.grad) < 1e-2, "dgamma"
    assert _rel(dy, yr.grad.permute(0, 2, 3, 1)) < 2e-2, ("dy", _rel(dy, yr.grad.permute(0, 2, 3, 1)))


@pytest.mark.parametrize("N,T", [(3, 137), (2, 100)])
def test_frontend_cl_matches_reference(cuda, N, T):
    from deepspeech_amd.models import DeepSpeech2
    torch.manual_seed(0)
    ref = DeepSpeech2(num_filters=32, num_hidden=64, num_rnn_layers=1, cell="gru").to(cuda)
    hip = DeepSpeech2(num_filters=32, num_hidden=64, num_rnn_layers=1, cell="gru").to(cuda)
    hip.load_state_dict(ref.state_dict())
    hip.set_engine("hip", torch.bfloat16)
    # the same front-end through the library-conv bf16 path (the pre-existing HIP-engine
    # path): its error against fp32 is the precision floor of a bf16 activation chain
    lib = DeepSpeech2(num_filters=32, num_hidden=64, num_rnn_layers=1, cell="gru").to(cuda)
    lib.load_state_dict(ref.state_dict())
    lib.set_engine("hip", torch.bfloat16)
    feats = torch.randn(N, T, 161, device=cuda)
    xr = ref.frontend(feats)
    xh = hip.frontend(feats.bfloat16())
    import os
    os.environ["DS2_CONV"] = "lib"
    try:
        xl = lib.frontend(feats.bfloat16())
    finally:
        os.environ.pop("DS2_CONV")
    assert xh.shape == xr.shape and xh.dtype == torch.bfloat16
    assert _rel(xh, xr) < 3e-2, _rel(xh, xr)
    g = torch.randn_like(xr)
    xr.backward(g)
    xh.backward(g.bfloat16())
    xl.backward(g.bfloat16())
    for name in ("conv1.weight", "conv1.bn_gamma", "conv1.bn_beta", "conv2.weight", "conv2.bn_gamma",
                 "conv2.bn_beta"):
        pr = dict(ref.named_parameters())[name].grad
        ph = dict(hip.named_parameters())[name].grad
        pl = dict(lib.named_parameters())[name].grad
        assert ph is not None, name
        floor = _rel(pl, pr)
        assert _rel(ph, pr) < max(5e-2, 1.5 * floor), (name, _rel(ph, pr), floor)
    # conv biases feed train-mode BN: their gradient is zero
    assert float(dict(hip.named_parameters())["conv2.bias"].grad.abs().max()) == 0.0
    # running statistics follow the reference update
    for blk in ("conv1", "conv2"):
        rm_r = getattr(ref, blk).running_mean
        rm_h = getattr(hip, blk).running_mean
        assert torch.allclose(rm_h, rm_r, atol=2e-3, rtol=2e-2), blk
