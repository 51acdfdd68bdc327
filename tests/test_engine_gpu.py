"""Whole-model parity of the HIP engine against the pure-PyTorch fp32 reference engine.

Covers the fused layer path end to end: bf16 weight shadows read from the arena, the
single [W_fw; W_bw] projection GEMM, in-kernel bias-gradient sums, weight gradients
written straight into the fp32 gradient arena (``main_grad``), fused head / conv / BN.
"""
import copy

import pytest
import torch

from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
from deepspeech_amd.models import DeepSpeech2
from deepspeech_amd.ops.optim import ParamArena

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _pair(cuda, cell, H, L, seq_bn="frozen", C=32):
    """fp32 reference engine + HIP engine copies. C = 32 filters: the hand-written
    channels-last conv kernels (other widths take the library-conv path)."""
    torch.manual_seed(11)
    ref = DeepSpeech2(num_filters=C, num_hidden=H, num_rnn_layers=L, cell=cell, seq_bn=seq_bn).to(cuda)
    hip = copy.deepcopy(ref)
    ref.set_engine("ref", torch.float32)
    hip.set_engine("hip", torch.bfloat16)
    return ref, hip


def _loss(model, batch, fused=False):
    model.train()
    if fused:
        return model.forward_loss(batch["feats"], batch["seq_lens"], batch["labels"], batch["label_lens"])
    logits, lens = model(batch["feats"], batch["seq_lens"])
    return model.loss(logits, lens, batch["labels"], batch["label_lens"])


def _compare_grads(ref, hip, lh, lr, cell, tol_rnn=0.06, tol_conv=None, tol_names=None):
    assert abs(float(lh) - float(lr)) / abs(float(lr)) < 3e-2, (float(lh), float(lr))
    gref = dict((n, p.grad) for n, p in ref.named_parameters())
    errs, bad = {}, []
    for n, p in hip.named_parameters():
        g = p.grad
        assert g is not None, n
        gr = gref[n]
        if n.endswith("conv1.bias") or n.endswith("conv2.bias"):
            # identically zero under train-mode BN (reference has only rounding noise)
            errs[n] = float(g.abs().max())
            if errs[n] > 1e-6:
                bad.append(n)
            continue
        errs[n] = round(_rel(g, gr), 5)
        # bf16 activations end to end: the conv front-end sits below every recurrent
        # layer, so its gradients carry the most accumulated rounding
        # (ReLU-RNN: bf16 rounding also flips clip masks, so the front-end sees more)
        tol = (tol_conv or (0.12 if cell == "gru" else 0.2)) if n.startswith("conv") else tol_rnn
        tol = (tol_names or {}).get(n, tol)
        if errs[n] > tol:
            bad.append(n)
    worst = ", ".join("%s %.4f" % kv for kv in sorted(errs.items(), key=lambda kv: -kv[1])[:12])
    assert not bad, "loss hip %.5f ref %.5f; over tolerance: %s; worst: %s" % (float(lh), float(lr), bad, worst)
    return errs


@pytest.mark.parametrize("cell", ["gru", "rnn_relu"])
@pytest.mark.parametrize("use_arena,fused", [(True, True), (True, False), (False, True)])
def test_model_grads_match_reference(cuda, cell, use_arena, fused):
    """fused=True: the training path (FC head + CTC fused, ops/ctc.py FusedHeadCTC);
    fused=False: forward() logits (fc_logits kernel) + the standalone fused CTC."""
    from deepspeech_amd.ops import rnn as RNN
    ref, hip = _pair(cuda, cell, H=64, L=2)
    batch = to_device(FixedShapeBatches(6, max_frames=260, seed=3, pool=1).next(), cuda)
    arena = ParamArena(hip, bf16_shadow=True) if use_arena else None
    if arena is not None:
        arena.zero_grad()
    lh = _loss(hip, batch, fused)
    lh.backward()
    if arena is not None:
        RNN.join_wgrad_streams()
    lr = _loss(ref, batch)
    lr.backward()
    torch.cuda.synchronize()
    RNN.check_errors()
    _compare_grads(ref, hip, lh, lr, cell)


@pytest.mark.parametrize("cell", ["gru", "rnn_relu"])
def test_headline_geometry_matches_reference(cuda, cell):
    """The headline shape end to end (32 filters, H=800, 5 layers, batch 32, 10-s
    utterances): HIP engine (bf16, every hand-written kernel, arena + side streams) vs the
    fp32 reference engine. The per-parameter relative errors are in the assert message."""
    from deepspeech_amd.ops import rnn as RNN
    ref, hip = _pair(cuda, cell, H=800, L=5)
    batch = to_device(FixedShapeBatches(32, max_frames=1000, seed=5, pool=1).next(), cuda)
    arena = ParamArena(hip, bf16_shadow=True)
    arena.zero_grad()
    lh = _loss(hip, batch, True)
    lh.backward()
    RNN.join_wgrad_streams()
    lr = _loss(ref, batch)
    lr.backward()
    torch.cuda.synchronize()
    RNN.check_errors()
    # Per-parameter bounds at ~1.5x the errors measured on MI355X (round 6, fixed seeds, bitwise
    # reproducible engine), so a 2x regression of any one gradient fails. GRU: every recurrent /
    # FC parameter <= 1.06 %; the conv front-end under 5 bf16 layers of rounding conv1.bn_beta
    # 13.1 % (a sum over 1.2 M positions with cancellation), conv1.weight 7.2 %, conv2.weight
    # 5.1 %, conv1.bn_gamma 4.2 %, conv2.bn_* 0.8 %. Clipped-ReLU RNN (loss ~2.8e4 at this random
    # init, bf16 rounding flips clip masks at 20 in every layer): recurrent <= 1.92 %,
    # conv1.weight 23.1 %, conv1.bn_beta 21.0 %, conv1.bn_gamma 16.6 %, conv2.weight 16.1 %.
    if cell == "gru":
        names = {"conv1.bn_beta": 0.20, "conv1.weight": 0.11, "conv2.weight": 0.08, "conv1.bn_gamma": 0.065,
                 "conv2.bn_beta": 0.015, "conv2.bn_gamma": 0.015}
        errs = _compare_grads(ref, hip, lh, lr, cell, tol_rnn=0.016, tol_conv=0.2, tol_names=names)
    else:
        names = {"conv1.weight": 0.35, "conv1.bn_beta": 0.32, "conv1.bn_gamma": 0.25, "conv2.weight": 0.25,
                 "conv2.bn_beta": 0.015, "conv2.bn_gamma": 0.015}
        errs = _compare_grads(ref, hip, lh, lr, cell, tol_rnn=0.03, tol_conv=0.35, tol_names=names)
    print("headline %s relative gradient errors:" % cell,
          ", ".join("%s %.4f" % kv for kv in sorted(errs.items(), key=lambda kv: -kv[1])))


@pytest.mark.parametrize("cell,H", [("gru", 1280), ("rnn_relu", 1760)])
def test_wide_layer_models_match_reference(cuda, cell, H):
    """Engine-level parity of the wide-layer configurations: BASELINE config 5's BiGRU-1280
    and the reference's own 1760-unit clipped-ReLU stack (src/train.sh:42), two layers each,
    batch 32 (the plans, GEMM routes and recurrence kernels of those geometries)."""
    from deepspeech_amd.ops import rnn as RNN
    ref, hip = _pair(cuda, cell, H=H, L=2)
    batch = to_device(FixedShapeBatches(32, max_frames=600, seed=8, pool=1).next(), cuda)
    arena = ParamArena(hip, bf16_shadow=True)
    arena.zero_grad()
    lh = _loss(hip, batch, True)
    lh.backward()
    RNN.join_wgrad_streams()
    lr = _loss(ref, batch)
    lr.backward()
    torch.cuda.synchronize()
    RNN.check_errors()
    _compare_grads(ref, hip, lh, lr, cell, tol_rnn=0.06, tol_conv=0.15 if cell == "gru" else 0.35)


class _RoundGrad(torch.autograd.Function):
    """Identity forward; backward rounds the incoming gradient to bf16 (a kernel that
    stores that gradient in bf16)."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def _st_round(t):
    """Value rounded to bf16 (a bf16 activation store), gradient passed straight through."""
    return t + (t.to(torch.bfloat16).to(t.dtype) - t).detach()


def _frontend_emulated(model, feats, dout, dbeta_mass=None):
    """float64 reference of the channels-last HIP front-end (ops/frontend.py FrontendCL) that
    stores what the kernels store in bf16 — the input, both weights, the conv outputs y1 / y2,
    the BN+clip outputs, and the backward's dy2, dz1, dy1 — so its gradients differ from the
    kernels' only by accumulation order. Returns the float64 parameter gradients;
    dbeta_mass (a dict) receives, per block, sum |dL/d(BN output)| per channel: the scale of
    the terms that the BN beta gradient sums."""
    import torch.nn.functional as F
    from deepspeech_amd.ops import reference as R
    c1, c2 = model.conv1, model.conv2
    leaves = {n: p.detach().double().requires_grad_(True) for n, p in
              (("conv1.weight", c1.weight), ("conv1.bn_gamma", c1.bn_gamma), ("conv1.bn_beta", c1.bn_beta),
               ("conv2.weight", c2.weight), ("conv2.bn_gamma", c2.bn_gamma), ("conv2.bn_beta", c2.bn_beta))}

    def block(x, blk, pre):
        y = F.conv2d(x, _st_round(leaves[pre + ".weight"]), blk.bias.detach().double(), stride=blk.stride)
        y = _RoundGrad.apply(y)                           # dy (BN backward output) stored bf16
        mean = y.mean(dim=(0, 2, 3), keepdim=True)        # statistics of the fp32 epilogue sums
        var = ((y - mean) ** 2).mean(dim=(0, 2, 3), keepdim=True)
        ys = _st_round(y)                                 # y stored bf16
        z = (ys - mean) * torch.rsqrt(var + blk.bn_eps) * leaves[pre + ".bn_gamma"].view(1, -1, 1, 1) \
            + leaves[pre + ".bn_beta"].view(1, -1, 1, 1)
        if dbeta_mass is not None:
            z.register_hook(lambda gz, pre=pre: dbeta_mass.__setitem__(pre, gz.abs().sum(dim=(0, 2, 3))))
        return _st_round(R.clipped_relu(z))              # BN + clip output stored bf16

    x = feats.to(torch.bfloat16).double().unsqueeze(1)
    z1 = _RoundGrad.apply(block(x, c1, "conv1"))         # dz1 (conv2 dgrad output) stored bf16
    z2 = block(z1, c2, "conv2")
    N, C, T2, F2 = z2.shape
    out = z2.permute(2, 0, 1, 3).reshape(T2, N, C * F2)
    out.backward(dout.double())
    return {n: t.grad for n, t in leaves.items()}


def test_frontend_backward_headline_same_upstream(cuda):
    """The conv front-end at the headline geometry (32 filters, batch 32, 10-s utterances)
    with the SAME upstream gradient fed to the HIP kernels and to a float64 reference that
    stores in bf16 exactly where the kernels do. Against the plain fp32 engine the conv1
    gradients of this random problem differ by 7 % (weight) and 26 % (BN beta): the BN2
    backward output is zero-mean per channel, so conv1's gradients are sums that cancel
    to far below their terms and the bf16 storage of dz1 / dy1 dominates them. With that
    storage emulated, what is left is the kernels' own arithmetic: every front-end weight /
    gamma gradient within 2 % (measured 0.4-0.9 %), so a kernel error of ~10 % cannot hide
    behind bf16 drift. conv1's BN beta gradient cancels to ~1e-5 of its terms, below fp32
    accumulation-order noise (measured per channel |error| 0.07-0.8 % of sum |dL/d(BN
    output)| over its 1.3 M terms), so it is held to its terms' scale instead: |error| <=
    1e-2 x sum |dL/d(BN output)|, which still catches a kernel that drops or double-counts a
    percent of the positions."""
    ref, hip = _pair(cuda, "gru", H=64, L=1)
    batch = to_device(FixedShapeBatches(32, max_frames=1000, seed=5, pool=1).next(), cuda)
    hip.train()
    xh = hip.frontend(batch["feats"].to(torch.bfloat16))
    torch.manual_seed(1)
    # an upstream gradient with a common component, like a loss gradient
    dout = ((torch.randn(xh.shape, device=cuda) + 0.3) * 1e-3).to(torch.bfloat16)
    xh.backward(dout)
    torch.cuda.synchronize()
    mass = {}
    want = _frontend_emulated(hip, batch["feats"], dout, mass)
    got = dict(hip.named_parameters())
    errs = {n: _rel(got[n].grad.double(), g) for n, g in want.items() if n != "conv1.bn_beta"}
    assert max(errs.values()) < 2e-2, errs
    d = (got["conv1.bn_beta"].grad.double() - want["conv1.bn_beta"]).abs()
    assert bool((d <= 1e-2 * mass["conv1"]).all()), (d / mass["conv1"]).max().item()


def test_fused_head_ctc_matches_reference(cuda):
    """FusedHeadCTC (MFMA FC + in-register log-softmax + CTC + GEMM backward) against the
    fp32 FC + torch CTC, gradients of h, W_fc and b_fc."""
    from deepspeech_amd.ops import ctc as CTC
    from deepspeech_amd.ops import reference as R
    torch.manual_seed(2)
    T, N, H, K = 120, 8, 256, 29
    h = (torch.randn(T, N, H, device=cuda) * 0.5).to(torch.bfloat16)
    W = (torch.randn(K, H, device=cuda) * 0.1)
    b = torch.randn(K, device=cuda) * 0.1
    lens = torch.tensor([120, 100, 77, 120, 31, 64, 119, 90], dtype=torch.int32, device=cuda)
    Ls = [30, 25, 20, 1, 8, 15, 40, 2]
    labels = torch.zeros(N, max(Ls), dtype=torch.int32)
    for i, L in enumerate(Ls):
        labels[i, :L] = torch.randint(0, K - 1, (L,))
    labels = labels.to(cuda)
    lab_lens = torch.tensor(Ls, dtype=torch.int32, device=cuda)
    Wb, bb = W.to(torch.bfloat16).float(), b.to(torch.bfloat16).float()
    hx = h.clone().requires_grad_(True)
    Wx, bx = Wb.clone().requires_grad_(True), bb.clone().requires_grad_(True)
    loss = CTC.head_ctc_mean_loss_hip(hx, Wx, bx, lens, labels, lab_lens)
    (loss * 0.5).backward()
    hr = h.float().clone().requires_grad_(True)
    Wr, br = Wb.clone().requires_grad_(True), bb.clone().requires_grad_(True)
    logits = hr @ Wr.t() + br
    lr = R.ctc_loss_ref(logits, labels, lens, lab_lens).mean()
    (lr * 0.5).backward()
    assert abs(float(loss) - float(lr)) / float(lr) < 2e-3, (float(loss), float(lr))
    assert _rel(hx.grad, hr.grad) < 2e-2
    assert _rel(Wx.grad, Wr.grad) < 2e-2
    assert _rel(bx.grad, br.grad) < 2e-2


def test_arena_groups_pack_directions(cuda):
    _, hip = _pair(cuda, "gru", H=64, L=2)
    arena = ParamArena(hip, bf16_shadow=True)
    for layer in hip.rnn:
        v = arena.group_view([layer.fw.W, layer.bw.W], "p16")
        assert v is not None and v.numel() == 2 * layer.fw.W.numel()
        assert torch.equal(v.view(-1, layer.fw.W.shape[1])[: layer.fw.W.shape[0]].float(),
                           layer.fw.W.detach().bfloat16().float())
        assert arena.group_view([layer.fw.b, layer.bw.b], "grad") is not None


def test_hip_engine_trains(cuda):
    """A few fused Adam steps on one batch lower the CTC loss (HIP engine, arena path)."""
    from deepspeech_amd.trainer import Trainer, LRSchedule
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=32, num_hidden=128, num_rnn_layers=2, cell="gru").to(cuda)
    m.set_engine("hip", torch.bfloat16)
    tr = Trainer(m, LRSchedule(3e-3, 1000, 0.9))
    batch = to_device(FixedShapeBatches(8, max_frames=300, seed=1, pool=1).next(), cuda)
    first = float(tr.step(batch))
    for _ in range(30):
        last = float(tr.step(batch))
    assert last < 0.8 * first, (first, last)


def test_streaming_hip_matches_full_forward(cuda):
    """Chunked streaming through the HIP engine (state carried between persistent-kernel
    launches) reproduces the whole-utterance forward of the same engine."""
    from deepspeech_amd.infer import StreamingRecognizer
    torch.manual_seed(3)
    m = DeepSpeech2(num_filters=8, num_hidden=128, num_rnn_layers=2, cell="gru", bidirectional=False).to(cuda)
    m.set_engine("hip", torch.bfloat16)
    m.eval()
    T, B = 640, 3
    feats = torch.randn(B, T, 161, device=cuda)
    with torch.no_grad():
        logits, _ = m(feats, torch.full((B,), T, dtype=torch.int32, device=cuda))
    full = torch.log_softmax(logits.float(), -1)
    rec = StreamingRecognizer(m, batch=B)
    for s in range(0, T, 100):
        rec.accept(feats[:, s:s + 100])
    got = torch.cat(rec.logprobs, 0)
    assert got.shape == full.shape
    assert (got - full).abs().max() < 0.15, (got - full).abs().max()
    assert _rel(got.exp(), full.exp()) < 3e-2


def test_fp8_projection_close_to_bf16(cuda):
    """fp8 e4m3 input projections (config 5): loss and gradients stay close to the bf16 engine."""
    ref, hip = _pair(cuda, "gru", H=128, L=2)
    hip8 = copy.deepcopy(hip)
    hip8.set_engine("hip", torch.bfloat16, fp8=True)
    batch = to_device(FixedShapeBatches(6, max_frames=260, seed=3, pool=1).next(), cuda)
    l16 = _loss(hip, batch)
    l16.backward()
    l8 = _loss(hip8, batch)
    l8.backward()
    assert abs(float(l8) - float(l16)) / abs(float(l16)) < 5e-2, (float(l8), float(l16))
    g16 = dict(hip.named_parameters())
    for n, p in hip8.named_parameters():
        if n.startswith("rnn.1") or n.startswith("fc"):
            assert _rel(p.grad, g16[n].grad) < 0.25, n


def test_fp8_recurrence_model_close_to_bf16(cuda):
    """Config 5's fp8 mode at its width AND production batch (H = 1280, N = 32: 8 rows per
    group, 2 layers): the recurrence runs on csrc/rnn_fp8.hip (e4m3 U and h exchange), the BPTT
    in bf16 on the saved state (a straight-through gradient of the quantised forward). First
    step: loss within 5 % of the bf16 engine, top-layer / head gradients within 25 %; then 3
    full training steps each (Trainer: fused Adam + EMA), losses within 5 % step by step."""
    from deepspeech_amd.ops import rnn as RNN
    from deepspeech_amd.trainer import LRSchedule, Trainer
    ref, hip = _pair(cuda, "gru", H=1280, L=2)
    hip8 = copy.deepcopy(hip)
    hip8.set_engine("hip", torch.bfloat16, fp8=True)
    batch = to_device(FixedShapeBatches(32, max_frames=260, seed=4, pool=1).next(), cuda)
    plan = RNN.plan_for(32, 1280, "gru", 2, cuda)
    assert RNN.fp8_recurrence_ok(plan, 32)
    t16, t8 = copy.deepcopy(hip), copy.deepcopy(hip8)
    l16 = _loss(hip, batch)
    l16.backward()
    l8 = _loss(hip8, batch)
    l8.backward()
    RNN.join_wgrad_streams()
    torch.cuda.synchronize()
    RNN.check_errors()
    assert abs(float(l8) - float(l16)) / abs(float(l16)) < 5e-2, (float(l8), float(l16))
    g16 = dict(hip.named_parameters())
    for n, p in hip8.named_parameters():
        if n.startswith("rnn.1") or n.startswith("fc"):
            assert _rel(p.grad, g16[n].grad) < 0.25, n
    tr16, tr8 = Trainer(t16, LRSchedule(1e-4, 1000, 0.9)), Trainer(t8, LRSchedule(1e-4, 1000, 0.9))
    for _ in range(3):
        a, b = float(tr16.step(batch)), float(tr8.step(batch))
        assert abs(a - b) / abs(a) < 5e-2, (a, b)
    RNN.check_errors()


def test_fp8_direction_pairs_are_bitwise_the_summed_stack(cuda, monkeypatch):
    """fp8 stack (config 5's mode at its width, 3 layers): each fp8 layer hands its two
    direction outputs to the next one, whose quantiser sums them (FusedBiLayer pair_out), instead
    of a torch.add per layer. Loss and every gradient are bitwise those of the summed stack, and
    the pair path leaves exactly one direction-sum add (the top layer's, feeding the head)."""
    from deepspeech_amd.ops import rnn as RNN
    torch.manual_seed(3)
    base = DeepSpeech2(num_filters=32, num_hidden=1280, num_rnn_layers=3, cell="gru").to(cuda)
    base.set_engine("hip", torch.bfloat16, fp8=True)
    batch = to_device(FixedShapeBatches(32, max_frames=200, seed=8, pool=1).next(), cuda)
    assert RNN.fp8_recurrence_ok(RNN.plan_for(32, 1280, "gru", 2, cuda), 32)
    res = []
    for pairs in (False, True):
        m = copy.deepcopy(base)
        if not pairs:
            monkeypatch.setattr(RNN, "pairs_ok", lambda layer: False)
        adds = []
        real_add = torch.add

        def counting_add(*a, **k):
            adds.append(1)
            return real_add(*a, **k)
        monkeypatch.setattr(torch, "add", counting_add)
        loss = _loss(m, batch)
        loss.backward()
        monkeypatch.setattr(torch, "add", real_add)
        monkeypatch.undo()
        RNN.join_wgrad_streams()
        torch.cuda.synchronize()
        RNN.check_errors()
        res.append((loss.detach(), {n: p.grad.clone() for n, p in m.named_parameters()}, len(adds)))
    (l0, g0, n0), (l1, g1, n1) = res
    assert torch.equal(l0, l1)
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n
    assert n0 - n1 == 2, (n0, n1)          # 3 layers: two sums moved into the quantisers


def test_step_is_bitwise_reproducible(cuda):
    """Two trainers from the same initial state on the same batch produce bitwise-identical
    losses, gradients and updated weights (every fused kernel reduces in a fixed order; the
    side-stream weight-gradient GEMMs write disjoint arena slices). SURVEY.md 5.2's
    'deterministic mode' is therefore the default on the HIP engine."""
    from deepspeech_amd.trainer import Trainer, LRSchedule
    torch.manual_seed(0)
    base = DeepSpeech2(num_filters=32, num_hidden=256, num_rnn_layers=3, cell="gru").to(cuda)
    batch = to_device(FixedShapeBatches(8, max_frames=300, seed=3, pool=1).next(), cuda)
    runs = []
    for _ in range(2):
        m = copy.deepcopy(base).set_engine("hip", torch.bfloat16)
        tr = Trainer(m, LRSchedule(1e-4, 1000, 0.9))
        losses = [float(tr.step(batch)) for _ in range(3)]
        torch.cuda.synchronize()
        runs.append((losses, tr.arena.grad.clone(), tr.arena.flat.clone()))
    (l0, g0, w0), (l1, g1, w1) = runs
    assert l0 == l1, (l0, l1)
    assert torch.equal(g0, g1), (g0 - g1).abs().max()
    assert torch.equal(w0, w1)


@pytest.mark.parametrize("H,partial", [(256, True), (800, True), (800, False)])
def test_early_optimizer_range_is_bitwise_whole_update(cuda, H, partial, monkeypatch):
    """Single device: the FC head's and recurrent stack's Adam + EMA range, issued on the
    weight-gradient stream beside the conv front-end's backward, gives bitwise the weights,
    moments and EMA of one whole-arena update after backward (three steps). H = 256: the
    BPTT leaves >= 96 CUs idle, so the weight gradients run beside each BPTT and the range of
    the head + layers >= 1 goes out beside layer 0's BPTT (two early ranges); H = 800 (the
    headline width, 8 rows per group, 56 idle CUs): layer 0's weight gradients in the grouped
    launch, the upper layers' beside the next BPTT on the idle CUs — two early ranges as well
    (DS2_DEFER_LAYERS unset, sequences of >= _PARTIAL_MIN_T steps); with every layer
    deferred (shorter sequences: ``partial`` False), one."""
    from deepspeech_amd.ops import rnn as RNN
    from deepspeech_amd.trainer import Trainer, LRSchedule
    monkeypatch.setattr(RNN, "_PARTIAL_MIN_T", 0 if partial else 1 << 30)
    torch.manual_seed(0)
    N = 8 if H == 256 else 32
    base = DeepSpeech2(num_filters=32, num_hidden=H, num_rnn_layers=3, cell="gru").to(cuda)
    batch = to_device(FixedShapeBatches(N, max_frames=300, seed=3, pool=1).next(), cuda)
    plan = RNN.plan_for(N, H, "gru", 2, cuda)
    two_stage = not RNN._defer_wgrad(plan, cuda) or RNN._defer_layers(plan, cuda, 64) < 3
    assert (not RNN._defer_wgrad(plan, cuda)) == (H == 256)
    if H == 800 and RNN._DEFER_LAYERS < 0:
        assert two_stage == partial
    runs = []
    # "upper_only": the lower early range is skipped after the upper one ran (the
    # fallback update must not apply [0, usplit) a second time)
    for mode in ("early", "none") + (("upper_only",) if two_stage else ()):
        early = mode != "none"
        m = copy.deepcopy(base).set_engine("hip", torch.bfloat16)
        tr = Trainer(m, LRSchedule(1e-4, 1000, 0.9))
        assert tr._early_split > 0 and tr.upper_range(1) is not None
        if not early:
            tr._early_split = 0
        sch = tr.arena.wgrad
        if mode == "upper_only":
            sch.run_early_update = lambda sch=sch: setattr(sch, "_early", None)
        for _ in range(3):
            tr.step(batch)
            assert sch.early_done == (mode == "early")
            assert sch.early_upper_done == (early and two_stage)
        torch.cuda.synchronize()
        runs.append((tr.arena.flat.clone(), tr.opt.m.clone(), tr.opt.v.clone(), tr.opt.ema.clone()))
    for other in runs[1:]:
        for a, b in zip(runs[0], other):
            assert torch.equal(a, b), (a - b).abs().max()


@pytest.mark.parametrize("cell", ["gru", "rnn_relu"])
def test_nhwc_graph_hip_matches_reference(cuda, cell):
    """--nchw False graph on the HIP engine (moments+EMA conv BN in the channels-last
    kernels, per-direction stacks as one-direction persistent layers over length-aware
    reversals) against the fp32 reference engine; EMA state advanced identically."""
    from deepspeech_amd.ops import rnn as RNN
    torch.manual_seed(12)
    ref = DeepSpeech2(num_filters=32, num_hidden=64, num_rnn_layers=3, cell=cell, layout="nhwc").to(cuda)
    hip = copy.deepcopy(ref)
    ref.set_engine("ref", torch.float32)
    hip.set_engine("hip", torch.bfloat16)
    batch = to_device(FixedShapeBatches(6, max_frames=260, seed=4, pool=1).next(), cuda)
    arena = ParamArena(hip, bf16_shadow=True)
    arena.zero_grad()
    lh = _loss(hip, batch, True)
    lh.backward()
    RNN.join_wgrad_streams()
    lr = _loss(ref, batch)
    lr.backward()
    torch.cuda.synchronize()
    RNN.check_errors()
    # clipped ReLU: layer 0's forward stack backpropagates through 3 one-direction layers of
    # bf16-rounded clip masks (measured rnn.0.fw.W 11.9 %, U 9.7 %, conv 15-17 %); the GRU,
    # through the same plumbing, stays within the 6 % of the bidirectional-layer tests
    if cell == "gru":
        _compare_grads(ref, hip, lh, lr, cell)
    else:
        _compare_grads(ref, hip, lh, lr, cell, tol_rnn=0.15, tol_conv=0.25)
    for blk in ("conv1", "conv2"):
        a, b = getattr(hip, blk), getattr(ref, blk)
        assert float(a.ema_steps) == float(b.ema_steps) == 1.0
        assert _rel(a.ema_mean_biased, b.ema_mean_biased) < 2e-2
        assert _rel(a.ema_var_biased, b.ema_var_biased) < 5e-2


def test_prefetcher_matches_direct_upload(cuda):
    """data/prefetch.py (pinned ring + copy stream + event) hands the step exactly the
    tensors a synchronous upload would, across bucket-size changes (ring slot regrowth)."""
    from deepspeech_amd.data.prefetch import DevicePrefetcher
    from deepspeech_amd.data.synthetic import DummyBucketWalk

    class Seq:
        def __init__(self):
            self.w = DummyBucketWalk(4, seed=9)
            self.i = 0

        def next(self):
            self.i += 1
            return self.w.batch_for([0, 3, 14, 1, 7][self.i % 5])
    ref_src, pf = Seq(), DevicePrefetcher(Seq(), cuda, depth=2)
    for _ in range(7):
        hb, dev = pf.next()
        want = to_device(ref_src.next(), cuda)
        for k, v in want.items():
            assert torch.equal(dev[k], v), k
        assert hb.feats.shape[1] == dev["feats"].shape[1]
    pf.close()


# every recurrence kernel family a bf16 plan can reach, at T = 241 and batch 32 (VERDICT r4
# item 6): (cell, H, input width, T, DS2_RNN_MODE, expected forward family)
_LAYER_CASES = [("gru", 800, 800, 241, "auto", "rnne_fwd"), ("gru", 800, 2400, 241, "auto", "rnne_fwd"),
                ("gru", 1280, 1280, 241, "auto", "rnnq_fwd"), ("rnn_relu", 800, 800, 241, "auto", "rnnq_fwd"),
                ("rnn_relu", 1760, 1760, 241, "auto", "rnnw_fwd"),
                ("gru", 1056, 1056, 241, "auto", "rnnx_fwd"),        # generation 2: H / 32 = 33
                ("rnn_relu", 2048, 2048, 241, "auto", "rnn_fwd"),    # wider than rnnw: generation 1
                ("gru", 800, 800, 241, "step", "rnn_fwd")]           # the non-persistent fallback


@pytest.mark.parametrize("cell,H,D,T,mode,family", _LAYER_CASES)
def test_recurrent_layer_same_upstream(cuda, monkeypatch, cell, H, D, T, mode, family):
    """ONE bidirectional recurrent layer at the production geometries (batch 32, ragged
    lengths) with the same bf16 input and the same upstream gradient fed to the HIP layer
    (projection GEMM, persistent recurrence, BPTT, dx / dW / dU GEMMs, in-kernel bias sums)
    and to an fp32 reference that rounds to bf16 where the kernels do (the W and U they
    multiply, the projection output gx, the hidden state fed to the recurrent product;
    gradients straight through). Errors do not accumulate through a stack here, so a kernel
    that is wrong by a few percent in any layer cannot hide under the whole-model tolerances
    above.

    GRU: every output / gradient within 1.5 % (measured 0.1-0.3 %). Clipped ReLU: the
    derivative is discontinuous at 0, where ~25 % of the units sit at this random init, so any
    bf16-level perturbation flips a small fraction of masks and each flip changes its term by
    100 %: the relative gradient error scales like the square root of the flip fraction, not
    with the perturbation (in the fp32 reference alone, rounding U to bf16 moves the ReLU-800
    gradients by 3.6 % at T = 5 and 4.2 % at T = 61, the GRU's by 0.05 %). The ReLU gradients
    are therefore held to 1.6 x the spread the reference itself shows under exactly that
    rounding of U (measured: kernels 5.0-5.2 %, spread 5.4-6.1 %); a kernel error of 10 % would
    add in quadrature to ~11 %, over the bound."""
    from deepspeech_amd.models.deepspeech2 import RecurrentLayer
    from deepspeech_amd.ops import reference as R
    from deepspeech_amd.ops import rnn as RNN
    monkeypatch.setenv("DS2_RNN_MODE", mode)
    torch.manual_seed(H + D)
    N = 32
    fams = RNN.kernel_families(RNN.plan_for(N, H, cell, 2, cuda))
    assert fams[0].startswith(family), fams
    ref = RecurrentLayer(D, H, cell, True, "frozen").to(cuda)
    with torch.no_grad():
        for d in ref.directions():
            d.b.normal_(0, 0.1)
            if d.b_h is not None:
                d.b_h.normal_(0, 0.1)
    hip = copy.deepcopy(ref)
    lens = torch.randint(T // 2, T + 1, (N,), device=cuda, dtype=torch.int32)
    lens[0] = T
    x = (torch.randn(T, N, D, device=cuda) * (1.0 if cell == "gru" else 2.0)).to(torch.bfloat16)
    dy = (torch.randn(T, N, H, device=cuda) * 1e-2).to(torch.bfloat16)
    mask = (torch.arange(T, device=cuda)[:, None] < lens[None, :].long()).to(torch.float32)[..., None]

    def reference(round_u: bool):
        ref.zero_grad()
        xr = x.float().requires_grad_(True)
        gx, Us, bh = [], [], []
        for d in ref.directions():
            y = xr @ _st_round(d.W).t()
            y = R.seq_batch_norm(y, lens, ref.seq_bn, d.sbn_mean, d.sbn_var, ref.training)
            gx.append(_st_round(y + d.b))
            Us.append(_st_round(d.U) if round_u else d.U)
            bh.append(d.b_h)
        yr = R.birnn_ref(cell, gx[0], gx[1], Us[0], Us[1], bh[0], bh[1], lens, mm_dtype=torch.bfloat16)
        (yr * mask * dy.float()).sum().backward()
        out = {"y": yr.detach() * mask, "dx": xr.grad}
        out.update({n: p.grad.clone() for n, p in ref.named_parameters()})
        return out

    want = reference(True)
    xh = x.clone().requires_grad_(True)
    yh = RNN.recurrent_layer_hip(hip, xh, lens)
    yh.backward(dy * mask.to(torch.bfloat16))
    RNN.join_wgrad_streams()
    torch.cuda.synchronize()
    RNN.check_errors()
    got = {"y": yh.float() * mask, "dx": xh.grad}
    got.update({n: p.grad for n, p in hip.named_parameters()})
    errs = {k: _rel(got[k], want[k]) for k in want}
    if cell == "gru":
        tol = {k: 0.015 for k in want}
    else:
        spread = reference(False)
        tol = {k: 0.015 if k == "y" else max(0.03, 1.6 * _rel(spread[k], want[k])) for k in want}
    print(fams, {k: (round(errs[k], 5), round(tol[k], 4)) for k in errs})
    bad = {k: (errs[k], tol[k]) for k in errs if errs[k] > tol[k]}
    assert not bad, (bad, errs)
