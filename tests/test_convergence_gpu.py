"""Training-dynamics parity: 200 Adam steps of the HIP engine (bf16 compute, fused kernels,
fp32 master weights in the arena) against the pure-PyTorch fp32 reference engine, same
initial weights, same batches ("a 200-step synthetic
loss-curve comparison, HIP-bf16 against ref-fp32, on a small model").

Per-step gradients already match within bf16 tolerance (test_engine_gpu.py); this checks
that the rounding does not accumulate into a different trajectory: windowed mean losses
must track each other and both runs must actually learn (the reference's training loop:
src/deepSpeech_train.py:292-380 — Adam, loss EMA, weight EMA).
"""
import copy

import pytest
import torch

from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
from deepspeech_amd.models import DeepSpeech2
from deepspeech_amd.trainer import LRSchedule, Trainer

pytestmark = pytest.mark.gpu

STEPS, WINDOW = 200, 20


def _curves(cuda, cell, steps=STEPS, lr=5e-4):
    torch.manual_seed(5)
    ref = DeepSpeech2(num_filters=32, num_hidden=64, num_rnn_layers=2, cell=cell).to(cuda)
    hip = copy.deepcopy(ref)
    ref.set_engine("ref", torch.float32)
    hip.set_engine("hip", torch.bfloat16)
    # 4 fixed batches cycled: the model can fit them, so the loss has somewhere to go
    batches = [to_device(FixedShapeBatches(8, max_frames=300, seed=s, pool=1).next(), cuda) for s in range(4)]
    sched = LRSchedule(lr, 10 ** 9, 1.0)
    t_ref = Trainer(ref, sched, moving_avg_decay=0.9999)
    t_hip = Trainer(hip, sched, moving_avg_decay=0.9999)
    lr_, lh_ = [], []
    for i in range(steps):
        b = batches[i % len(batches)]
        lr_.append(t_ref.step(b).detach().float())
        lh_.append(t_hip.step(b).detach().float())
    torch.cuda.synchronize()
    return torch.stack(lr_).cpu(), torch.stack(lh_).cpu(), t_ref, t_hip


@pytest.mark.parametrize("cell", ["gru", "rnn_relu"])
def test_loss_curve_hip_bf16_tracks_ref_fp32(cuda, cell):
    lr_, lh_, t_ref, t_hip = _curves(cuda, cell)
    assert torch.isfinite(lr_).all() and torch.isfinite(lh_).all()
    wr = lr_.view(-1, WINDOW).mean(1)
    wh = lh_.view(-1, WINDOW).mean(1)
    rel = ((wh - wr).abs() / wr).tolist()
    table = " ".join("%.1f/%.1f" % (a, b) for a, b in zip(wr.tolist(), wh.tolist()))
    # both engines learn the 4 batches ...
    assert wr[-1] < 0.7 * wr[0] and wh[-1] < 0.7 * wh[0], "windowed ref/hip loss: " + table
    # ... along the same trajectory: every 20-step window mean within 5 % for the GRU (measured
    # on MI355X: 134 -> 1.2 with max window difference 0.2 %, weights 1.1 % apart). The
    # clipped-ReLU net is chaotic enough that the fp32 REFERENCE itself is not reproducible: in
    # five round-4 runs the HIP curve was bitwise the same (164.2 ... 4.2 2.3 1.5 1.1) while the
    # reference's late windows moved by up to 3 % between runs (9.5-9.8, 3.9-4.0), and the max
    # window difference came out 5.2-8.1 % (1.6 % in an earlier round): 10 % for ReLU
    tol = 0.05 if cell == "gru" else 0.10
    assert max(rel) < tol, "windowed ref/hip loss: %s (max rel diff %.3f)" % (table, max(rel))
    # the master weights stay close too (fp32 arena in both; only the compute is bf16). The
    # clipped-ReLU net drifts further: bf16 rounding flips clip masks, and Adam's normalised
    # steps turn small gradient differences into full-size weight differences
    w_rel = ((t_hip.arena.flat - t_ref.arena.flat).norm() / t_ref.arena.flat.norm()).item()
    print("%s windowed ref/hip loss: %s; max rel %.4f; weights rel %.4f" % (cell, table, max(rel), w_rel))
    assert w_rel < (0.05 if cell == "gru" else 0.12), w_rel


def test_fp8_projection_training_tracks_bf16(cuda):
    """BASELINE config 5's fp8 mode (e4m3 per-tensor-scaled input projections, bf16
    recurrence and gradients) trains along the bf16 trajectory: 300 steps, same weights and
    batches, windowed losses within 10 % (validate fp8 convergence on
    synthetic data). Measured on MI355X: 124.8 -> 0.6 with max window difference 1.7 %."""
    torch.manual_seed(9)
    base = DeepSpeech2(num_filters=32, num_hidden=64, num_rnn_layers=2, cell="gru").to(cuda)
    f8 = copy.deepcopy(base)
    base.set_engine("hip", torch.bfloat16)
    f8.set_engine("hip", torch.bfloat16, fp8=True)
    batches = [to_device(FixedShapeBatches(8, max_frames=300, seed=20 + s, pool=1).next(), cuda) for s in range(4)]
    sched = LRSchedule(5e-4, 10 ** 9, 1.0)
    tb, tf = Trainer(base, sched), Trainer(f8, sched)
    lb, lf = [], []
    for i in range(300):
        b = batches[i % 4]
        lb.append(tb.step(b).detach().float())
        lf.append(tf.step(b).detach().float())
    torch.cuda.synchronize()
    lb, lf = torch.stack(lb).cpu(), torch.stack(lf).cpu()
    assert torch.isfinite(lf).all()
    wb, wf = lb.view(-1, 30).mean(1), lf.view(-1, 30).mean(1)
    rel = ((wf - wb).abs() / wb)
    table = " ".join("%.1f/%.1f" % (a, c) for a, c in zip(wb.tolist(), wf.tolist()))
    print("fp8 windowed bf16/fp8 loss: %s; max rel %.4f" % (table, float(rel.max())))
    assert wf[-1] < 0.5 * wf[0], table
    assert float(rel.max()) < 0.10, table


def test_fp8_recurrence_training_tracks_bf16(cuda):
    """Config 5's full fp8 mode — MX-fp8 projections, the e4m3 forward recurrence AND the fp8
    BPTT of csrc/rnn_fp8.hip (H % 256 == 0, so this geometry really routes through both
    kernels: asserted) — trains along the bf16 trajectory: 300 steps, same weights and
    batches. The BPTT multiplies an e4m3 U^T and requantises the gate gradients per (row,
    32-unit group) every step; its gradient is straight-through with respect to the
    quantisation of the exchanged h. The reference has no fp8 mode (parity unpinned).
    Measured on MI355X with the fp8 BPTT (round 5, tests run with -s print the windows):
    175.0/184.7 48.9/53.7 9.4/11.3 2.6/3.0 1.3/1.4 0.9/0.9 0.6/0.7 0.5/0.5 0.4/0.4 0.3/0.3,
    max window difference 19 % (round 4, bf16 BPTT on the same fp8 forward: 24 %), again on
    the steep part of the descent. Pinned: every window within 25 % (was 35 %), the last three
    within 12 % (was 15 %), both runs learn > 100x."""
    from deepspeech_amd.ops import rnn as RNN
    torch.manual_seed(11)
    N, H = 8, 256
    base = DeepSpeech2(num_filters=32, num_hidden=H, num_rnn_layers=2, cell="gru").to(cuda)
    f8 = copy.deepcopy(base)
    base.set_engine("hip", torch.bfloat16)
    f8.set_engine("hip", torch.bfloat16, fp8=True)
    assert RNN.fp8_recurrence_ok(RNN.plan_for(N, H, "gru", 2, cuda), N)
    assert RNN.fp8_bptt_ok(RNN.plan_for(N, H, "gru", 2, cuda), N)
    batches = [to_device(FixedShapeBatches(N, max_frames=300, seed=40 + s, pool=1).next(), cuda) for s in range(4)]
    sched = LRSchedule(3e-4, 10 ** 9, 1.0)
    tb, tf = Trainer(base, sched), Trainer(f8, sched)
    lb, lf = [], []
    for i in range(300):
        b = batches[i % 4]
        lb.append(tb.step(b).detach().float())
        lf.append(tf.step(b).detach().float())
    torch.cuda.synchronize()
    RNN.check_errors()
    lb, lf = torch.stack(lb).cpu(), torch.stack(lf).cpu()
    assert torch.isfinite(lf).all()
    wb, wf = lb.view(-1, 30).mean(1), lf.view(-1, 30).mean(1)
    rel = ((wf - wb).abs() / wb)
    table = " ".join("%.1f/%.1f" % (a, c) for a, c in zip(wb.tolist(), wf.tolist()))
    print("fp8-recurrence windowed bf16/fp8 loss: %s; max rel %.4f" % (table, float(rel.max())))
    assert wf[-1] < 0.01 * wf[0] and wb[-1] < 0.01 * wb[0], table
    assert float(rel.max()) < 0.25, table
    assert float(rel[-3:].max()) < 0.12, table
