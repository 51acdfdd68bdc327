"""csrc/stats.hip: device histogram / moments / zero fraction against the numpy path, and the
per-step non-finite watch (one launch per step, read later)."""
import numpy as np
import pytest
import torch

from deepspeech_amd.utils import stats as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_device_histogram_matches_host(cuda, dtype):
    torch.manual_seed(0)
    x = torch.randn(3_000_017, device=cuda) * torch.logspace(-6, 6, 3_000_017, device=cuda)
    x[::97] = 0.0
    x[5] = float("nan")
    x = x.to(dtype)
    d = S.histogram(x)
    h = S.histogram(x.cpu())
    assert d.num == h.num and d.zeros == h.zeros and d.nonfinite == h.nonfinite == 1
    # float32 __logf vs float64 log moves values lying within ~1e-6 (relative) of a bucket
    # limit by one bucket: measured 5e-4 of the values (fp32 input) and 1.9e-3 (bf16 input,
    # whose 8-bit-mantissa grid puts some points right at limits); totals are unaffected
    assert np.abs(d.counts - h.counts).sum() <= 3e-3 * h.num
    assert d.counts.sum() == h.counts.sum()
    assert d.min == h.min and d.max == h.max
    assert abs(d.sum - h.sum) <= 1e-4 * max(1.0, abs(h.sum_sq) ** 0.5 * 100)
    assert abs(d.sum_sq - h.sum_sq) / h.sum_sq < 1e-4


def test_device_nonfinite_watch(cuda):
    w = S.NonfiniteWatch(cuda)
    w.reset(100)
    for v in (1.0, float("inf"), float("nan")):
        w.update(torch.tensor(v, device=cuda))
    assert w.first_bad_step() == 101


@pytest.mark.parametrize("fused", [True, False])
def test_nan_logits_reach_the_loss_and_the_watch(cuda, fused):
    """A diverged model (NaN in the head's output) must produce a NaN loss even with
    zero_infinity, so the per-step watch (and --nan_policy abort) sees it. The CTC kernels
    used to treat NaN log-likelihoods as infeasible utterances (loss 0, zero gradient)."""
    from deepspeech_amd.ops import ctc as CTC
    torch.manual_seed(0)
    T, N, H, K = 40, 4, 64, 29
    lens = torch.full((N,), T, dtype=torch.int32, device=cuda)
    labels = torch.randint(0, 28, (N, 8), dtype=torch.int32, device=cuda)
    label_lens = torch.full((N,), 8, dtype=torch.int32, device=cuda)
    if fused:
        h = torch.randn(T, N, H, device=cuda).bfloat16()
        h[7, 2, 5] = float("nan")                   # one utterance's hidden state diverged
        w = torch.randn(K, H, device=cuda) * 0.1
        b = torch.zeros(K, device=cuda)
        loss = CTC.head_ctc_mean_loss_hip(h, w, b, lens, labels, label_lens)
    else:
        logits = torch.randn(T, N, K, device=cuda)
        logits[7, 2, 3] = float("nan")
        loss = CTC.ctc_mean_loss_hip(logits, lens, labels, label_lens)
    assert torch.isnan(loss).item()
    w = S.NonfiniteWatch(cuda)
    w.reset(7)
    w.update(torch.tensor(1.0, device=cuda))
    w.update(loss.detach())
    assert w.first_bad_step() == 8


def test_trainer_fused_loss_watch(cuda):
    """The HIP engine's head + CTC writes the batch-mean loss and runs the step's divergence
    watch in its gradient launch (ops/ctc.py loss_watch): the watch counts every step, records
    the first NaN step, and the loss is the mean of the per-utterance losses."""
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.ops import ctc as CTC
    from deepspeech_amd.trainer import LRSchedule, Trainer
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=32, num_hidden=128, num_rnn_layers=2, cell="gru").to(cuda).set_engine("hip", torch.bfloat16)
    tr = Trainer(m, LRSchedule(1e-4, 100, 0.9))
    b = to_device(FixedShapeBatches(4, max_frames=200, seed=0, pool=1).next(), cuda)
    with CTC.loss_watch(tr.watch) as lw:
        loss = m.forward_loss(b["feats"], b["seq_lens"], b["labels"], b["label_lens"])
    assert lw.consumed and loss.dim() == 0 and torch.isfinite(loss).item()
    assert int(tr.watch.counter.item()) == 1
    tr.watch.reset(0)
    for _ in range(3):
        tr.step(b)
    assert int(tr.watch.counter.item()) == 3 and tr.first_nonfinite_step() is None
    with torch.no_grad():
        m.fc_weight.data.fill_(float("nan"))
    tr.arena.mark_dirty()
    tr.step(b)
    tr.step(b)
    assert int(tr.watch.counter.item()) == 5 and tr.first_nonfinite_step() == 3
