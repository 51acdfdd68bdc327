"""Multi-step numerics at the PRODUCTION geometries.

The schedules that only switch on at production shapes — partial weight-gradient deferral
(T >= 200 recurrence steps, >= 56 idle CUs), capped beside grids, the early upper optimizer
range, the optimizer update carried into the next forward (Trainer defer_update), and the
64-unit fp8 H = 1280 kernels — were so far checked per step or over two steps. A cross-stream
ordering race there would show only as drift, so these tests train several dozen steps:

* the headline model (2 x conv + 5 x BiGRU-800, batch 32, 1000 frames) on the HIP engine with
  the bench's full schedule against the pure-PyTorch fp32 reference engine, same weights and
  batches: windowed losses and master weights within the small-model GRU tolerances
  (tests/test_convergence_gpu.py);
* BASELINE config 5 (7 x BiGRU-1280) in fp8 mode (MX-fp8 projections, e4m3 forward recurrence,
  fp8 BPTT) against its bf16 run.

Reference training loop: src/deepSpeech_train.py:292-380 (Adam, weight EMA per step).
"""
import copy

import pytest
import torch

from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
from deepspeech_amd.models import DeepSpeech2
from deepspeech_amd.trainer import LRSchedule, Trainer

pytestmark = pytest.mark.gpu


def _windows(a, b, w):
    a, b = torch.stack(a).float().cpu(), torch.stack(b).float().cpu()
    wa, wb = a.view(-1, w).mean(1), b.view(-1, w).mean(1)
    rel = (wb - wa).abs() / wa
    table = " ".join("%.1f/%.1f" % (x, y) for x, y in zip(wa.tolist(), wb.tolist()))
    return a, b, wa, wb, rel, table


def test_headline_40_steps_hip_tracks_ref_fp32(cuda):
    from deepspeech_amd.ops import rnn as RNN
    torch.manual_seed(21)
    ref = DeepSpeech2(num_filters=32, num_hidden=800, num_rnn_layers=5, cell="gru").to(cuda)
    hip = copy.deepcopy(ref)
    ref.set_engine("ref", torch.float32)
    hip.set_engine("hip", torch.bfloat16)
    batches = [to_device(FixedShapeBatches(32, max_frames=1000, seed=60 + s, pool=1).next(), cuda) for s in range(2)]
    from deepspeech_amd.ops import reference as R
    T2 = int(R.get_rnn_seqlen(batches[0]["seq_lens"]).max())
    plan = RNN.plan_for(32, 800, "gru", 2, cuda)
    sch = RNN.schedule_for(plan, T2, False, False, RNN._ext.num_cus(0))
    # the production schedule really is the one under test
    assert sch.defer_wgrad and sch.defer_layers == 1 and sch.upper_trigger == 1 and sch.beside_grid > 0, sch
    # a learning rate in the stable regime of this model (at 3e-4 the loss first climbs 2.8k ->
    # 3.6k and the fp32 and bf16 runs part ways chaotically: nothing to compare)
    sched = LRSchedule(3e-5, 10 ** 9, 1.0)
    t_ref = Trainer(ref, sched)
    t_hip = Trainer(hip, sched, defer_update=True)
    lr_, lh_ = [], []
    for i in range(40):
        b = batches[i % 2]
        lr_.append(t_ref.step(b).detach())
        lh_.append(t_hip.step(b).detach())
    t_hip.flush()
    torch.cuda.synchronize()
    RNN.check_errors()
    a, b, wr, wh, rel, table = _windows(lr_, lh_, 10)
    w_rel = ((t_hip.arena.flat - t_ref.arena.flat).norm() / t_ref.arena.flat.norm()).item()
    print("headline windowed ref/hip loss: %s; max rel %.4f; weights rel %.4f" % (table, float(rel.max()), w_rel))
    assert torch.isfinite(a).all() and torch.isfinite(b).all()
    assert wr[-1] < 0.9 * wr[0] and wh[-1] < 0.9 * wh[0], table       # both learn
    assert float(rel.max()) < 0.05, table
    assert w_rel < 0.05, w_rel
    ema_rel = ((t_hip.opt.ema - t_ref.opt.ema).norm() / t_ref.opt.ema.norm()).item()
    assert ema_rel < 0.05, ema_rel


def test_config5_fp8_30_steps_tracks_bf16(cuda):
    from deepspeech_amd.ops import rnn as RNN
    torch.manual_seed(22)
    N, H = 32, 1280
    base = DeepSpeech2(num_filters=32, num_hidden=H, num_rnn_layers=7, cell="gru").to(cuda)
    f8 = copy.deepcopy(base)
    base.set_engine("hip", torch.bfloat16)
    f8.set_engine("hip", torch.bfloat16, fp8=True)
    plan = RNN.plan_for(N, H, "gru", 2, cuda)
    assert RNN.fp8_recurrence_ok(plan, N) and RNN.fp8_bptt_ok(plan, N)     # the 64-unit fp8 kernels
    batches = [to_device(FixedShapeBatches(N, max_frames=1000, seed=80 + s, pool=1).next(), cuda) for s in range(2)]
    sched = LRSchedule(2e-5, 10 ** 9, 1.0)
    tb, tf = Trainer(base, sched, defer_update=True), Trainer(f8, sched, defer_update=True)
    lb, lf = [], []
    for i in range(30):
        b = batches[i % 2]
        lb.append(tb.step(b).detach())
        lf.append(tf.step(b).detach())
    tb.flush()
    tf.flush()
    torch.cuda.synchronize()
    RNN.check_errors()
    a, b, wb, wf, rel, table = _windows(lb, lf, 10)
    print("config5 windowed bf16/fp8 loss: %s; max rel %.4f" % (table, float(rel.max())))
    assert torch.isfinite(a).all() and torch.isfinite(b).all()
    assert wb[-1] < 0.9 * wb[0] and wf[-1] < 0.9 * wf[0], table
    assert float(rel.max()) < 0.25, table
