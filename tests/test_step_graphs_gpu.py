"""Captured training steps (Trainer(step_graphs=True)): a replayed step graph is bitwise the
eager step — losses, gradients, weights, Adam moments, EMA and bf16 shadows — over several
shapes, learning-rate changes and an interleaved eager step.
Reference step: src/deepSpeech_train.py:292-380 (sess.run of forward, CTC, backward, Adam,
EMA per step); the dummy bucket walk it is meant for: src/deepSpeech_dummy.py:54-87."""
import copy

import pytest
import torch

from deepspeech_amd.data.synthetic import DummyBucketWalk, FixedShapeBatches, to_device
from deepspeech_amd.models import DeepSpeech2

pytestmark = pytest.mark.gpu


def _padded(batch, width=None):
    S = batch["labels"].shape[1]
    w = width or max(16, -(-S // 16) * 16)
    assert w >= S
    b = dict(batch)
    b["labels"] = torch.nn.functional.pad(batch["labels"], (0, w - S))
    return b


def _state(tr):
    return [tr.arena.flat, tr.arena.grad, tr.opt.m, tr.opt.v, tr.opt.ema, tr.arena.p16]


@pytest.mark.parametrize("H,layers,N", [(256, 2, 8), (800, 3, 32)])
def test_graph_step_bitwise_equals_eager(cuda, H, layers, N):
    from deepspeech_amd.trainer import LRSchedule, Trainer
    torch.manual_seed(0)
    base = DeepSpeech2(num_filters=32, num_hidden=H, num_rnn_layers=layers, cell="gru").to(cuda)
    # two shapes, interleaved; the LR decays every 3 steps so the replayed update must read
    # the staged device scalars, not the values it was captured with
    feeds = {T: FixedShapeBatches(N, max_frames=T, seed=T, pool=3) for T in (200, 400)}
    order = [200, 200, 400, 200, 400, 400, 200, 400, 200, 400]
    batches = [_padded(to_device(feeds[T].next(), cuda), 64 if T == 400 else 32) for T in order]
    sched = LRSchedule(1e-3, 3, 0.5)
    eager = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), sched)
    graph = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), sched, step_graphs=True,
                    graph_warmup=1)
    assert graph.graphs_active()
    le, lg = [], []
    for i, b in enumerate(batches):
        le.append(eager.step(b))
        lg.append(graph.step(b))
        if i == 6:
            # an eager step between replays (e.g. a DP-less debug step): state stays shared
            graph.step_graphs = False
            le.append(eager.step(batches[0]))
            lg.append(graph.step(batches[0]))
            graph.step_graphs = True
    torch.cuda.synchronize()
    assert len(graph._graphs) == 2                     # one graph per shape
    assert [float(x) for x in le] == [float(x) for x in lg]
    for x, y in zip(_state(eager), _state(graph)):
        assert torch.equal(x, y), (x.float() - y.float()).abs().max()


def test_graph_step_bucket_walk_and_ema_swap(cuda):
    """The reference's dummy epoch order (ascending buckets, several shapes) through graphs,
    with an EMA swap (eval on the shadow weights, src/deepSpeech_test.py:217-220) between
    replays: the replay after the swap-back sees the restored bf16 shadows."""
    from deepspeech_amd.trainer import LRSchedule, Trainer
    torch.manual_seed(1)
    base = DeepSpeech2(num_filters=32, num_hidden=256, num_rnn_layers=2, cell="gru").to(cuda)
    walk = DummyBucketWalk(8, seed=0, scale_factor=1)
    bs = []
    for i in (0, 0, 0, 3, 3, 3, 4, 4, 4, 0):
        bs.append(to_device(walk.batch_for(i), cuda))
    eager = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), LRSchedule(1e-3, 100, 0.9))
    graph = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), LRSchedule(1e-3, 100, 0.9),
                    step_graphs=True, graph_warmup=2)
    for i, b in enumerate(bs):
        b = _padded(b)
        eager.step(b)
        graph.step(b)
        if i == 7:
            for tr in (eager, graph):
                tr.swap_ema()
                tr.swap_ema()
    torch.cuda.synchronize()
    assert len(graph._graphs) == 3
    for x, y in zip(_state(eager), _state(graph)):
        assert torch.equal(x, y), (x.float() - y.float()).abs().max()


def test_auto_mode_decides_per_shape_and_stays_bitwise(cuda):
    """step_graphs="auto": each shape times eager steps against replays once and keeps the
    faster; whichever it keeps, the trajectory is bitwise the eager one."""
    from deepspeech_amd.trainer import LRSchedule, Trainer
    torch.manual_seed(2)
    base = DeepSpeech2(num_filters=32, num_hidden=256, num_rnn_layers=2, cell="gru").to(cuda)
    feeds = {T: FixedShapeBatches(8, max_frames=T, seed=T, pool=2) for T in (100, 300)}
    order = [100] * 10 + [300] * 10 + [100, 300] * 2
    batches = [_padded(to_device(feeds[T].next(), cuda), 32 if T == 100 else 64) for T in order]
    eager = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), LRSchedule(1e-3, 4, 0.7))
    auto = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), LRSchedule(1e-3, 4, 0.7),
                   step_graphs="auto", graph_warmup=1)
    for b in batches:
        eager.step(b)
        auto.step(b)
    torch.cuda.synchronize()
    assert len(auto.graph_modes) == 2
    for mode, te, tg in auto.graph_modes.values():
        assert mode in ("eager", "graph") and te > 0 and tg > 0
    for x, y in zip(_state(eager), _state(auto)):
        assert torch.equal(x, y), (x.float() - y.float()).abs().max()


def test_auto_mode_recaptures_after_every_graph_was_dropped(cuda, monkeypatch):
    """Every shape so far decided for eager (its graph dropped, and with the last graph PyTorch
    frees the shared memory pool): the next shape's capture must start a fresh pool instead of
    naming the dead one (allocator assert at capture_begin, seen on config 5's epoch walk)."""
    from deepspeech_amd import trainer as TRN
    from deepspeech_amd.trainer import LRSchedule, Trainer
    torch.manual_seed(4)
    base = DeepSpeech2(num_filters=32, num_hidden=256, num_rnn_layers=2, cell="gru").to(cuda)
    feeds = {T: FixedShapeBatches(8, max_frames=T, seed=T, pool=2) for T in (100, 200, 300)}
    order = [100] * 6 + [200] * 6 + [300] * 6
    batches = [_padded(to_device(feeds[T].next(), cuda), 32 if T == 100 else 64) for T in order]
    eager = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), LRSchedule(1e-3, 4, 0.7))
    auto = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), LRSchedule(1e-3, 4, 0.7),
                   step_graphs="auto", graph_warmup=1)
    # a frozen host clock: every eager step looks free to issue, so every shape picks eager
    monkeypatch.setattr(TRN, "_clock", lambda: 0.0)
    for b in batches:
        eager.step(b)
        auto.step(b)
        torch.cuda.synchronize()
    assert len(auto.graph_modes) == 3 and all(m == "eager" for m, _, _ in auto.graph_modes.values())
    for x, y in zip(_state(eager), _state(auto)):
        assert torch.equal(x, y), (x.float() - y.float()).abs().max()


def test_timing_only_knobs_refused_and_masked(cuda, monkeypatch):
    """DS2_RNNX_KNOBS bits that skip work (2, 4, 8, 32) make a training step refuse to run and
    never reach a kernel outside an explicit timing session (DS2_TIMING_ONLY=1) (VERDICT r4
    item 6)."""
    from deepspeech_amd.ops import rnn as RNN
    from deepspeech_amd.trainer import LRSchedule, Trainer
    monkeypatch.delenv("DS2_TIMING_ONLY", raising=False)
    m = DeepSpeech2(num_filters=32, num_hidden=64, num_rnn_layers=1, cell="gru").to(cuda)
    m.set_engine("hip", torch.bfloat16)
    for bit in (2, 4, 8, 32):
        monkeypatch.setattr(RNN, "RNNX_KNOBS", bit | 16384)
        with pytest.raises(RuntimeError, match="timing only"):
            Trainer(m, LRSchedule(1e-3, 10, 0.9))
        # masked at every launch regardless (the poll-timing default bits aside)
        assert RNN._kernel_knobs() & ~RNN.POLL_MASK == 16384
        assert RNN._kernel_knobs() & RNN.POLL_MASK == RNN.POLL_DEFAULT
    monkeypatch.setattr(RNN, "RNNX_KNOBS", 16384)      # a schedule variant with correct results
    RNN.check_knobs()
    monkeypatch.setenv("DS2_TIMING_ONLY", "1")
    monkeypatch.setattr(RNN, "RNNX_KNOBS", 4)
    RNN.check_knobs()
    assert RNN._kernel_knobs() == 4 | RNN.POLL_DEFAULT
    monkeypatch.setattr(RNN, "RNNX_KNOBS", 4 | RNN.POLL_EXPLICIT)    # explicit poll timing 0
    assert RNN._kernel_knobs() == 4 | RNN.POLL_EXPLICIT
