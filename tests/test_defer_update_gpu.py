"""Optimizer update carried into the next step (Trainer(defer_update=True), VERDICT r5 next-round
item 1a): the FC head's and recurrent layers >= 1's Adam + EMA range of step s runs on the side
stream beside step s+1's first recurrence instead of in step s's tail. Every element's update is
independent of when and in which launch it runs, so the trajectory must be BITWISE the plain
schedule's: losses (step s+1's forward reads the carried weights), gradients, weights, Adam
moments, EMA and bf16 shadows, through step graphs, an EMA swap and a checkpoint.
Reference: src/deepSpeech_train.py:457-465 (apply_gradients + EMA grouped as train_op, run every
step before the next sess.run)."""
import copy
import os

import pytest
import torch

from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
from deepspeech_amd.models import DeepSpeech2

pytestmark = pytest.mark.gpu


def _state(tr):
    return [tr.arena.flat, tr.arena.grad, tr.opt.m, tr.opt.v, tr.opt.ema, tr.arena.p16]


def _pair(cuda, H, layers, sched, **kw):
    from deepspeech_amd.trainer import Trainer
    torch.manual_seed(0)
    base = DeepSpeech2(num_filters=32, num_hidden=H, num_rnn_layers=layers, cell="gru").to(cuda)
    plain = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), sched, **kw)
    carry = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), sched, defer_update=True, **kw)
    return plain, carry


def test_carried_update_bitwise_at_the_headline(cuda, tmp_path):
    """20 steps of the headline model (5 x BiGRU-800, batch 32, 1000 frames: partial weight-
    gradient deferral, capped beside grids and the carried upper range are all active), an EMA
    swap in the middle, then a checkpoint after flush(): bitwise the plain schedule."""
    from deepspeech_amd.trainer import LRSchedule
    from deepspeech_amd.utils import checkpoint as CK
    plain, carry = _pair(cuda, 800, 5, LRSchedule(1e-3, 5, 0.7))
    feed = FixedShapeBatches(32, max_frames=1000, seed=3, pool=3)
    batches = [to_device(feed.next(), cuda) for _ in range(3)]
    lp, lc = [], []
    for i in range(20):
        b = batches[i % 3]
        lp.append(plain.step(b))
        lc.append(carry.step(b))
        if i == 0:
            torch.cuda.synchronize()
            # the update really was carried: a range is pending after the step
            assert carry.arena.has_pending_update()
            assert not plain.arena.has_pending_update()
        if i == 9:
            for tr in (plain, carry):
                tr.swap_ema()
                tr.swap_ema()
    carry.flush()
    torch.cuda.synchronize()
    assert not carry.arena.has_pending_update()
    assert [float(x) for x in lp] == [float(x) for x in lc]
    for x, y in zip(_state(plain), _state(carry)):
        assert torch.equal(x, y), (x.float() - y.float()).abs().max()
    # checkpoints through the asynchronous writer (device snapshot -> pinned -> file)
    saved = []
    for name, tr in (("plain", plain), ("carry", carry)):
        d = os.path.join(str(tmp_path), name)
        m = CK.CheckpointManager(d, async_save=True)
        m.save(tr, 19, force=True)
        m.close()
        saved.append(CK.read_checkpoint(CK.latest_checkpoint(d)))
    a, b = saved
    assert sorted(a) == sorted(b)
    for k in a:
        if isinstance(a[k], torch.Tensor):
            assert torch.equal(a[k], b[k]), k
        else:
            assert a[k] == b[k], k


def test_carried_update_with_step_graphs(cuda):
    """Eager steps that carry their update and replayed step graphs (which never carry one)
    interleaved over two shapes: bitwise the plain eager trajectory."""
    from deepspeech_amd.trainer import LRSchedule, Trainer
    torch.manual_seed(1)
    base = DeepSpeech2(num_filters=32, num_hidden=256, num_rnn_layers=3, cell="gru").to(cuda)
    feeds = {T: FixedShapeBatches(8, max_frames=T, seed=T, pool=2) for T in (300, 1000)}
    order = [1000, 1000, 300, 300, 1000, 300, 1000, 1000, 300, 1000]
    batches = [to_device(feeds[T].next(), cuda) for T in order]
    for b in batches:
        S = b["labels"].shape[1]
        b["labels"] = torch.nn.functional.pad(b["labels"], (0, 256 - S))
    sched = LRSchedule(1e-3, 3, 0.5)
    plain = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), sched)
    mixed = Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), sched, defer_update=True,
                    step_graphs=True, graph_warmup=1)
    lp, lm = [], []
    for i, b in enumerate(batches):
        lp.append(plain.step(b))
        if i in (4, 5):
            mixed.step_graphs = False       # eager steps between replays carry their update
        lm.append(mixed.step(b))
        mixed.step_graphs = True
    mixed.flush()
    torch.cuda.synchronize()
    assert [float(x) for x in lp] == [float(x) for x in lm]
    for x, y in zip(_state(plain), _state(mixed)):
        assert torch.equal(x, y), (x.float() - y.float()).abs().max()
