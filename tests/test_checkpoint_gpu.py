"""Non-blocking checkpoints on the GPU (utils/checkpoint.py CheckpointManager, VERDICT r4 item 3;
reference cadence src/deepSpeech_train.py:354-356, saver at :471)."""
import copy
import os
import time

import pytest
import torch

from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
from deepspeech_amd.models import DeepSpeech2

pytestmark = pytest.mark.gpu


def _trainer(base, **kw):
    from deepspeech_amd.trainer import LRSchedule, Trainer
    return Trainer(copy.deepcopy(base).set_engine("hip", torch.bfloat16), LRSchedule(1e-3, 100, 0.9), **kw)


def _base(cuda, H=256):
    torch.manual_seed(0)
    return DeepSpeech2(num_filters=32, num_hidden=H, num_rnn_layers=2, cell="gru").to(cuda)


@pytest.mark.parametrize("graphs", [False, True])
def test_async_checkpoint_is_bitwise_the_synchronous_snapshot(cuda, tmp_path, graphs):
    """Save at step 2 without any host synchronisation, keep training (the next steps rewrite
    the weights, moments and EMA the snapshot was taken from), then compare the file with a
    synchronous snapshot of an identical trainer stopped at the same step."""
    from deepspeech_amd.utils import checkpoint as CK
    base = _base(cuda)
    batches = [to_device(b, cuda) for b in FixedShapeBatches(8, max_frames=300, seed=5, pool=3).batches]
    a = _trainer(base, step_graphs=graphs, graph_warmup=1)
    ck = CK.CheckpointManager(str(tmp_path / "a"))
    for i in range(3):
        a.step(batches[i % 3])
    ck.save(a, 2)
    for i in range(3, 9):
        a.step(batches[i % 3])
    ck.close()
    got = CK.load_checkpoint_file(str(tmp_path / "a" / "model.ckpt-2"))
    b = _trainer(base)
    for i in range(3):
        b.step(batches[i % 3])
    torch.cuda.synchronize()
    # the synchronous path's file, through the same (TF bundle) format
    CK.CheckpointManager(str(tmp_path / "b"), async_save=False).save(b, 2)
    want = CK.load_checkpoint_file(str(tmp_path / "b" / "model.ckpt-2"))
    assert set(got) == set(want)
    for k, v in want.items():
        if isinstance(v, torch.Tensor):
            assert torch.equal(got[k], v), k
        else:
            assert got[k] == v, k
    assert CK.latest_checkpoint(str(tmp_path / "a")).endswith("model.ckpt-2")
    # the restored trainer continues exactly like the one that was never stopped
    c = _trainer(base)
    assert CK.restore(c, str(tmp_path / "a")) == 2 and c.global_step == 3
    for i in range(3, 5):
        b.step(batches[i % 3])
        c.step(batches[i % 3])
    torch.cuda.synchronize()
    assert torch.equal(b.arena.flat, c.arena.flat) and torch.equal(b.opt.ema, c.opt.ema)


def test_writer_behind_skips_saves_without_blocking(cuda, tmp_path):
    """Writer busy: saves requested meanwhile take no snapshot and return at once (the training
    thread never waits for the disk); a forced save (end of training) waits and is written."""
    from deepspeech_amd.utils import checkpoint as CK
    base = _base(cuda)
    batch = to_device(FixedShapeBatches(8, max_frames=300, seed=6, pool=1).next(), cuda)
    a = _trainer(base)
    ck = CK.CheckpointManager(str(tmp_path))
    real = ck._write

    def slow(snap, step):
        time.sleep(1.0)
        real(snap, step)
    ck._write = slow
    t0 = time.perf_counter()
    paths = []
    for s in range(4):
        a.step(batch)
        paths.append(ck.save(a, s))
    issued = time.perf_counter() - t0
    a.step(batch)
    assert ck.save(a, 4, force=True) is not None
    ck.close()
    assert issued < 1.0, issued                 # never waited for the 1 s writes
    assert paths[0] is not None and paths[1:] == [None] * 3
    assert ck.written == [0, 4] and ck.skipped == [1, 2, 3]
    assert CK.latest_checkpoint(str(tmp_path)).endswith("model.ckpt-4")


@pytest.mark.parametrize("policy", ["skip", "abort"])
def test_nonfinite_step_and_async_saves(cuda, tmp_path, policy):
    """a NaN loss injected at step 1 (a NaN FC bias for that one step: the clipped
    ReLUs would scrub non-finite features). Under nan_policy skip the update is skipped (every
    weight as before the step), and every later asynchronous save is still written; under abort
    the saves at or after the bad step are dropped and reported."""
    from deepspeech_amd.trainer import LRSchedule, Trainer
    from deepspeech_amd.utils import checkpoint as CK
    base = _base(cuda)
    m = copy.deepcopy(base).set_engine("hip", torch.bfloat16)
    tr = Trainer(m, LRSchedule(1e-3, 100, 0.9), nan_policy=policy)
    good = to_device(FixedShapeBatches(8, max_frames=300, seed=7, pool=1).next(), cuda)
    ck = CK.CheckpointManager(str(tmp_path), nan_policy=policy)
    tr.step(good)
    torch.cuda.synchronize()
    before = tr.arena.flat.clone()
    saved = m.fc_bias.detach().clone()
    with torch.no_grad():
        m.fc_bias[0] = float("nan")
    tr.arena.mark_dirty()
    loss = tr.step(good)
    with torch.no_grad():
        m.fc_bias.copy_(saved)
    tr.arena.mark_dirty()
    torch.cuda.synchronize()
    assert not torch.isfinite(loss).all()
    w_after_bad = tr.arena.flat.clone()
    if policy == "skip":
        assert torch.equal(w_after_bad, before)          # the whole update was skipped
    tr.step(good)
    ck.save(tr, 2, force=True)
    ck.close()
    torch.cuda.synchronize()
    assert tr.first_nonfinite_step() == 1
    if policy == "skip":
        assert torch.isfinite(w_after_bad).all() and torch.isfinite(tr.arena.flat).all()
        assert ck.written == [2] and ck.dropped == []
        assert CK.latest_checkpoint(str(tmp_path)).endswith("model.ckpt-2")
    else:
        assert ck.written == [] and ck.dropped == [2]
