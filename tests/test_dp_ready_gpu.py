"""Data-parallel readiness on one GPU (no 8-GPU node needed); the 2-rank gradient path is
tests/test_dp_gpu.py.

* co-residency: the persistent recurrence (200 co-resident workgroups at the headline
  shape) must complete without a spin timeout while RCCL-channel-shaped workgroups hold CUs,
  whichever launches first (tools/coresidency.py);
* the data-parallel step machinery (process group over RCCL at world size 1, gradient
  buckets, collectives on the ordering stream) produces the same update as the plain step.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("blocks,lds", [(32, 16384), (64, 16384), (56, 100 * 1024)])
def test_recurrence_coresident_with_channel_blocks(cuda, blocks, lds):
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import coresidency
    res = coresidency.run([blocks], threads=256, lds=lds, spin_ms=2.0, iters=2)
    for r in res:
        assert r["timeout"] is None, r
        # the layer may wait for the spinners' CUs but never longer than the spin itself
        assert r["layer_ms"] < r["layer_ms_alone"] + 2.0 * r["spin_ms"] + 1.0, r


def test_fp8_recurrence_coresident_with_channel_blocks(cuda):
    """BASELINE config 5's fp8 layer (BiGRU-1280, batch 32: e4m3 forward recurrence, fp8
    BPTT, their projection and weight gradients) beside 32 RCCL-channel-shaped workgroups,
    whichever launches first: no spin timeout, bounded delay."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import coresidency
    res = coresidency.run([32], threads=256, lds=16384, spin_ms=2.0, iters=2, H=1280, N=32, T=121, fp8=True)
    for r in res:
        assert r["timeout"] is None, r
        assert r["layer_ms"] < r["layer_ms_alone"] + 2.0 * r["spin_ms"] + 1.0, r


# (hidden, layers, fp8, batch, bucket_split_after): the round-1 small GRU; the same with a bucket
# that holds conv2.weight alone, so its Adam range (which rewrites the bf16 shadow conv2's data
# gradient reads) is issued the moment conv2.weight reports; BASELINE config 5
# (7 x BiGRU-1280, fp8 projections / recurrence / BPTT, batch 32)
_DP_CASES = [(128, 2, False, 8, ()), (128, 2, False, 8, ("conv2.bias", "conv2.weight")),
             (1280, 7, True, 32, ())]


@pytest.mark.parametrize("H,layers,fp8,N,split_after", _DP_CASES)
def test_dp_machinery_world1_matches_plain_step(cuda, H, layers, fp8, N, split_after):
    """force_buckets: gradient buckets + collectives at world size 1 give the plain update."""
    import copy
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.parallel.dist import init_distributed, shutdown
    from deepspeech_amd.trainer import LRSchedule, Trainer
    ctx = init_distributed("cuda", force_group=True)
    try:
        torch.manual_seed(0)
        base = DeepSpeech2(num_filters=32, num_hidden=H, num_rnn_layers=layers, cell="gru").to(cuda)
        batch = to_device(FixedShapeBatches(N, max_frames=300, seed=2, pool=1).next(), cuda)
        outs = []
        # plain step; buckets + one update after finish(); buckets + per-bucket Adam ranges
        for force, per_bucket in ((False, False), (True, False), (True, True)):
            m = copy.deepcopy(base).set_engine("hip", torch.bfloat16, fp8=fp8)
            tr = Trainer(m, LRSchedule(1e-4, 1000, 0.9), force_buckets=force, bucket_split_after=split_after)
            if split_after and force:
                last = [tr.arena.names[idx[-1]] for _, _, idx in tr.bucketer.buckets]
                assert [tr.arena.names[i] for i in tr.bucketer.buckets[last.index("conv2.weight")][2]] == \
                    ["conv2.weight"]
            tr.per_bucket_update = per_bucket
            assert tr.bucketer.enabled == force
            for _ in range(2):
                tr.step(batch)
            torch.cuda.synchronize()
            outs.append((tr.arena.flat.clone(), tr.opt.ema.clone(), tr.arena.p16.clone()))
        # the two bucketed runs share one gradient schedule: bitwise the same update
        for x, y in zip(outs[1], outs[2]):
            assert torch.equal(x, y), (x.float() - y.float()).abs().max()
        # the plain single-device step defers every weight gradient into one grouped GEMM
        # (full-K tiles) where the bucketed schedule runs them per layer (split-K beside the
        # BPTT): the same update up to fp32 summation order
        for x, y in zip(outs[0][:2], outs[1][:2]):
            d = (x - y).abs()
            tol = 1e-6 + 1e-5 * y.abs().max()
            if not fp8:
                assert d.max() <= tol
            else:
                # 146 M parameters: Adam's first steps move ~lr * sign(g), so an element whose
                # gradient is ~0 may step the other way under a different summation order
                assert (d > tol).float().mean() < 1e-4 and d.max() <= 4e-4
        assert (outs[0][2] != outs[1][2]).float().mean() < 1e-3     # bf16 shadows: rare 1-ulp flips
    finally:
        shutdown(ctx)           # later GPU tests must not run with a live RCCL group


@pytest.mark.parametrize("H,layers,N,mb", [(128, 3, 8, 1.0), (800, 5, 32, 32.0)])
def test_dp_carried_bucket_updates_bitwise(cuda, H, layers, N, mb):
    """Data parallel + defer_update (world size 1 over RCCL, force_buckets): the head's and upper
    layers' bucket updates go to the next forward (waiting for their all-reduce events), the
    rest stay behind their collectives; only for long sequences. 6 steps over two shapes:
    bitwise the per-bucket run."""
    import copy
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.parallel.dist import init_distributed, shutdown
    from deepspeech_amd.trainer import LRSchedule, Trainer
    ctx = init_distributed("cuda", force_group=True)
    try:
        torch.manual_seed(3)
        base = DeepSpeech2(num_filters=32, num_hidden=H, num_rnn_layers=layers, cell="gru").to(cuda)
        bs = [to_device(FixedShapeBatches(N, max_frames=T, seed=T, pool=1).next(), cuda) for T in (300, 1000)]
        outs, losses = [], []
        for carry in (False, True):
            m = copy.deepcopy(base).set_engine("hip", torch.bfloat16)
            tr = Trainer(m, LRSchedule(1e-3, 2, 0.5), force_buckets=True, defer_update=carry,
                         bucket_mb=mb)
            ls = []
            for i in range(6):
                ls.append(float(tr.step(bs[i % 2])))
                if carry:
                    # carried after the 1000-frame steps only (>= 200 recurrence steps)
                    assert tr.arena.has_pending_update() == (i % 2 == 1)
            tr.flush()
            torch.cuda.synchronize()
            losses.append(ls)
            outs.append((tr.arena.flat.clone(), tr.opt.m.clone(), tr.opt.v.clone(), tr.opt.ema.clone(),
                         tr.arena.p16.clone()))
        assert losses[0] == losses[1]
        for x, y in zip(*outs):
            assert torch.equal(x, y), (x.float() - y.float()).abs().max()
    finally:
        shutdown(ctx)


def test_dp_step_graphs_bitwise_eager(cuda):
    """The data-parallel step captured into per-shape HIP graphs (Trainer dp_graphs: RCCL
    all-reduces, per-bucket Adam + EMA and the ordering stream inside the graph) at world size 1
    over RCCL: 10 steps over two shapes, bitwise the eager --force_dp step in losses, weights,
    Adam moments, EMA and bf16 shadows."""
    import copy
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.parallel.dist import init_distributed, shutdown
    from deepspeech_amd.trainer import LRSchedule, Trainer
    ctx = init_distributed("cuda", force_group=True)
    try:
        torch.manual_seed(5)
        base = DeepSpeech2(num_filters=32, num_hidden=256, num_rnn_layers=3, cell="gru").to(cuda)
        bs = [to_device(FixedShapeBatches(16, max_frames=T, seed=T, pool=1).next(), cuda) for T in (100, 300)]
        outs, losses = [], []
        for graphs in (False, True):
            m = copy.deepcopy(base).set_engine("hip", torch.bfloat16)
            tr = Trainer(m, LRSchedule(1e-3, 3, 0.5), force_buckets=True, bucket_mb=1.0,
                         step_graphs=graphs, dp_graphs=graphs, graph_warmup=1, defer_update=True)
            assert tr.graphs_active() == graphs
            ls = [float(tr.step(bs[(i // 2) % 2])) for i in range(10)]
            if graphs:
                assert len(tr._graphs) == 2                   # both shapes captured and replayed
            tr.flush()
            torch.cuda.synchronize()
            losses.append(ls)
            outs.append((tr.arena.flat.clone(), tr.opt.m.clone(), tr.opt.v.clone(), tr.opt.ema.clone(),
                         tr.arena.p16.clone()))
        assert losses[0] == losses[1], losses
        for x, y in zip(*outs):
            assert torch.equal(x, y), (x.float() - y.float()).abs().max()
    finally:
        shutdown(ctx)
