"""Worker of tests/test_dp_gpu.py (run under torch.distributed.run, 2 ranks on cuda:0 over
gloo): checks that the all-reduced gradient of the HIP engine — with the recurrent weight
gradients produced on the side stream and small buckets that mix streams — equals the sum
of the ranks' local gradients, and that a full training-mode DP step (per-rank BN, Adam
ranges issued per bucket behind the all-reduces) gives the update of the averaged local
gradients."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device  # noqa: E402
from deepspeech_amd.models import DeepSpeech2  # noqa: E402
from deepspeech_amd.ops.rnn import join_wgrad_streams  # noqa: E402
from deepspeech_amd.parallel.dist import init_distributed, shutdown  # noqa: E402
from deepspeech_amd.trainer import LRSchedule, Trainer  # noqa: E402


# geometries: "small" (2 x BiGRU-64) and BASELINE config 5's (7 x BiGRU-1280 in fp8 mode: MX-fp8
# projections, e4m3 forward recurrence, fp8 BPTT), selected by DS2_DP_GEOM
GEOMS = {"small": dict(num_hidden=64, num_rnn_layers=2, fp8=False, batch=4, bucket_mb=0.05),
         "config5": dict(num_hidden=1280, num_rnn_layers=7, fp8=True, batch=8, bucket_mb=32.0)}


def geom(name=None):
    return GEOMS[name or os.environ.get("DS2_DP_GEOM", "small")]


def model(dev, name=None):
    g = geom(name)
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=32, num_hidden=g["num_hidden"], num_rnn_layers=g["num_rnn_layers"],
                    cell="gru").to(dev)
    return m.set_engine("hip", torch.bfloat16, fp8=g["fp8"])


def step_grads(tr, batch):
    """Local gradient of the fused training path Trainer.step runs (forward_loss)."""
    tr.model.train()
    tr.arena.zero_grad(lazy=True)
    tr.model.forward_loss(batch["feats"], batch["seq_lens"], batch["labels"], batch["label_lens"]).backward()
    join_wgrad_streams()
    tr.arena.zero_unwritten()
    torch.cuda.synchronize()
    return tr.arena.grad.clone()


def grads(tr, batch, dp):
    tr.model.train()
    tr.arena.zero_grad(lazy=True)
    logits, lens = tr.model(batch["feats"], batch["seq_lens"])
    tr.model.loss(logits, lens, batch["labels"], batch["label_lens"]).backward()
    join_wgrad_streams()
    tr.arena.zero_unwritten()
    if dp:
        tr.bucketer.finish()
    torch.cuda.synchronize()
    return tr.arena.grad.clone()


def diagnose(out, names_offsets):
    g = [torch.load("%s.%d" % (out, k), weights_only=True) for k in range(2)]
    want = g[0]["local"] + g[1]["local"]
    for name, (o, n) in names_offsets:
        w = want[o:o + n]
        for k in range(2):
            d = g[k]["dp"][o:o + n]
            err = ((d - w).norm() / (w.norm() + 1e-30)).item()
            if err > 1e-5:
                print("rank%d %-22s err %.3e  |dp| %.3e |want| %.3e |local%d| %.3e" % (
                    k, name, err, d.norm(), w.norm(), k, g[k]["local"][o:o + n].norm()))


def main():
    out = sys.argv[1]
    ctx = init_distributed("cuda")
    dev = ctx.device
    batch = to_device(FixedShapeBatches(geom()["batch"], max_frames=300, seed=100 + ctx.rank, pool=1).next(), dev)
    local = Trainer(model(dev), LRSchedule(1e-3, 10 ** 6, 0.9), world_size=1)
    g_local = grads(local, batch, dp=False)
    bmb = float(os.environ.get("DS2_DP_BUCKET_MB", str(geom()["bucket_mb"])))
    dp = Trainer(model(dev), LRSchedule(1e-3, 10 ** 6, 0.9), world_size=ctx.world_size, bucket_mb=bmb)
    assert len(dp.bucketer.buckets) >= (3 if bmb < 1 else 1)
    if ctx.rank == 0 and os.environ.get("DS2_DP_DIAG"):
        for bi, (s0, e0, idx) in enumerate(dp.bucketer.buckets):
            print("bucket", bi, s0, e0, [dp.arena.names[i] for i in idx])
    g_dp = grads(dp, batch, dp=True)
    # one full DP training step (per-bucket optimizer) from the initial weights
    g_step = step_grads(Trainer(model(dev), LRSchedule(1e-3, 10 ** 6, 0.9), world_size=1), batch)
    tr = Trainer(model(dev), LRSchedule(1e-3, 10 ** 6, 0.9), world_size=ctx.world_size, bucket_mb=bmb)
    assert tr.bucketer.enabled and tr.per_bucket_update
    tr.step(batch)
    torch.cuda.synchronize()
    from deepspeech_amd.ops.rnn import check_errors
    check_errors()           # a recurrence that timed out (grid not co-resident) fails loudly
    torch.save({"local": g_local.cpu(), "dp": g_dp.cpu(), "step_local": g_step.cpu(),
                "w_step": tr.arena.flat.cpu(), "ema_step": tr.opt.ema.cpu()}, "%s.%d" % (out, ctx.rank))
    torch.distributed.barrier()
    if ctx.rank == 0 and os.environ.get("DS2_DP_DIAG"):
        diagnose(out, list(zip(dp.arena.names, dp.arena.offsets)))
    shutdown(ctx)


if __name__ == "__main__":
    main()

