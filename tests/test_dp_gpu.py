"""Data-parallel gradient path of the HIP engine on a GPU: 2 ranks sharing cuda:0 over gloo
(torch.distributed.run), side-stream weight gradients + multi-bucket all-reduce."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("geom", ["small", "config5"])
def test_dp2_gradients_equal_sum_of_local(cuda, tmp_path, geom):
    """2 ranks on one GPU over gloo: the all-reduced gradient equals the sum of the local ones,
    and a full per-bucket DP step equals one update of the averaged gradients. "config5":
    BASELINE config 5's 7 x BiGRU-1280 in fp8 mode."""
    out = str(tmp_path / "g")
    env = dict(os.environ, PYTHONPATH=ROOT, DS2_DIST_BACKEND="gloo", DS2_DEVICE_INDEX="0", OMP_NUM_THREADS="2",
               DS2_DP_GEOM=geom)
    if geom == "config5":
        # Both ranks share ONE GPU here: each persistent recurrence grid of this geometry needs
        # 160 of the 256 CUs co-resident, so when the two ranks' recurrences overlap in time
        # neither grid is fully resident and their bounded spins time out (error word 0x3, the
        # outputs garbage: measured 2-4 steps in 13). On one GPU per rank that cannot happen;
        # this test therefore runs the recurrences as per-step launches (generation 1, no
        # co-residency), which keeps the fp8 projections, the buckets, the all-reduces and the
        # per-bucket optimizer of the config-5 geometry. The fp8 recurrence itself under the
        # DP schedule is covered at world size 1 (tests/test_dp_ready_gpu.py, force_dp).
        env["DS2_RNN_MODE"] = "step"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dp_gpu_worker.py"), out]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    g = [torch.load("%s.%d" % (out, k), weights_only=True) for k in range(2)]
    want = g[0]["local"] + g[1]["local"]
    for k in range(2):
        err = ((g[k]["dp"] - want).norm() / want.norm()).item()
        assert err < 1e-5, (k, err)
    # the full step: both ranks hold the same weights, equal to one Adam update of the
    # averaged local gradients (per-rank BN statistics, as single-device training)
    assert torch.equal(g[0]["w_step"], g[1]["w_step"]) and torch.equal(g[0]["ema_step"], g[1]["ema_step"])
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from deepspeech_amd.trainer import LRSchedule, Trainer
    import dp_gpu_worker as W
    tr = Trainer(W.model(cuda, geom), LRSchedule(1e-3, 10 ** 6, 0.9))
    w0 = tr.arena.flat.clone()
    tr.arena.grad.copy_((g[0]["step_local"] + g[1]["step_local"]).to(cuda))
    tr.opt.step(tr.lr, 0, gscale=0.5)
    w_ref = tr.arena.flat.cpu()
    moved = (w_ref - w0.cpu()).abs()
    assert moved.max() > 1e-4                                 # the step did something
    # Adam's first update is ~lr * sign(g): the same weights up to elements whose averaged
    # gradient is ~eps-sized (float summation order)
    assert ((g[0]["w_step"] - w_ref).abs() > 1e-5).float().mean() < 1e-3
    assert (g[0]["w_step"] - w_ref).abs().max() < 2.5e-3
    del tr
    torch.cuda.empty_cache()


def test_bench_gpus2_self_launch_on_one_gpu():
    """bench.py --gpus 2 without torchrun on the GPU path: two HIP-engine ranks started by
    bench.py itself (parallel/launch.py), sharing cuda:0 over gloo (RCCL refuses two ranks
    on one device), full DP step (bucketed all-reduce + per-bucket Adam); rank 0 prints the
    2-rank job's JSON line."""
    import json
    env = dict(os.environ, PYTHONPATH=ROOT, DS2_DIST_BACKEND="gloo", DS2_DEVICE_INDEX="0", OMP_NUM_THREADS="2")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2",
           "--batch_size", "8", "--frames", "300", "--num_hidden", "256", "--num_rnn_layers", "2"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    rows = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(rows) == 1 and rows[0]["n_gpus"] == 2 and rows[0]["config"]["parallelism"] == "dp2"
    assert rows[0]["config"]["engine"] == "hip" and rows[0]["final_loss"] == rows[0]["final_loss"]
