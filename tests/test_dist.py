"""Data parallelism without a cluster: gloo process groups on CPU (world size 2)."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(n=2):
    from deepspeech_amd.data.synthetic import FixedShapeBatches
    return [FixedShapeBatches(2, max_frames=140, seed=10 + i, pool=1).next() for i in range(n)]


def _make_trainer(world, bucket_mb):
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.trainer import LRSchedule, Trainer
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=2, cell="gru")
    # BN batch statistics are per rank (parity with the single-device reference); freeze
    # them in eval mode here so that DP == one big batch exactly
    return Trainer(m, LRSchedule(1e-2, 10 ** 6, 0.9), moving_avg_decay=0.99, world_size=world,
                   bucket_mb=bucket_mb)


def _eval_mode_step(tr, batch, update=True):
    tr.model.eval()
    tr.arena.zero_grad()
    logits, lens = tr.model(batch["feats"], batch["seq_lens"])
    loss = tr.model.loss(logits, lens, batch["labels"], batch["label_lens"])
    loss.backward()
    tr.bucketer.finish()
    if update:
        tr.opt.step(tr.lr, tr.global_step, gscale=1.0 / tr.world)
        tr.global_step += 1


def _worker(rank, world, port, bucket_mb, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from deepspeech_amd.data.synthetic import to_device
    from deepspeech_amd.parallel.dist import init_distributed, shutdown
    ctx = init_distributed("cpu")
    tr = _make_trainer(world, bucket_mb)
    assert len(tr.bucketer.buckets) >= (2 if bucket_mb < 0.01 else 1)
    b = _batches()[rank]
    _eval_mode_step(tr, to_device(b, torch.device("cpu")), update=False)
    g = tr.arena.grad.clone() / world
    tr.opt.step(tr.lr, 0, gscale=1.0 / world)
    if rank == 0:
        torch.save({"w": tr.arena.flat.clone(), "g": g}, out)
    shutdown(ctx)


@pytest.mark.parametrize("bucket_mb", [0.001, 32.0])
def test_dp2_equals_single_process_big_batch(tmp_path, bucket_mb):
    from deepspeech_amd.data.synthetic import Batch, to_device
    import numpy as np
    out = str(tmp_path / "dp.pt")
    mp.spawn(_worker, args=(2, _free_port(), bucket_mb, out), nprocs=2, join=True)
    res = torch.load(out, weights_only=True)
    # single process: the mean CTC over the concatenated 4-utterance batch equals the
    # average of the two ranks' per-batch means (equal batch sizes)
    b0, b1 = _batches()
    T = max(b0.feats.shape[1], b1.feats.shape[1])

    def pad(a, T):
        o = np.zeros((a.shape[0], T, a.shape[2]), np.float32)
        o[:, : a.shape[1]] = a
        return o

    L = max(b0.labels.shape[1], b1.labels.shape[1])

    def padl(a):
        o = np.full((a.shape[0], L), -1, np.int32)
        o[:, : a.shape[1]] = a
        return o

    big = Batch(np.concatenate([pad(b0.feats, T), pad(b1.feats, T)]), np.concatenate([b0.seq_lens, b1.seq_lens]),
                np.concatenate([padl(b0.labels), padl(b1.labels)]), np.concatenate([b0.label_lens, b1.label_lens]))
    tr = _make_trainer(1, 32.0)
    _eval_mode_step(tr, to_device(big, torch.device("cpu")), update=False)
    gr = tr.arena.grad.clone()
    tr.opt.step(tr.lr, 0)
    # the all-reduced mean gradient, then one Adam step from identical starts
    # (Adam divides by sqrt(v): elements with |g| ~ eps amplify float-order noise)
    assert torch.allclose(res["w"], tr.arena.flat, atol=2e-3), (res["w"] - tr.arena.flat).abs().max()
    g = res["g"]
    assert ((g - gr).norm() / gr.norm()) < 1e-5


def test_fault_injection_and_resume(tmp_path):
    """Kill the job at step 7, resume from the last checkpoint (step 5) and finish."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    common = [sys.executable, "-m", "deepspeech_amd.train", "--dummy", "True", "--batch_size", "2",
              "--num_hidden", "16", "--num_rnn_layers", "1", "--num_filters", "4", "--device", "cpu",
              "--checkpoint_every", "5", "--log_every", "1000"]
    d = str(tmp_path / "run")
    r = subprocess.run(common + ["--train_dir", d, "--max_steps", "20", "--fault_inject_step", "7"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 17, r.stdout + r.stderr
    from deepspeech_amd.utils import checkpoint as CK
    assert CK.latest_checkpoint(d).endswith("model.ckpt-5")
    r = subprocess.run(common + ["--train_dir", d, "--checkpoint", d, "--max_steps", "12"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert CK.latest_checkpoint(d).endswith("model.ckpt-11")
    assert "has checkpoint" in r.stdout


def test_torchrun_gloo_two_ranks(tmp_path):
    """The real launcher path: torch.distributed.run with 2 CPU ranks over gloo."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", "deepspeech_amd.train",
           "--dummy", "True", "--batch_size", "2", "--num_hidden", "16", "--num_rnn_layers", "1",
           "--num_filters", "4", "--device", "cpu", "--max_steps", "13", "--train_dir", str(tmp_path / "tr"),
           "--log_every", "12"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "step 12" in r.stdout


def test_train_gpus_flag_spawns_ranks_without_launcher(tmp_path):
    """python -m deepspeech_amd.train --gpus 2 (no torchrun): the driver starts its two ranks
    itself (parallel/launch.py), as bench.py does."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", DS2_DIST_BACKEND="gloo")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "deepspeech_amd.train", "--gpus", "2",
           "--dummy", "True", "--batch_size", "2", "--num_hidden", "16", "--num_rnn_layers", "1",
           "--num_filters", "4", "--device", "cpu", "--max_steps", "13", "--train_dir", str(tmp_path / "tr"),
           "--log_every", "12"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "step 12" in r.stdout and "world: 2" in r.stdout


def _run_bench(nproc, extra_env, args, timeout=600):
    import json
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", **extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % nproc,
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def test_bench_two_ranks_json_contract():
    """bench.py under torch.distributed.run with 2 ranks (gloo on CPU): one JSON line, whole-job
    aggregate value (summed audio / max elapsed), n_gpus and dp degree reported."""
    out = _run_bench(2, {"CUDA_VISIBLE_DEVICES": ""},
                     ["--gpus", "2", "--steps", "2", "--warmup", "1", "--batch_size", "2", "--frames", "200",
                      "--num_hidden", "32", "--num_rnn_layers", "1", "--num_filters", "4", "--no_infer"])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 4
    assert out["value"] > 0 and out["ms_per_step"] > 0
    # value is the job aggregate: per-GPU figure x world
    assert abs(out["value"] - 2 * out["per_gpu_audio_sec_per_sec"]) <= 0.02 * out["value"]
    # two ranks' audio (different seeds) summed over 2 steps: lengths are drawn from the
    # top 100-frame bucket, (100, 200] frames at --frames 200 -> 4 utterances x 2 steps x (1, 2] s
    total = out["value"] * out["ms_per_step"] * 2 / 1000.0
    assert 8.0 < total <= 16.0 * 1.01, total


def _run_bench_direct(args, timeout=600):
    import json
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    return r, [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


_TINY = ["--steps", "2", "--warmup", "1", "--batch_size", "2", "--frames", "200", "--num_hidden", "32",
         "--num_rnn_layers", "1", "--num_filters", "4"]
_TINY_NOINF = _TINY + ["--no_infer"]


def test_bench_gpus_flag_spawns_ranks_without_launcher():
    """python bench.py --gpus 2 (no torchrun): bench.py starts the two ranks itself
    (parallel/launch.py) and rank 0 prints one JSON line for the 2-rank job."""
    r, rows = _run_bench_direct(["--gpus", "2", "--infer_seconds", "1"] + _TINY)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert len(rows) == 1, r.stdout
    out = rows[0]
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 4 and out["value"] > 0
    # the inference half of the BASELINE metric: streaming RTF, greedy and beam-16, 1 / 32 streams
    inf = out["inference"]
    for k in ("rtf_greedy_streams1", "rtf_beam16_streams1", "rtf_greedy_streams32", "rtf_beam16_streams32"):
        assert inf[k] > 0, k


def test_bench_gpus_mismatch_with_launcher_fails():
    """--gpus 3 under a 2-rank torchrun is an error, not a silent 2-rank run."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "3"] + _TINY_NOINF
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "does not match the launcher's WORLD_SIZE=2" in r.stdout + r.stderr


def test_launcher_failing_rank_stops_job(tmp_path):
    """A rank that fails ends the job with its exit code and the other ranks are stopped."""
    sys.path.insert(0, ROOT)
    from deepspeech_amd.parallel.launch import spawn_local
    script = tmp_path / "w.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "assert os.environ['WORLD_SIZE'] == '3' and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
                      "open(os.environ['OUT'] + str(r), 'w').write(os.environ['LOCAL_RANK'])\n"
                      "sys.exit(7) if r == 1 else time.sleep(600)\n")
    import time
    t0 = time.time()
    code = spawn_local(3, [sys.executable, str(script)], {"OUT": str(tmp_path / "r")})
    assert code == 7 and time.time() - t0 < 60
    assert sorted(p.name for p in tmp_path.glob("r*")) == ["r0", "r1", "r2"]


def test_scale_harness_cpu_table(tmp_path):
    """tools/scale.py over gloo: the 1- and 2-rank benches plus the bucket-size all-reduce,
    one table with weak-scaling efficiency and busbw."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    out = tmp_path / "scale"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scale.py"), "--cpu", "--worlds", "1,2",
                        "--bucket_mb", "0.5", "--out", str(out), "--"] + _TINY_NOINF,
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    import json
    res = json.loads((out / "scale.json").read_text())
    assert [row["n_gpus"] for row in res["runs"]] == [1, 2]
    assert set(res["allreduce"]) == {"fp32", "bf16"} and res["allreduce"]["fp32"][0]["world"] == 2
    md = (out / "scale.md").read_text()
    assert "| 1 |" in md and "| 2 |" in md and "busbw" in md


def test_allreduce_bandwidth_tool_two_ranks():
    """tools/bench_allreduce.py (nccl-tests conventions) under torch.distributed.run, 2 CPU
    ranks over gloo: one JSON line per size on rank 0 with busbw = algbw * 2(n-1)/n."""
    import json
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tools", "bench_allreduce.py"), "--device", "cpu", "--sizes_mb", "1,2",
           "--iters", "2", "--warmup", "1"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    rows = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert [row["bytes"] for row in rows] == [2 ** 20, 2 * 2 ** 20]
    for row in rows:
        assert row["world"] == 2 and row["backend"] == "gloo"
        assert abs(row["busbw_GBps"] - row["algbw_GBps"] * 2 * (2 - 1) / 2) <= 0.011


def _train_worker(rank, world, port, mode, out):
    """mode 'fp32' / 'bf16': one TRAINING-mode step (per-rank BN batch statistics) with the
    whole-arena update after finish(); 'bucket': the same step with the per-bucket optimizer
    (GradBucketer.set_optimizer: each bucket's Adam range behind its all-reduce)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from deepspeech_amd.data.synthetic import to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.parallel.dist import init_distributed, shutdown
    from deepspeech_amd.trainer import LRSchedule, Trainer
    ctx = init_distributed("cpu")
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=2, cell="gru")
    tr = Trainer(m, LRSchedule(1e-2, 10 ** 6, 0.9), moving_avg_decay=0.99, world_size=world,
                 bucket_mb=0.001, allreduce_bf16=(mode == "bf16"))
    tr.per_bucket_update = mode == "bucket"
    assert len(tr.bucketer.buckets) >= 3
    grads = []
    orig_finish = tr.bucketer.finish

    def finish():                          # capture the reduced (summed) gradient
        orig_finish()
        grads.append(tr.arena.grad.clone())
    tr.bucketer.finish = finish
    losses = [float(tr.step(to_device(b, torch.device("cpu")))) for b in _batches(2 * world)[rank::world]]
    if rank == 0:
        torch.save({"w": tr.arena.flat.clone(), "ema": tr.opt.ema.clone(), "g": grads[0],
                    "losses": torch.tensor(losses)}, out)
    shutdown(ctx)


def _dp_train(tmp_path, mode):
    out = str(tmp_path / ("dp_%s.pt" % mode))
    mp.spawn(_train_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True)
    return torch.load(out, weights_only=True)


def test_dp2_training_mode_equals_local_steps_plus_averaged_update(tmp_path):
    """Training mode (per-rank BN statistics, as in the single-device reference): the DP step
    equals each rank's local gradient computed single-process, averaged, then one Adam step."""
    from deepspeech_amd.data.synthetic import to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.trainer import LRSchedule, Trainer
    res = _dp_train(tmp_path, "fp32")
    bs = _batches(4)
    local = []
    for r in range(2):
        torch.manual_seed(0)
        m = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=2, cell="gru")
        tr = Trainer(m, LRSchedule(1e-2, 10 ** 6, 0.9), moving_avg_decay=0.99)
        tr.model.train()
        tr.arena.zero_grad()
        b = to_device(bs[r], torch.device("cpu"))
        loss = tr.model.forward_loss(b["feats"], b["seq_lens"], b["labels"], b["label_lens"])
        loss.backward()
        local.append(tr.arena.grad.clone())
    gsum = local[0] + local[1]
    assert ((res["g"] - gsum).norm() / gsum.norm()) < 1e-5
    # one Adam step from the same start with the averaged gradient
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=2, cell="gru")
    tr = Trainer(m, LRSchedule(1e-2, 10 ** 6, 0.9), moving_avg_decay=0.99)
    w0 = tr.arena.flat.clone()
    tr.arena.grad.copy_(res["g"])
    tr.opt.step(tr.lr, 0, gscale=0.5)
    assert not torch.equal(tr.arena.flat, w0)


def test_dp2_per_bucket_optimizer_matches_single_update(tmp_path):
    """Per-bucket Adam behind each all-reduce (DP-native ordering) gives bitwise the weights
    and EMA of one whole-arena update after finish(), over two steps."""
    a, b = _dp_train(tmp_path, "bucket"), _dp_train(tmp_path, "fp32")
    assert torch.equal(a["losses"], b["losses"])
    assert torch.equal(a["w"], b["w"]) and torch.equal(a["ema"], b["ema"])


def test_dp2_bf16_compressed_allreduce_close_to_fp32(tmp_path):
    """--allreduce_bf16: buckets summed in bf16 on the wire match the fp32 all-reduce within
    bf16 rounding: each rank's value and the sum round to 8 mantissa bits, so the error of an
    element is ~2^-8 of the ranks' magnitudes (a sum that cancels can be off by more than
    2^-8 of itself), and the gradient norm is off by far less."""
    a, b = _dp_train(tmp_path, "bf16"), _dp_train(tmp_path, "fp32")
    ga, gb = a["g"], b["g"]
    assert not torch.equal(ga, gb)                    # really compressed
    assert ((ga - gb).norm() / gb.norm()) < 8e-3
    assert (ga - gb).abs().max() < 2 ** -7 * gb.abs().max()
