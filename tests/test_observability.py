"""Summaries, divergence detection and elastic resume (CPU).

Reference: activation histograms + sparsity (src/helper_routines.py:15-28), gradient /
variable histograms (src/deepSpeech_train.py:401-416), the per-step NaN assert (:325) and
the manual --checkpoint resume (:383-398). Extensions: device-side divergence watch read at
sync points, --resume auto / torchrun --max-restarts.
"""
import glob
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from deepspeech_amd.utils import stats as S
from deepspeech_amd.utils.summary import read_events, read_histograms

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_tf_bucket_limits_shape():
    lim = S.limits()
    assert lim.shape == (S.NBUCKET,)
    assert np.all(np.diff(lim) > 0)
    assert lim[S.NPOS] == 0.0 and abs(lim[S.NPOS + 1] - 1e-12) < 1e-24 and abs(lim[S.NPOS - 1] + 1e-12) < 1e-24


def test_histogram_buckets_contain_their_values():
    rng = np.random.default_rng(0)
    v = np.concatenate([rng.standard_normal(5000) * 10.0 ** rng.integers(-8, 8, 5000), np.zeros(100),
                        [np.nan, np.inf]]).astype(np.float32)
    st = S.histogram(torch.from_numpy(v))
    assert st.num == 5100 and st.nonfinite == 2 and st.zeros == 100
    assert abs(st.zero_fraction - 100 / 5100) < 1e-12
    assert st.counts.sum() == 5100
    lim = S.limits()
    fin = v[np.isfinite(v)].astype(np.float64)
    idx = S._bucket_index_np(fin)
    lo = np.where(idx > 0, lim[np.maximum(idx - 1, 0)], -np.inf)
    hi = lim[idx]
    # value within its bucket (relative slack for float32 log rounding at a limit)
    assert np.all(fin <= hi * (1 + 1e-5) + 1e-30 * (hi == 0))
    assert np.all(fin >= lo * (1 + 1e-5) - 1e-30)


def test_nonfinite_watch_records_first_bad_step():
    w = S.NonfiniteWatch(torch.device("cpu"))
    w.reset(10)
    for v in (1.0, 2.0, float("nan"), 3.0, float("inf")):
        w.update(torch.tensor(v))
    assert w.first_bad_step() == 12


def test_trainer_detects_divergence_without_sync():
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.trainer import LRSchedule, Trainer
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=1, cell="gru")
    tr = Trainer(m, LRSchedule(1e-4, 100, 0.9))
    b = to_device(FixedShapeBatches(2, max_frames=200, seed=0, pool=1).next(), torch.device("cpu"))
    tr.step(b)
    assert tr.first_nonfinite_step() is None
    with torch.no_grad():
        m.fc_weight.data.fill_(float("nan"))
    tr.step(b)
    assert tr.first_nonfinite_step() == 1


def _train(args, env=None, timeout=300):
    e = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    e.update(env or {})
    cmd = [sys.executable, "-m", "deepspeech_amd.train", "--dummy", "True", "--batch_size", "2",
           "--num_hidden", "16", "--num_rnn_layers", "1", "--num_filters", "4", "--device", "cpu",
           "--log_every", "1000"] + args
    return subprocess.run(cmd, env=e, cwd=ROOT, capture_output=True, text=True, timeout=timeout)


def test_summaries_histograms_and_sparsity(tmp_path):
    d = str(tmp_path / "run")
    r = _train(["--train_dir", d, "--max_steps", "3", "--summary_every", "2", "--summaries_on_dummy", "True",
                "--cell", "gru"])
    assert r.returncode == 0, r.stdout + r.stderr
    ev = glob.glob(os.path.join(d, "events.out.tfevents.*"))
    assert len(ev) == 1
    tags = {t for _, t, _ in read_histograms(ev[0])}
    for a in ("conv1", "conv2", "rnn", "softmax_linear"):
        assert a + "/activations" in tags, tags
    assert "softmax_linear/weights/gradients" in tags and "conv1/weights" in tags
    assert any(t.startswith("rnn/brnn-0/") and t.endswith("/gradients") for t in tags)
    scalars = {t for _, t, _ in read_events(ev[0])}
    assert {"conv1/sparsity", "rnn/sparsity", "learning_rate", "ctc_loss"} <= scalars
    steps = {s for s, _, _ in read_histograms(ev[0])}
    assert steps == {0, 2}
    h = [h for _, t, h in read_histograms(ev[0]) if t == "conv1/activations"][0]
    assert sum(h["counts"]) == h["num"] and h["min"] >= 0.0 and h["max"] <= 20.0   # clipped ReLU


def test_resume_auto_continues_instead_of_wiping(tmp_path):
    from deepspeech_amd.utils import checkpoint as CK
    d = str(tmp_path / "run")
    r = _train(["--train_dir", d, "--max_steps", "4", "--checkpoint_every", "2"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert CK.latest_checkpoint(d).endswith("model.ckpt-3")
    r = _train(["--train_dir", d, "--max_steps", "6", "--checkpoint_every", "2", "--resume", "auto"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "has checkpoint" in r.stdout
    assert CK.latest_checkpoint(d).endswith("model.ckpt-5")
    # metrics rows are written at log / summary steps and the last step (checkpoint steps no
    # longer synchronise the host): the first run's last row is step 3, the second run appends
    # to the same file (not wiped) and its rows start after it
    rows = [json.loads(l) for l in open(os.path.join(d, "metrics.jsonl"))]
    steps = [r["step"] for r in rows if "event" not in r]        # checkpoint events are extra rows
    assert any(r.get("event") == "checkpoint_summary" and r["checkpoints_written"] >= 1 for r in rows)
    assert steps[0] == 3 and steps[-1] == 5 and sorted(steps) == steps and steps.count(3) == 1


def test_torchrun_restart_resumes_after_rank_kill(tmp_path):
    """Rank 1 dies at step 5 of the first attempt; torchrun --max-restarts=1 relaunches both
    ranks, which resume from train_dir's latest checkpoint (step 4) and finish. Each
    attempt builds its process group under its own store prefix (parallel/dist.py): without
    it a relaunched rank could dial a peer address left by the killed attempt."""
    from deepspeech_amd.utils import checkpoint as CK
    d = str(tmp_path / "tr")
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--max-restarts=1",
           "--rdzv-backend", "c10d", "--rdzv-endpoint", "127.0.0.1:%d" % _free_port(), "-m",
           "deepspeech_amd.train",
           "--dummy", "True", "--batch_size", "2", "--num_hidden", "16", "--num_rnn_layers", "1",
           "--num_filters", "4", "--device", "cpu", "--max_steps", "9", "--train_dir", d, "--log_every", "1000",
           "--checkpoint_every", "2", "--fault_inject_step", "5", "--fault_inject_rank", "1"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "fault injection at step 5 on rank 1" in out
    assert "has checkpoint" in out
    assert CK.latest_checkpoint(d).endswith("model.ckpt-8")
