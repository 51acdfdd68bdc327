"""Flag parity with the reference CLI, checkpoint layout / round trip, resume."""
import json
import os

import pytest
import torch

from deepspeech_amd import config as C
from deepspeech_amd.models import DeepSpeech2
from deepspeech_amd.trainer import LRSchedule, Trainer
from deepspeech_amd.utils import checkpoint as CK
from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device


REF_TRAIN_DEFAULTS = {
    # src/deepSpeech_train.py:40-103
    "train_dir": "../models/librispeech/train", "data_dir": "", "max_steps": 20000, "batch_size": 32,
    "temporal_stride": 1, "shuffle": True, "use_fp16": False, "keep_prob": 0.5, "num_hidden": 1024,
    "num_rnn_layers": 2, "checkpoint": None, "rnn_type": "bidirectional", "initial_lr": 1e-5,
    "num_filters": 32, "moving_avg_decay": 0.9999, "num_epochs_per_decay": 5, "lr_decay_factor": 0.9,
    "intra_op": 44, "inter_op": 1, "engine": "tf", "debug": False, "nchw": True, "dummy": False,
}


def test_train_flag_defaults_match_reference():
    a = C.parse_train_args([])
    for k, v in REF_TRAIN_DEFAULTS.items():
        assert getattr(a, k) == v, k


def test_reference_headline_command_line_parses():
    # src/train.sh:42
    a = C.parse_train_args("--batch_size 32 --no-shuffle --max_steps 40000 --num_rnn_layers 7 "
                           "--num_hidden 1760 --num_filters 32 --initial_lr 1e-4 --temporal_stride 4 "
                           "--train_dir x --data_dir y --debug False --nchw True --engine mkl --dummy True".split())
    assert a.shuffle is False and a.num_rnn_layers == 7 and a.num_hidden == 1760 and a.dummy is True


def test_eval_flag_defaults(tmp_path):
    json.dump({"num_hidden": 64, "num_rnn_layers": 3, "rnn_type": "bidirectional", "num_filters": 8,
               "use_fp16": False, "moving_avg_decay": 0.99}, open(tmp_path / "deepSpeech_parameters.json", "w"))
    a = C.parse_eval_args(["--checkpoint_dir", str(tmp_path)])
    assert a.eval_data == "val" and a.batch_size == 1 and a.eval_interval_secs == 300
    assert a.num_hidden == 64 and a.num_rnn_layers == 3 and a.moving_avg_decay == 0.99


def test_engine_aliases():
    cpu, gpu = torch.device("cpu"), torch.device("cuda")
    for e in ("tf", "mkl", "mkldnn_rnn", "cudnn_rnn"):
        assert C.resolve_engine(e, cpu) == "ref"
        assert C.resolve_engine(e, gpu) == "hip"
    with pytest.raises(ValueError):
        C.resolve_engine("hip", cpu)


def test_resume_reads_architecture_from_json(tmp_path):
    a = C.parse_train_args(["--num_hidden", "48", "--cell", "gru", "--train_dir", str(tmp_path)])
    C.dump_param_json(a, str(tmp_path))
    b = C.parse_train_args(["--checkpoint", str(tmp_path), "--num_hidden", "999"])
    assert b.num_hidden == 48 and b.cell == "gru"


def _trainer(cell="rnn_relu"):
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=2, cell=cell)
    return Trainer(m, LRSchedule(1e-3, 100, 0.9), moving_avg_decay=0.99)


def _batch():
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    return to_device(FixedShapeBatches(2, max_frames=120, seed=0, pool=1).next(), torch.device("cpu"))


@pytest.mark.parametrize("cell", ["rnn_relu", "gru"])
def test_tf_names_and_orientation(cell):
    t = _trainer(cell)
    names = CK.model_to_tf(t.model)
    assert "conv1/weights" in names and tuple(names["conv1/weights"].shape) == (20, 5, 1, 4)  # HWIO
    assert tuple(names["conv2/weights"].shape) == (10, 5, 4, 4)
    scope = "CustomRNNCell2" if cell == "rnn_relu" else "GRUCell"
    assert "rnn/brnn-0/bidirectional_rnn/fw/%s/W" % scope in names
    assert "rnn/brnn-1/bidirectional_rnn/bw/%s/U" % scope in names
    assert tuple(names["softmax_linear/weights"].shape) == (29, 16)


@pytest.mark.parametrize("fmt", ["tf", "torch"])
def test_checkpoint_roundtrip_and_state_file(tmp_path, fmt):
    t = _trainer()
    b = _batch()
    for _ in range(3):
        t.step(b)
    mgr = CK.CheckpointManager(str(tmp_path), max_to_keep=2, async_save=True, fmt=fmt)
    for s in (1, 2, 3):
        mgr.save(t, s)
    mgr.wait()
    files = sorted(os.listdir(tmp_path))
    if fmt == "tf":
        # TF Saver-V2 layout: <prefix>.index + <prefix>.data-00000-of-00001, old ones deleted
        assert "model.ckpt-3.index" in files and "model.ckpt-3.data-00000-of-00001" in files
        assert not any(f.startswith("model.ckpt-1") for f in files) and "checkpoint" in files
        from deepspeech_amd.utils import tf_bundle as TB
        raw = TB.read_bundle(str(tmp_path / "model.ckpt-3"))
        assert raw["global_step"].dtype == torch.int64 and int(raw["global_step"]) == 3
        assert abs(float(raw["beta1_power"]) - 0.9 ** 3) < 1e-7
        data = CK.load_checkpoint_file(str(tmp_path / "model.ckpt-3"))
    else:
        assert "model.ckpt-1" not in files and "model.ckpt-3" in files and "checkpoint" in files
        data = torch.load(str(tmp_path / "model.ckpt-3"), weights_only=True)
    assert CK.latest_checkpoint(str(tmp_path)).endswith("model.ckpt-3")
    assert "conv1/weights/ExponentialMovingAverage" in data and "conv1/weights/Adam" in data
    # restore into a fresh trainer: identical weights, slots and continued trajectory
    t2 = _trainer()
    CK.restore(t2, str(tmp_path))
    assert torch.allclose(t.arena.flat, t2.arena.flat)
    assert torch.allclose(t.opt.m, t2.opt.m) and torch.allclose(t.opt.ema, t2.opt.ema)
    assert t2.global_step == t.global_step == 3 and t2.opt.t == t.opt.t
    assert t2.lr == t.lr
    l1, l2 = float(t.step(b)), float(t2.step(b))
    assert abs(l1 - l2) < 1e-4
    # the continued trajectories agree after the update too (LR schedule, Adam t and the
    # EMA's num_updates all restored at the same step)
    assert t2.global_step == t.global_step
    assert torch.allclose(t.arena.flat, t2.arena.flat, atol=1e-6)
    assert torch.allclose(t.opt.ema, t2.opt.ema, atol=1e-6)


def test_eval_restores_ema_weights(tmp_path):
    t = _trainer()
    b = _batch()
    for _ in range(2):
        t.step(b)
    mgr = CK.CheckpointManager(str(tmp_path), async_save=False)
    mgr.save(t, 2)
    m = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=2)
    data = CK.load_checkpoint_file(str(tmp_path / "model.ckpt-2"))
    CK.load_model_from_tf(m, {k: v for k, v in data.items() if torch.is_tensor(v)}, use_ema=True)
    ema = t.arena.views(t.opt.ema)
    assert torch.allclose(m.fc_weight, ema["fc_weight"])


def test_debug_step_writes_profiles_and_tools_parse_them(tmp_path):
    """--debug (reference src/deepSpeech_train.py:358-380): chrome trace + params / flops /
    per-layer reports at step 20; tools/prof.py and tools/parse_log.py read them."""
    import subprocess
    import sys
    from deepspeech_amd import train as T
    d = tmp_path / "run"
    rc = T.main(["--train_dir", str(d), "--dummy", "True", "--max_steps", "22", "--batch_size", "2",
                 "--num_hidden", "32", "--num_rnn_layers", "2", "--debug", "True", "--device", "cpu",
                 "--checkpoint_every", "100", "--summary_every", "100", "--engine", "ref"])
    assert rc == 0
    for f in ("profiling.json", "params.log", "flops.log", "profile_layers.txt", "profile_ops.txt"):
        assert (d / f).exists(), f
    layers = (d / "profile_layers.txt").read_text()
    assert "rnn_forward_cell_0" in layers and "conv1_forward" in layers, layers
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "prof.py"), "-i", str(d / "profiling.json"),
                        "-o", str(tmp_path / "Output")], capture_output=True, text=True)
    assert r.returncode == 0 and "rnn_forward_cell_1" in r.stdout, r.stderr
    assert (tmp_path / "Output" / "layers_exeTime.csv").exists()
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "parse_log.py"), "--train_dir", str(d)],
                       capture_output=True, text=True)
    assert r.returncode == 0 and (d / "prf1.txt").exists() and "rnn_cell_0" in (d / "prf1.txt").read_text()


def test_launch_scripts_train_then_test(tmp_path):
    """scripts/train.sh and scripts/test.sh (reference src/train.sh, src/test.sh) end to end
    on CPU with synthetic data; the config guard rejects unknown engines."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, dummy="True", engine="ref", layers="1", hidden="32", cell="gru",
               train_dir=str(tmp_path / "train"),
               extra_args="--max_steps 3 --batch_size 2 --device cpu --checkpoint_every 1")
    r = subprocess.run(["bash", os.path.join(root, "scripts", "train.sh")], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert (tmp_path / "train" / "deepSpeech_parameters.json").exists()
    env2 = dict(os.environ, engine="ref", checkpoint_dir=str(tmp_path / "train"),
                extra_args="--dummy True --num_examples 2 --batch_size 2 --device cpu --eval_dir %s"
                           % (tmp_path / "eval"))
    r = subprocess.run(["bash", os.path.join(root, "scripts", "test.sh")], env=env2, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "char_err_rate" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
    bad = dict(env, engine="cuda")
    r = subprocess.run(["bash", os.path.join(root, "scripts", "train.sh")], env=bad, capture_output=True, text=True)
    assert r.returncode != 0 and "unsupported" in r.stdout


def test_setenvs_platforms(monkeypatch):
    from deepspeech_amd.utils import setenvs as S
    monkeypatch.delenv("HIP_FORCE_DEV_KERNARG", raising=False)
    got = S.setenvs(["x", "--platform", "mi355x"])
    assert os.environ["HIP_FORCE_DEV_KERNARG"] == "1" and "HIP_FORCE_DEV_KERNARG" in got
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    S.setenvs([], platform="knl")
    assert os.environ["OMP_NUM_THREADS"] == "3"          # existing values win
    with pytest.raises(ValueError):
        S.setenvs([], platform="pentium")


@pytest.mark.parametrize("seq_bn", ["frozen", "batch"])
def test_mkldnn_blob_layout_roundtrip(tmp_path, seq_bn):
    """engine=mkldnn_rnn checkpoints: one rnn_weights blob per layer/direction
    (src/mkldnn_rnn_op.py:37), W | R | b_W | b_R order; weights, Adam and EMA slots round-trip,
    and learned sequence-BN statistics (--seq_bn batch) are kept beside the blob."""
    from deepspeech_amd.utils import mkldnn_blob as MB
    from deepspeech_amd.trainer import Trainer, LRSchedule
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=2, cell="rnn_relu", seq_bn=seq_bn)
    m.param_layout = "mkldnn"
    tr = Trainer(m, LRSchedule(1e-4, 100, 0.9))
    b = to_device(FixedShapeBatches(2, max_frames=200, seed=0, pool=1).next(), torch.device("cpu"))
    tr.step(b)
    mgr = CK.CheckpointManager(str(tmp_path), async_save=False)
    path = mgr.save(tr, 0)
    data = CK.load_checkpoint_file(path)
    key = "rnn/brnn-1/bidirectional_rnn/bw/MkldnnRNNCell/rnn_weights"
    assert key in data and data[key].numel() == MB.params_size(16, 16)
    assert key + "/Adam" in data and key + "/ExponentialMovingAverage" in data
    assert not any("CustomRNNCell2" in k for k in data)
    assert "rnn/brnn-0/bidirectional_rnn/fw/MkldnnRNNCell/sbn/moving_mean" in data
    blob = data["rnn/brnn-0/bidirectional_rnn/fw/MkldnnRNNCell/rnn_weights"]
    W = m.rnn[0].fw.W.detach()
    assert torch.equal(blob[: W.numel()], W.reshape(-1))
    assert torch.equal(blob[-16:], torch.zeros(16))          # b_R exported as zeros
    if seq_bn == "batch":
        assert not torch.equal(m.rnn[0].fw.sbn_mean, torch.zeros(16))     # learned statistics
    m2 = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=2, cell="rnn_relu", seq_bn=seq_bn)
    tr2 = Trainer(m2, LRSchedule(1e-4, 100, 0.9))
    CK.restore(tr2, str(tmp_path))
    for (n, p), (_, q) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.equal(p, q), n
    assert torch.equal(tr.opt.m, tr2.opt.m) and torch.equal(tr.opt.ema, tr2.opt.ema)
    for i in range(2):
        for d in ("fw", "bw"):
            a, c = getattr(m.rnn[i], d), getattr(m2.rnn[i], d)
            assert torch.equal(a.sbn_mean, c.sbn_mean) and torch.equal(a.sbn_var, c.sbn_var)
    # a recurrent bias split across b_W / b_R imports as their sum
    W3, U3, b3 = MB.unpack(MB.pack(W, W[:, :16], torch.ones(16), torch.full((16,), 2.0)), 16, W.shape[1])
    assert torch.equal(b3, torch.full((16,), 3.0))


def test_setenvs_hw_queue_floor(monkeypatch):
    """GPU_MAX_HW_QUEUES is raised to at least 8 (a DP step has > 4 streams), never lowered."""
    from deepspeech_amd.utils import setenvs as S
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    S.setenvs([], platform="mi355x")
    assert os.environ["GPU_MAX_HW_QUEUES"] == "8"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "16")
    S.setenvs([], platform="mi355x")
    assert os.environ["GPU_MAX_HW_QUEUES"] == "16"
    # an explicit A/B arm keeps its exported value
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    monkeypatch.setenv("DS2_KEEP_HW_QUEUES", "1")
    S.setenvs([], platform="mi355x")
    assert os.environ["GPU_MAX_HW_QUEUES"] == "4"
