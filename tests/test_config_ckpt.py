"""Flag parity with the reference CLI, checkpoint layout / round trip, resume."""
import json
import os

import pytest
import torch

from deepspeech_amd import config as C
from deepspeech_amd.models import DeepSpeech2
from deepspeech_amd.trainer import LRSchedule, Trainer
from deepspeech_amd.utils import checkpoint as CK


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


def test_checkpoint_roundtrip_and_state_file(tmp_path):
    t = _trainer()
    b = _batch()
    for _ in range(3):
        t.step(b)
    mgr = CK.CheckpointManager(str(tmp_path), max_to_keep=2, async_save=True)
    for s in (1, 2, 3):
        mgr.save(t, s)
    mgr.wait()
    files = sorted(os.listdir(tmp_path))
    assert "model.ckpt-1" not in files and "model.ckpt-3" in files and "checkpoint" in files
    assert CK.latest_checkpoint(str(tmp_path)).endswith("model.ckpt-3")
    data = torch.load(str(tmp_path / "model.ckpt-3"), weights_only=True)
    assert "conv1/weights/ExponentialMovingAverage" in data and "conv1/weights/Adam" in data
    # restore into a fresh trainer: identical weights, slots and continued trajectory
    t2 = _trainer()
    CK.restore(t2, str(tmp_path))
    assert torch.allclose(t.arena.flat, t2.arena.flat)
    assert torch.allclose(t.opt.m, t2.opt.m) and torch.allclose(t.opt.ema, t2.opt.ema)
    assert t2.global_step == 4 and t2.opt.t == t.opt.t
    l1, l2 = float(t.step(b)), float(t2.step(b))
    assert abs(l1 - l2) < 1e-4


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
