"""The reference's NHWC graph (--nchw False, src/deepSpeech.py): moments + zero-debiased EMA
conv BN (eps 1e-5, decay 0.5; src/custom_ops.py:163-181), per-direction deep RNN stacks
summed at the top (bidirectional_dynamic_rnn over two MultiRNNCells, src/deepSpeech.py:
165-185), channels-last flatten order at the checkpoint boundary."""
import copy
import os
import subprocess
import sys

import pytest
import torch

from deepspeech_amd.models import DeepSpeech2
from deepspeech_amd.models.deepspeech2 import NHWC_BN_EPS
from deepspeech_amd.ops import reference as R
from deepspeech_amd.utils import checkpoint as CK

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _batch(N=3, T=220, seed=0):
    g = torch.Generator().manual_seed(seed)
    feats = torch.randn(N, T, 161, generator=g)
    lens = torch.tensor([T, T - 40, T - 17][:N], dtype=torch.int32)
    return feats, lens


def test_moments_ema_bn_training_and_eval():
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=1, cell="gru", layout="nhwc")
    c1 = m.conv1
    assert c1.bn == "moments_ema" and c1.bn_eps == NHWC_BN_EPS
    x = torch.randn(2, 1, 60, 161)
    m.train()
    y = c1.forward_ref(x)
    z = torch.nn.functional.conv2d(x, c1.weight, c1.bias, stride=c1.stride)
    mean, var = z.mean((0, 2, 3)), z.var((0, 2, 3), unbiased=False)
    ref = R.clipped_relu((z - mean.view(1, -1, 1, 1)) * torch.rsqrt(var + 1e-5).view(1, -1, 1, 1))
    assert torch.allclose(y, ref, atol=1e-5)
    # one update: the debiased EMA equals the batch moments exactly (zero_debias=True)
    em, ev = c1.ema_moments()
    assert torch.allclose(em, mean, atol=1e-6) and torch.allclose(ev, var, atol=1e-5)
    c1.forward_ref(2 * x)
    em2, _ = c1.ema_moments()
    z2 = torch.nn.functional.conv2d(2 * x, c1.weight, c1.bias, stride=c1.stride)
    want = (0.5 * 0.5 * mean + 0.5 * z2.mean((0, 2, 3))) / (1 - 0.25)
    assert torch.allclose(em2, want, atol=1e-5)
    m.eval()
    ye = c1.forward_ref(x)
    em, ev = c1.ema_moments()
    refe = R.clipped_relu((z - em.view(1, -1, 1, 1)) * torch.rsqrt(ev + 1e-5).view(1, -1, 1, 1))
    assert torch.allclose(ye, refe, atol=1e-5)


def test_direction_stacks_match_manual_construction():
    torch.manual_seed(1)
    m = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=3, cell="rnn_relu", layout="nhwc")
    T, N = 30, 3
    x = torch.randn(T, N, m.rnn_in)
    lens = torch.tensor([30, 21, 9], dtype=torch.int32)
    out = m.recurrent(x, lens)
    xf = xb = x
    for layer in m.rnn:
        gf = layer.input_projection_ref(xf, layer.fw, lens)
        yf, _ = R.rnn_relu_scan(gf, layer.fw.U, lens)
        gb = layer.input_projection_ref(xb, layer.bw, lens)
        yb, _ = R.rnn_relu_scan(R.reverse_sequence(gb, lens), layer.bw.U, lens)
        xf, xb = yf, R.reverse_sequence(yb, lens)
    assert torch.allclose(out, xf + xb, atol=1e-5)
    # one layer: both topologies coincide
    m1 = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=1, cell="gru", layout="nhwc")
    m2 = copy.deepcopy(m1)
    m2.layout = "nchw"
    x1 = torch.randn(T, N, m1.rnn_in)
    assert torch.allclose(m1.recurrent(x1, lens), m2.recurrent(x1, lens), atol=1e-5)


def test_nhwc_checkpoint_names_and_column_order(tmp_path):
    torch.manual_seed(2)
    m = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=2, cell="rnn_relu", layout="nhwc")
    tf = CK.model_to_tf(m)
    assert "bidirectional_rnn/fw/multi_rnn_cell/cell_1/CustomRNNCell2/U" in tf
    assert "conv1/bn/gamma" in tf and "conv2/bn/moments/Squeeze_1/ExponentialMovingAverage/biased" in tf
    assert not any("bn2" in k or "brnn-" in k for k in tf)
    W = m.rnn[0].fw.W.detach()
    Wt = tf["bidirectional_rnn/fw/multi_rnn_cell/cell_0/CustomRNNCell2/W"]
    C, F2 = m.num_filters, m.rnn_in // m.num_filters
    c, f = 3, 70
    assert torch.equal(Wt[:, f * C + c], W[:, c * F2 + f])
    # layer 1 reads H-wide inputs: no permutation
    assert torch.equal(tf["bidirectional_rnn/bw/multi_rnn_cell/cell_1/CustomRNNCell2/W"], m.rnn[1].bw.W.detach())
    m2 = DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=2, cell="rnn_relu", layout="nhwc")
    CK.load_model_from_tf(m2, tf)
    for (n, p), (_, q) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.equal(p, q), n


def test_train_and_eval_cli_nhwc(tmp_path):
    d = str(tmp_path / "run")
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "deepspeech_amd.train", "--dummy", "True", "--batch_size", "2",
                        "--num_hidden", "16", "--num_rnn_layers", "2", "--num_filters", "4", "--device", "cpu",
                        "--nchw", "False", "--max_steps", "3", "--train_dir", d, "--log_every", "1000"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    data = CK.load_checkpoint_file(CK.latest_checkpoint(d))
    assert any(k.startswith("bidirectional_rnn/fw/multi_rnn_cell/cell_0/") for k in data)
    assert float(data["conv1/bn/moments/Squeeze/ExponentialMovingAverage/local_step"]) == 3.0
