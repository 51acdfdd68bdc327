"""The MKL-DNN RNN cell's single parameter blob (engine=mkldnn_rnn / cudnn_rnn checkpoints).

Reference: src/mkldnn_rnn_op.py:16-45 — ``MkldnnRNNCell`` wraps
``mkldnn_rnn_ops.MkldnnRNNRelu(1 layer, H, input_size)`` whose weights are ONE flat
variable ``rnn_weights [params_size]`` (initialised to 1/params_size, :37), created per
layer and direction under ``rnn/brnn-<i>/bidirectional_rnn/{fw,bw}/MkldnnRNNCell`` when the
NCHW graph runs with --engine mkldnn_rnn or cudnn_rnn (src/deepSpeech_NCHW.py:173-176).

Blob layout (the canonical order of a one-layer uni-directional RELU RNN, as the cuDNN /
MKL-DNN opaque-parameter converters of TF's contrib RNN ops define it): the input matrix
W [H, in] row-major, the recurrent matrix R [H, H] row-major, then the input bias b_W [H]
and the recurrent bias b_R [H]:  params_size = H*in + H*H + 2*H.

Mapping onto this framework's rnn_relu direction (W, U, b): W <-> W, U <-> R, b <-> b_W + b_R
(export writes b_R = 0). The MKL cell has no sequence-wise BN: models exported to or
imported from blobs are meant for ``seq_bn='none'``; with the default frozen SBN the input
projection carries its 1/sqrt(1+eps) factor, which export/import do not fold in.
"""
from __future__ import annotations

import re
from typing import Dict, Tuple

import torch

SLOT_SUFFIXES = ("", "/Adam", "/Adam_1", "/ExponentialMovingAverage")
_SCOPE = re.compile(r"^(rnn/brnn-\d+/bidirectional_rnn/(?:fw|bw))/CustomRNNCell2/W$")


def params_size(hidden: int, in_dim: int) -> int:
    return hidden * in_dim + hidden * hidden + 2 * hidden


def pack(W: torch.Tensor, U: torch.Tensor, b: torch.Tensor, b_r: torch.Tensor = None) -> torch.Tensor:
    H, D = W.shape
    if U.shape != (H, H) or b.shape != (H,):
        raise ValueError("rnn_relu direction shapes expected: W [H,in], U [H,H], b [H]")
    b_r = torch.zeros_like(b) if b_r is None else b_r
    return torch.cat([W.reshape(-1), U.reshape(-1), b.reshape(-1), b_r.reshape(-1)])


def unpack(blob: torch.Tensor, hidden: int, in_dim: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(W, U, b_W + b_R) from a blob."""
    H, D = hidden, in_dim
    if blob.numel() != params_size(H, D):
        raise ValueError("blob has %d values, expected %d for H=%d in=%d" % (blob.numel(), params_size(H, D), H, D))
    o = 0
    W = blob[o:o + H * D].view(H, D)
    o += H * D
    U = blob[o:o + H * H].view(H, H)
    o += H * H
    b = blob[o:o + H] + blob[o + H:o + 2 * H]
    return W.clone(), U.clone(), b.clone()


def to_mkldnn_layout(tensors: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """TF-named checkpoint dict (CustomRNNCell2 variables) -> the MkldnnRNNCell blob layout,
    for the weights and their Adam / EMA slots. SBN statistics are kept as they are."""
    out = dict(tensors)
    for key in list(tensors):
        m = _SCOPE.match(key)
        if not m:
            continue
        scope = m.group(1)
        cell = scope + "/CustomRNNCell2"
        for sfx in SLOT_SUFFIXES:
            if cell + "/W" + sfx not in out:
                continue
            W, U, B = out.pop(cell + "/W" + sfx), out.pop(cell + "/U" + sfx), out.pop(cell + "/B" + sfx)
            out[scope + "/MkldnnRNNCell/rnn_weights" + sfx] = pack(W, U, B)
        # the sequence-BN moving statistics are not blob parameters: they are stored next to
        # the blob (a --seq_bn batch run learns them; dropping them would reset a resumed or
        # evaluated model to mean 0 / variance 1)
        for k in ("/sbn/moving_mean", "/sbn/moving_variance"):
            if cell + k in out:
                out[scope + "/MkldnnRNNCell" + k] = out.pop(cell + k)
    return out


def from_mkldnn_layout(tensors: Dict[str, torch.Tensor], hidden: int, in_dims) -> Dict[str, torch.Tensor]:
    """Inverse of :func:`to_mkldnn_layout`. ``in_dims[i]`` is layer i's input width. SBN
    moving statistics stored beside the blob are kept; absent ones (a checkpoint written by
    the reference's MKL cell, which has no SBN) come back as mean 0 / variance 1."""
    out = dict(tensors)
    pat = re.compile(r"^(rnn/brnn-(\d+)/bidirectional_rnn/(?:fw|bw))/MkldnnRNNCell/rnn_weights(.*)$")
    for key in list(tensors):
        m = pat.match(key)
        if not m:
            continue
        scope, layer, sfx = m.group(1), int(m.group(2)), m.group(3)
        W, U, b = unpack(out.pop(key).float(), hidden, in_dims[layer])
        cell = scope + "/CustomRNNCell2"
        out[cell + "/W" + sfx], out[cell + "/U" + sfx], out[cell + "/B" + sfx] = W, U, b
        if sfx == "":
            for k, fill in (("/sbn/moving_mean", torch.zeros), ("/sbn/moving_variance", torch.ones)):
                v = out.pop(scope + "/MkldnnRNNCell" + k, None)
                out.setdefault(cell + k, v if v is not None else fill(hidden))
    return out


def is_mkldnn_checkpoint(tensors: Dict[str, torch.Tensor]) -> bool:
    return any("/MkldnnRNNCell/rnn_weights" in k for k in tensors)
