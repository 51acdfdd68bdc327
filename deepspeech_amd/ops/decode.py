"""CTC decoding entry points.

greedy: csrc/decode.hip on the GPU (argmax + merge repeats + drop blank + path score in one
        kernel per utterance; reference tf.nn.ctc_greedy_decoder, src/deepSpeech_test.py:212-215),
        plain PyTorch (ops/reference.py) on the CPU.
beam:   CTC prefix beam search: csrc/beam.hip on the GPU (beams resident on the device, one
        wave64 per utterance / stream, GpuBeamSearch), the native host runtime
        (runtime/decoder.cpp, one thread per utterance) on the CPU.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from .. import BLANK
from . import reference as R


def greedy_decode(logits: torch.Tensor, lens: torch.Tensor, blank: int = BLANK,
                  with_scores: bool = False):
    """logits [T, N, K] time-major (raw logits or log-probs) -> label lists (and the
    greedy-path log-probabilities when ``with_scores``)."""
    if logits.is_cuda:
        from . import _ext
        T, N, _ = logits.shape
        lg = logits if logits.dtype in (torch.float32, torch.bfloat16) else logits.float()
        lg = lg.contiguous()
        lens_d = lens.to(device=lg.device, dtype=torch.int32).contiguous()
        labels = torch.empty(N, T, device=lg.device, dtype=torch.int32)
        counts = torch.empty(N, device=lg.device, dtype=torch.int32)
        score = torch.empty(N, device=lg.device, dtype=torch.float32)
        _ext.ext().ctc_greedy(lg, lens_d, labels, counts, blank, score)
        counts_h = counts.cpu().tolist()
        lab_h = labels.cpu().numpy()
        out = [lab_h[n, :counts_h[n]].tolist() for n in range(N)]
        return (out, score.cpu()) if with_scores else out
    lp = torch.log_softmax(logits.float(), -1)
    out = R.greedy_decode(lp, lens, blank)
    if not with_scores:
        return out
    L = lens.cpu()
    sc = torch.stack([lp[: int(L[n]), n].max(-1).values.sum() for n in range(lp.shape[1])])
    return out, sc


def beam_decode(logits: torch.Tensor, lens: torch.Tensor, beam_width: int = 16, blank: int = BLANK,
                prune: float = -10.0) -> List[List[int]]:
    """logits [T, N, K] time-major -> the best prefix of each utterance's beam search."""
    if logits.is_cuda and beam_width <= GpuBeamSearch.MAX_BEAM:
        T, N, _ = logits.shape
        bs = GpuBeamSearch(N, beam_width, blank, prune, logits.device, frames_hint=T)
        bs.feed(torch.log_softmax(logits.float(), dim=-1), lens)
        return bs.best()
    from ..runtime import native
    lp = torch.log_softmax(logits.float(), dim=-1).cpu().numpy()
    return native.load().beam_search_batch(lp, lens.cpu().numpy().astype(np.int32), beam_width, blank, prune)


class GpuBeamSearch:
    """CTC prefix beam search of B streams with the beams resident on the device
    (csrc/beam.hip): :meth:`feed` advances every stream by a [T, B, K] block of log-probs in
    one launch on the current stream (no host synchronisation, so a streaming recogniser feeds
    each chunk straight from its log-softmax), :meth:`results` / :meth:`best` walk the trie on
    the device and read the prefixes back once. Same search as runtime/decoder.cpp
    PrefixBeamSearch (prune window, blank / repeat rules, merged prefixes)."""
    MAX_BEAM = 32

    def __init__(self, streams: int, beam: int, blank: int = BLANK, prune: float = -10.0,
                 device: torch.device = None, frames_hint: int = 256):
        if not 1 <= beam <= self.MAX_BEAM:
            raise ValueError("GpuBeamSearch: 1 <= beam <= %d" % self.MAX_BEAM)
        self.B, self.W, self.blank, self.prune = int(streams), int(beam), int(blank), float(prune)
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.cap = 1 + self.W * max(16, int(frames_hint))
        i32 = dict(device=self.dev, dtype=torch.int32)
        f32 = dict(device=self.dev, dtype=torch.float32)
        self.node = torch.empty(self.B, self.W, **i32)
        self.last = torch.empty(self.B, self.W, **i32)
        self.parent = torch.empty(self.B, self.W, **i32)
        self.pb = torch.empty(self.B, self.W, **f32)
        self.pnb = torch.empty(self.B, self.W, **f32)
        self.nbeam = torch.empty(self.B, **i32)
        self.nnodes = torch.empty(self.B, **i32)
        self.nodes = torch.zeros(self.B, self.cap, 2, **i32)
        self.err = torch.zeros(1, **i32)
        self.reset()

    def reset(self) -> None:
        """Every stream back to the empty prefix (log p = 0, ending in blank)."""
        self.node.zero_()
        self.last.fill_(-1)
        self.parent.fill_(-1)
        self.pb.fill_(float("-inf"))
        self.pb[:, 0] = 0.0
        self.pnb.fill_(float("-inf"))
        self.nbeam.fill_(1)
        self.nnodes.fill_(1)
        self.frames = 0          # frames fed so far (upper bound over streams): sizes the trie

    def _ensure(self, more: int) -> None:
        need = 1 + self.W * (self.frames + more)
        if need <= self.cap:
            return
        cap = max(need, 2 * self.cap)
        nodes = torch.zeros(self.B, cap, 2, device=self.dev, dtype=torch.int32)
        nodes[:, : self.cap] = self.nodes
        self.nodes, self.cap = nodes, cap

    def feed(self, lp: torch.Tensor, frames=None) -> None:
        """lp [T, B, K] log-probs on the device; frames: None (all T), an int, or a [B] tensor
        of per-stream frame counts (<= T)."""
        from . import _ext
        if lp.dim() != 3 or lp.shape[1] != self.B:
            raise ValueError("GpuBeamSearch.feed: lp must be [T, %d, K]" % self.B)
        T = int(lp.shape[0])
        if T == 0:
            return
        lp = lp.float().contiguous()
        fr = None
        if isinstance(frames, int):
            if frames < T:
                fr = torch.full((self.B,), frames, device=self.dev, dtype=torch.int32)
        elif frames is not None:
            fr = frames.to(device=self.dev, dtype=torch.int32).contiguous()
        self._ensure(T)
        _ext.ext().ctc_beam(lp, fr, self.blank, self.prune, self.node, self.last, self.parent, self.pb,
                            self.pnb, self.nbeam, self.nodes, self.nnodes, self.err)
        self.frames += T

    def results(self) -> List[List[Tuple[List[int], float]]]:
        """Per stream, the live hypotheses best first: (labels, log p). Synchronises."""
        from . import _ext
        L = max(1, self.frames)
        out = torch.empty(self.B, self.W, L, device=self.dev, dtype=torch.int32)
        out_len = torch.empty(self.B, self.W, device=self.dev, dtype=torch.int32)
        score = torch.empty(self.B, self.W, device=self.dev, dtype=torch.float32)
        _ext.ext().ctc_beam_backtrack(self.node, self.last, self.parent, self.pb, self.pnb, self.nbeam,
                                      self.nodes, self.nnodes, out, out_len, score)
        if int(self.err.item()) != 0:
            raise RuntimeError("GpuBeamSearch: trie node table overflow")
        o, n, s = out.cpu().numpy(), out_len.cpu().numpy(), score.cpu().numpy()
        return [[(o[b, h, : n[b, h]].tolist(), float(s[b, h])) for h in range(self.W) if n[b, h] >= 0]
                for b in range(self.B)]

    def best(self) -> List[List[int]]:
        return [r[0][0] if r else [] for r in self.results()]
