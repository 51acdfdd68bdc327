"""Streaming inference (BASELINE.json north-star config 4: unidirectional GRU + CTC
beam-search decoder, real-time factor on one MI355X).

The reference only evaluates whole utterances (src/deepSpeech_test.py:112-136, greedy
CTC on a bidirectional model). A unidirectional model (``rnn_type='uni-dir'``, which the
reference's NHWC path supports: src/deepSpeech.py:173-183) can instead run on audio as it
arrives:

  * conv front-end: output frame t2 sees input frames [4*t2, 4*t2 + 38) (two strided VALID
    convs, kernel 20 / 10, stride 2 / 2 in time), so each chunk re-runs the convs on the
    38-frame-overlapping slice that produces exactly the NEW output frames; BatchNorm is in
    inference mode (running statistics), so frames are independent;
  * recurrent stack: every layer carries its final hidden state to the next chunk (the
    persistent kernels start from an initial state: ops/rnn.py:recurrent_layer_infer);
  * head + log-softmax per new frame; greedy decoding collapses across chunk boundaries
    incrementally, and the prefix beam search also advances chunk by chunk, so a transcript is
    ready when the audio ends: on the GPU the beams stay on the device (csrc/beam.hip, one
    launch per chunk, no log-prob copy), on the CPU the native runtime runs it (one host
    thread per stream group).

Batched streams: ``StreamingRecognizer`` takes [B, T_chunk, F] chunks of B concurrent
streams (equal chunk schedule, per-stream valid lengths), which is how a server batches.
"""
from __future__ import annotations

import os
import time
from typing import List, Optional

import numpy as np
import torch

from . import BLANK
from .models.deepspeech2 import DeepSpeech2, conv_out_len
from .ops import reference as R

RECEPTIVE = 38     # input frames seen by one output frame (see module docstring)
STRIDE = 4         # input frames per output frame


def frames_out(T: int) -> int:
    return conv_out_len(T)[1] if T >= RECEPTIVE else 0


class StreamingRecognizer:
    def __init__(self, model: DeepSpeech2, decoder: str = "greedy", beam_width: int = 16, batch: int = 1,
                 graphs: Optional[bool] = None):
        if model.bidirectional:
            raise ValueError("streaming needs a unidirectional model (rnn_type='uni-dir')")
        self.model = model.eval()
        self.decoder = decoder
        self.beam_width = beam_width
        self.B = batch
        self.dev = model.fc_weight.device
        # HIP graphs: a chunk's ~40 launches (conv front-end, 5 x (projection GEMM, sentinel
        # fill, persistent recurrence), head, log-softmax, argmax) are captured once per chunk
        # shape and replayed, so the per-chunk cost is GPU time, not host launch overhead.
        # The recurrent state lives in static buffers the graph reads and rewrites.
        if graphs is None:
            graphs = os.environ.get("DS2_INFER_GRAPHS", "1") != "0"
        self.use_graphs = bool(graphs) and self.dev.type == "cuda" and model.engine == "hip"
        self._graphs = {}
        self._h = None
        self.reset()

    def reset(self) -> None:
        self.buf = torch.zeros(self.B, 0, self.model.freq_bins, device=self.dev)
        self.buf_start = 0                  # absolute frame index of buf[:, 0]
        self.total = 0                      # frames received
        self.done = 0                       # output (post-conv) frames emitted
        self.states: List[Optional[torch.Tensor]] = [None] * len(self.model.rnn)
        if self._h is not None:
            for h in self._h:
                h.zero_()
        self.logprobs: List[torch.Tensor] = []
        self.beams = None
        self.gbeams = None
        if self.decoder == "beam":
            from .ops.decode import GpuBeamSearch
            if self.dev.type == "cuda" and self.beam_width <= GpuBeamSearch.MAX_BEAM:
                self.gbeams = GpuBeamSearch(self.B, self.beam_width, BLANK, -10.0, self.dev)
            else:
                from .runtime import native
                self.beams = native.load().BatchBeamSearch(self.B, self.beam_width, BLANK, -10.0)
        self.last_sym = [-1] * self.B
        self.greedy: List[List[int]] = [[] for _ in range(self.B)]
        self.compute_s = 0.0

    @torch.no_grad()
    def accept(self, chunk: torch.Tensor) -> List[List[int]]:
        """Feed [B, T_c, F] feature frames; returns the newly decoded (greedy) labels per stream."""
        t0 = time.perf_counter()
        m = self.model
        chunk = chunk.to(self.dev, torch.float32)
        self.buf = torch.cat([self.buf, chunk], 1)
        self.total += chunk.shape[1]
        t2_total = frames_out(self.total)
        new = t2_total - self.done
        out: List[List[int]] = [[] for _ in range(self.B)]
        if new <= 0:
            return out
        lo = STRIDE * self.done - self.buf_start
        hi = STRIDE * (t2_total - 1) + RECEPTIVE - self.buf_start
        feats = self.buf[:, lo:hi]
        if m.engine == "hip":
            feats = feats.to(m.compute_dtype)
        if not m.stack_fix:
            raise ValueError("streaming requires stack_fix=True")
        if self.use_graphs:
            lp, best_t = self._graph_chunk(feats.contiguous())
        else:
            x = m.frontend(feats)                              # [new, B, C*F2]
            assert x.shape[0] == new, (x.shape, new)
            lens = torch.full((self.B,), new, dtype=torch.int32, device=self.dev)
            for i, layer in enumerate(m.rnn):
                x, self.states[i] = self._layer(layer, x, lens, self.states[i])
            logits = m.head(x).float()
            lp = torch.log_softmax(logits, -1)                 # [new, B, K]
            best_t = lp.argmax(-1)
        assert lp.shape[0] == new, (lp.shape, new)
        self.logprobs.append(lp)
        best = best_t.cpu().numpy()                            # [new, B]
        if self.gbeams is not None:
            # prefix beam search advances chunk by chunk, beams resident on the device
            self.gbeams.feed(lp)
        elif self.beams is not None:
            # prefix beam search advances chunk by chunk (beams carried in the native
            # runtime, streams decoded on parallel host threads)
            self.beams.feed(lp.cpu().numpy(), np.full((self.B,), new, dtype=np.int32))
        for b in range(self.B):
            for t in range(best.shape[0]):
                s = int(best[t, b])
                if s != self.last_sym[b] and s != BLANK:
                    out[b].append(s)
                self.last_sym[b] = s
            self.greedy[b].extend(out[b])
        self.done = t2_total
        # keep only the input frames future outputs can still see
        keep_from = STRIDE * self.done
        if keep_from > self.buf_start:
            self.buf = self.buf[:, keep_from - self.buf_start:]
            self.buf_start = keep_from
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)
        self.compute_s += time.perf_counter() - t0
        if m.engine == "hip":
            from .ops import rnn as RNN
            RNN.check_errors()        # after the chunk's sync: one 4-byte read
        return out

    # ---- HIP-graph path -------------------------------------------------------------
    def _chunk_body(self, feats):
        """The whole GPU part of a chunk on static state buffers (capturable: no host sync)."""
        m = self.model
        x = m.frontend(feats)
        lens = torch.full((self.B,), x.shape[0], dtype=torch.int32, device=self.dev)
        for i, layer in enumerate(m.rnn):
            x, _ = self._layer(layer, x, lens, self._h[i], out=self._h[i])   # state carried in place
        lp = torch.log_softmax(m.head(x).float(), -1)
        return lp, lp.argmax(-1)

    def _graph_chunk(self, feats):
        if self._h is None:
            self._h = [torch.zeros(self.B, layer.hidden, device=self.dev, dtype=torch.float32)
                       for layer in self.model.rnn]
        key = tuple(feats.shape)
        g = self._graphs.get(key)
        if g is None:
            # first chunk of this shape: run it eagerly (real result, warms plans/handles),
            # then capture the same work into a graph for every later chunk of this shape
            lp, best = self._chunk_body(feats)
            static_in = feats.clone()
            saved = [h.clone() for h in self._h]              # capture records, never runs
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = self._chunk_body(static_in)
            for h, s in zip(self._h, saved):
                h.copy_(s)
            self._graphs[key] = (graph, static_in, out)
            return lp.clone(), best.clone()
        graph, static_in, out = g
        static_in.copy_(feats)
        graph.replay()
        return out[0].clone(), out[1].clone()

    def _layer(self, layer, x, lens, h0, out=None):
        """One uni-directional layer from state h0 [B, H]; returns (y, h_last [B, H]), h_last
        written into `out` when given (it may be h0 itself: the kernel has read h0 by then)."""
        m = self.model
        if m.engine == "hip":
            from .ops import rnn as RNN
            y, h = RNN.recurrent_layer_infer(layer, x, lens, None if h0 is None else h0.unsqueeze(0),
                                             h_out=None if out is None else out.unsqueeze(0))
            return y, h[0]
        gx = layer.input_projection_ref(x, layer.fw, lens)
        bh = layer.fw.b_h.to(x.dtype) if layer.fw.b_h is not None else None
        y, h = R.recurrent_scan(layer.cell, gx, layer.fw.U.to(x.dtype), bh, lens, h0)
        if out is not None:
            out.copy_(h)
            h = out
        return y, h

    @torch.no_grad()
    def finish(self) -> List[List[int]]:
        """Final transcript label ids per stream (beam search over the whole stream if the
        decoder is 'beam', otherwise the incremental greedy result)."""
        if self.gbeams is not None:
            return self.gbeams.best()
        if self.beams is None:
            return [list(g) for g in self.greedy]
        return self.beams.best()


def rtf(model: DeepSpeech2, seconds: float = 10.0, chunk_s: float = 1.0, batch: int = 1,
        decoder: str = "greedy", beam_width: int = 16, seed: int = 0):
    """Real-time factor of streaming synthetic audio: compute time / audio time (per stream;
    ``batch`` streams are processed together). Returns (rtf, transcripts)."""
    g = torch.Generator().manual_seed(seed)
    T = int(round(seconds * 100))
    feats = torch.randn(batch, T, model.freq_bins, generator=g)
    rec = StreamingRecognizer(model, decoder=decoder, beam_width=beam_width, batch=batch)
    step = max(1, int(round(chunk_s * 100)))
    for s in range(0, T, step):
        rec.accept(feats[:, s:s + step])
    res = rec.finish()
    return rec.compute_s / seconds, res
