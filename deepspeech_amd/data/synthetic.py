"""Synthetic LibriSpeech-shaped batches (the reference's "dummy" mode).

Two generators:

* :class:`DummyBucketWalk` — behavioural twin of src/deepSpeech_dummy.py: a
  pre-generated Gaussian feature buffer, buckets served in ascending length order
  (SortaGrad-like, :54-87), one bucket = ``counts[i]*scale*batch`` utterances. Quirk Q6
  is fixed: labels are drawn from the 28 real characters (the reference appends the
  blank index 28 and its dense->sparse conversion drops label 0).
* :class:`FixedShapeBatches` — the benchmark feed: every batch is ``[N, T, 161]`` with
  per-utterance lengths inside one 100-frame bucket (like bucket_by_sequence_length,
  src/deepSpeech_input.py:53-60), label lengths at LibriSpeech's ~15 chars/s.

Both produce numpy batches generated off the timed path; :func:`to_device` moves one
to pinned host memory and then to the GPU asynchronously.
"""
from __future__ import annotations

import random
from dataclasses import dataclass
from typing import Dict, Iterator, List, Optional

import numpy as np
import torch

from .. import FREQ_BINS, NUM_CLASSES
from ..config import get_rnn_seqlen_py

# reference tables: src/deepSpeech_dummy.py:9-16
UTT_LENGTHS = [100, 200, 100, 400, 500, 600, 700, 800, 900, 1000, 1100, 1200, 1300, 1400, 1500]
COUNTS = [30, 3, 3, 3, 14, 13, 9, 8, 5, 4, 3, 2, 2, 2, 1]
LABEL_LENGTHS = [7, 17, 7, 48, 62, 78, 93, 107, 120, 134, 148, 163, 178, 193, 209]
SCALE_FACTOR = 10
EXTRA = 1000
CHARS_PER_SEC = 15.0   # LibriSpeech read speech ~ 14-16 characters / second


@dataclass
class Batch:
    feats: np.ndarray          # [N, T, F] float32
    seq_lens: np.ndarray       # [N] int32 (frames)
    labels: np.ndarray         # [N, S] int32 dense, padded with -1
    label_lens: np.ndarray     # [N] int32

    @property
    def audio_seconds(self) -> float:
        return float(self.seq_lens.sum()) / 100.0   # 10 ms frames

    def flat_labels(self) -> np.ndarray:
        return np.concatenate([self.labels[i, : self.label_lens[i]] for i in range(len(self.label_lens))])

    def validate(self) -> "Batch":
        """Reject lengths the CTC kernels cannot honour, on the host before upload: a label
        length past the padded label width (the kernels clamp it only as an out-of-bounds guard,
        which would train on a truncated transcript; the reference's ctc_loss rejects it,
        src/deepSpeech_NCHW.py:225) or a sequence length past the padded frame count."""
        if len(self.label_lens) and int(self.label_lens.max()) > self.labels.shape[1]:
            raise ValueError("label length %d exceeds the padded label width %d"
                             % (int(self.label_lens.max()), self.labels.shape[1]))
        if len(self.seq_lens) and int(self.seq_lens.max()) > self.feats.shape[1]:
            raise ValueError("sequence length %d exceeds the padded frame count %d"
                             % (int(self.seq_lens.max()), self.feats.shape[1]))
        if len(self.label_lens) and int(self.label_lens.min()) < 0:
            raise ValueError("negative label length")
        return self


def random_labels(rng: np.random.Generator, n: int, length: int) -> np.ndarray:
    return rng.integers(0, NUM_CLASSES - 1, size=(n, length), dtype=np.int32)


def feasible_label_len(frames: int, want: int, labels: Optional[np.ndarray] = None) -> int:
    """Largest L <= want such that CTC has a path (README.md:63-65, quirk Q15): the
    label plus one blank between each repeated pair must fit in T2 frames. Without the
    concrete labels the worst case (all repeats: 2L-1 <= T2) is assumed."""
    t2 = get_rnn_seqlen_py(frames)
    if labels is None:
        return max(1, min(want, (t2 + 1) // 2))
    L = max(1, min(want, len(labels), t2))
    while L > 1 and L + int(np.sum(labels[1:L] == labels[:L - 1])) > t2:
        L -= 1
    return L


class DummyBucketWalk:
    """Replays the reference dummy epoch: buckets in ascending order of index."""

    def __init__(self, batch_size: int, seed: int = 0, scale_factor: int = SCALE_FACTOR):
        self.batch_size = batch_size
        self.rng = np.random.default_rng(seed)
        self.scale = scale_factor
        self.buffer = self.rng.standard_normal(
            (batch_size * (UTT_LENGTHS[-1] + EXTRA), FREQ_BINS)).astype(np.float32)
        self._reset()

    def _reset(self) -> None:
        self.remaining = [c * self.scale * self.batch_size for c in COUNTS]
        self.current = 0

    @property
    def utterances_per_epoch(self) -> int:
        return sum(COUNTS) * self.scale * self.batch_size

    def steps_per_epoch(self) -> int:
        return sum(-(-c * self.scale * self.batch_size // self.batch_size) for c in COUNTS)

    def next(self) -> Batch:
        if self.current >= len(self.remaining):
            self._reset()
        B = self.batch_size
        i = self.current
        if self.remaining[i] > B:
            n = B
            self.remaining[i] -= B
        else:
            n = self.remaining[i]
            self.remaining[i] = 0
            self.current += 1
        return self.batch_for(i, n)

    def batch_for(self, i: int, n: Optional[int] = None) -> Batch:
        """One batch of bucket i (n utterances, default the batch size), as next() makes it."""
        n = self.batch_size if n is None else n
        B = self.batch_size
        T = UTT_LENGTHS[i]
        start = int(self.rng.integers(0, EXTRA + B * (UTT_LENGTHS[-1] - T)))
        feats = self.buffer[start: start + T * n].reshape(n, T, FREQ_BINS)
        label = random_labels(self.rng, 1, LABEL_LENGTHS[i])
        L = feasible_label_len(T, LABEL_LENGTHS[i], label[0])
        label = label[:, :L]
        labels = np.repeat(label, n, axis=0)     # reference replicates one label per batch
        return Batch(feats=np.ascontiguousarray(feats), seq_lens=np.full(n, T, np.int32),
                     labels=labels, label_lens=np.full(n, L, np.int32))

    def __iter__(self) -> Iterator[Batch]:
        while True:
            yield self.next()


class FixedShapeBatches:
    """Benchmark feed: [N, T, 161] batches, lengths in (T - bucket, T]."""

    def __init__(self, batch_size: int, max_frames: int = 1000, bucket: int = 100,
                 seed: int = 0, pool: int = 4, chars_per_sec: float = CHARS_PER_SEC,
                 variable_lengths: bool = True):
        self.batch_size = batch_size
        self.T = max_frames
        self.rng = np.random.default_rng(seed)
        self.batches: List[Batch] = []
        for _ in range(pool):
            feats = self.rng.standard_normal((batch_size, max_frames, FREQ_BINS)).astype(np.float32)
            if variable_lengths:
                lens = self.rng.integers(max(21 + 18, max_frames - bucket + 1), max_frames + 1,
                                         size=batch_size).astype(np.int32)
                lens[0] = max_frames          # the batch is padded to its longest utterance
            else:
                lens = np.full(batch_size, max_frames, np.int32)
            want = [max(1, int(round(chars_per_sec * l / 100.0))) for l in lens]
            rows = [self.rng.integers(0, NUM_CLASSES - 1, size=w).astype(np.int32) for w in want]
            L = np.array([feasible_label_len(int(l), w, r) for l, w, r in zip(lens, want, rows)], np.int32)
            labels = np.full((batch_size, int(L.max())), -1, np.int32)
            for b in range(batch_size):
                labels[b, : L[b]] = rows[b][: L[b]]
                feats[b, lens[b]:] = 0.0
            self.batches.append(Batch(feats, lens, labels, L))
        self.i = 0

    def next(self) -> Batch:
        b = self.batches[self.i % len(self.batches)]
        self.i += 1
        return b

    def __iter__(self) -> Iterator[Batch]:
        while True:
            yield self.next()


def to_device(batch: Batch, device: torch.device, non_blocking: bool = True) -> Dict[str, torch.Tensor]:
    """Move a batch to ``device``: pinned staging + async H2D on the current stream."""
    pin = device.type == "cuda"

    def mv(a: np.ndarray) -> torch.Tensor:
        t = torch.from_numpy(np.ascontiguousarray(a))
        if pin:
            t = t.pin_memory()
        return t.to(device, non_blocking=non_blocking)

    flat = batch.validate().flat_labels().astype(np.int32)
    return {
        "feats": mv(batch.feats),
        "seq_lens": mv(batch.seq_lens.astype(np.int32)),
        "labels": mv(np.where(batch.labels < 0, 0, batch.labels).astype(np.int32)),
        "label_lens": mv(batch.label_lens.astype(np.int32)),
        "flat_labels": mv(flat),
    }
