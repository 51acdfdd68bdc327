"""On-disk utterance store + datasets feeding the native batch loader.

Store layout (``<prefix>`` = e.g. ``processed/train-clean-100``):
  <prefix>.feats    float32 [total_frames, 161], utterances back to back (mmap'ed)
  <prefix>.index.npz offsets[int64], lengths[int32], labels[int32 flat],
                     label_offsets[int64], label_lens[int32], (optional) transcripts

It replaces the reference's per-length-bin TFRecord files (src/preprocess_LibriSpeech.py:
143-176, read back by src/deepSpeech_input.py) with one mmap-able file per partition; the
length bucketing happens at batch-planning time instead (runtime/loader.cpp). TFRecord
input/output stays available through :func:`tfrecords_to_store` / :func:`store_to_tfrecords`.
"""
from __future__ import annotations

import glob
import os
from dataclasses import dataclass
from typing import Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from .. import FREQ_BINS
from ..config import get_rnn_seqlen_py


class StoreWriter:
    def __init__(self, prefix: str, freq: int = FREQ_BINS):
        os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
        self.prefix = prefix
        self.freq = freq
        self._f = open(prefix + ".feats", "wb")
        self.offsets: List[int] = []
        self.lengths: List[int] = []
        self.labels: List[np.ndarray] = []
        self.transcripts: List[str] = []
        self._frames = 0

    def add(self, feats: np.ndarray, labels: Sequence[int], transcript: str = "") -> None:
        feats = np.ascontiguousarray(feats, dtype=np.float32)
        assert feats.ndim == 2 and feats.shape[1] == self.freq, feats.shape
        self._f.write(feats.tobytes())
        self.offsets.append(self._frames)
        self.lengths.append(feats.shape[0])
        self.labels.append(np.asarray(labels, dtype=np.int32))
        self.transcripts.append(transcript)
        self._frames += feats.shape[0]

    def close(self) -> str:
        self._f.close()
        lab_lens = np.array([len(l) for l in self.labels], np.int32)
        lab_off = np.concatenate([[0], np.cumsum(lab_lens)[:-1]]).astype(np.int64) if len(lab_lens) else np.zeros(0, np.int64)
        np.savez(self.prefix + ".index.npz",
                 offsets=np.array(self.offsets, np.int64), lengths=np.array(self.lengths, np.int32),
                 labels=np.concatenate(self.labels).astype(np.int32) if self.labels else np.zeros(0, np.int32),
                 label_offsets=lab_off, label_lens=lab_lens, freq=np.int32(self.freq),
                 transcripts=np.array(self.transcripts))
        return self.prefix


@dataclass
class StoreIndex:
    prefix: str
    offsets: np.ndarray
    lengths: np.ndarray
    labels: np.ndarray
    label_offsets: np.ndarray
    label_lens: np.ndarray
    freq: int

    @staticmethod
    def load(prefix: str) -> "StoreIndex":
        z = np.load(prefix + ".index.npz", allow_pickle=False)
        return StoreIndex(prefix, z["offsets"], z["lengths"], z["labels"], z["label_offsets"],
                          z["label_lens"], int(z["freq"]))

    def __len__(self) -> int:
        return int(len(self.lengths))

    def min_frames(self) -> np.ndarray:
        """Frames needed so the conv front-end leaves room for the label (README.md:63-65, Q15)."""
        need = []
        for L, o in zip(self.label_lens, self.label_offsets):
            lab = self.labels[o:o + L]
            rep = int(np.sum(lab[1:] == lab[:-1])) if L > 1 else 0
            t2 = L + rep
            # smallest T with get_rnn_seqlen(T) >= t2 (T2 = ceil((ceil((T-19)/2)-9)/2)) is 4*t2+34
            need.append(4 * t2 + 34)
        return np.array(need, np.int32)


class StoreBatches:
    """Bucketed SortaGrad batches from a store via the native threaded loader.

    Epoch e < sortagrad_epochs: ascending length order (reference --no-shuffle first
    epoch, README.md:93-94); later epochs: buckets and batch groups shuffled.
    Distributed: all ranks plan the same global order and rank r takes every world-th
    batch, so the `world` batches of one step come from the same length bucket."""

    def __init__(self, prefix: str, batch_size: int, rank: int = 0, world: int = 1,
                 max_frames: int = 1800, bucket: int = 100, sortagrad_epochs: int = 1,
                 shuffle: bool = True, seed: int = 0, num_threads: int = 4, prefetch: int = 8):
        from ..runtime import native
        self.N = native.load()
        self.index = StoreIndex.load(prefix)
        self.batch_size = batch_size
        self.rank, self.world = rank, world
        self.max_frames, self.bucket = max_frames, bucket
        self.sortagrad_epochs = sortagrad_epochs
        self.shuffle = shuffle
        self.seed = seed
        self.prefetch = prefetch
        ix = self.index
        self.loader = self.N.BatchLoader(prefix + ".feats", ix.freq, ix.offsets, ix.lengths, ix.labels,
                                         ix.label_offsets, ix.label_lens, num_threads, 1)
        self._min = ix.min_frames()
        self.epoch = 0
        self._queue: List[List[int]] = []
        self._submitted = 0

    def plan_epoch(self, epoch: int) -> List[List[int]]:
        sorted_ = epoch < self.sortagrad_epochs or not self.shuffle
        plan = self.N.plan_batches(self.index.lengths, self._min, self.batch_size, self.bucket,
                                   self.max_frames, sorted_, self.seed + epoch, self.world, True)
        return [b for i, b in enumerate(plan) if i % self.world == self.rank]

    def steps_per_epoch(self) -> int:
        return len(self.plan_epoch(0))

    def _fill(self) -> None:
        while self.loader.pending() < self.prefetch:
            if not self._queue:
                self._queue = self.plan_epoch(self.epoch)
                self.epoch += 1
                if not self._queue:
                    raise RuntimeError("no feasible batches in store %s" % self.index.prefix)
            self.loader.submit([self._queue.pop(0)])

    def next(self):
        from .synthetic import Batch
        self._fill()
        feats, seq, lab, ll = self.loader.next()
        self._fill()
        return Batch(feats=feats, seq_lens=seq, labels=lab, label_lens=ll)

    def close(self) -> None:
        self.loader.shutdown()


# ---------------------------------------------------------------- TFRecord interop
def tfrecords_to_store(files: Iterable[str], prefix: str) -> str:
    """Convert reference-format TFRecord SequenceExamples (src/deepSpeech_input.py:34-49)."""
    from ..runtime import native
    N = native.load()
    w = None
    for path in files:
        for rec in N.read_records(path, True):
            seq_len, labels, feats = N.parse_sequence_example(rec, "feats")
            if w is None:
                w = StoreWriter(prefix, feats.shape[1])
            w.add(feats, labels)
    if w is None:
        raise ValueError("no records found")
    return w.close()


def store_to_tfrecords(prefix: str, path: str, indices: Optional[Sequence[int]] = None) -> str:
    """Write utterances as reference-compatible SequenceExamples (one TFRecord file)."""
    from ..runtime import native
    N = native.load()
    ix = StoreIndex.load(prefix)
    mm = np.memmap(prefix + ".feats", dtype=np.float32, mode="r").reshape(-1, ix.freq)
    recs = []
    for i in (range(len(ix)) if indices is None else indices):
        o, L = int(ix.offsets[i]), int(ix.lengths[i])
        lab = ix.labels[ix.label_offsets[i]: ix.label_offsets[i] + ix.label_lens[i]].astype(np.int64)
        recs.append(N.make_sequence_example(L, np.asarray(mm[o:o + L]), lab, "feats"))
    N.write_records(path, recs)
    return path


def find_partition_files(data_dir: str, eval_data: str) -> List[str]:
    """Glob real file names (quirk Q10) for 'train' / 'val' / 'test' TFRecords."""
    pat = {"train": "train*/*.tfrecords", "val": "dev*/*.tfrecords", "test": "test*/*.tfrecords"}[eval_data]
    return sorted(glob.glob(os.path.join(data_dir, pat)))


def find_store(data_dir: str, eval_data: str) -> Optional[str]:
    pat = {"train": "train*", "val": "dev*", "test": "test*"}[eval_data]
    c = sorted(glob.glob(os.path.join(data_dir, pat + ".index.npz")))
    return c[0][: -len(".index.npz")] if c else None
