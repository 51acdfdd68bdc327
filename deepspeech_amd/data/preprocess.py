"""Offline LibriSpeech preprocessing (reference: src/preprocess_LibriSpeech.py).

  python -m deepspeech_amd.data.preprocess --audio_path ../data/LibriSpeech/audio \
         --out_dir ../data/LibriSpeech/processed [--features mfcc|spectrogram] [--tfrecords]

For every partition directory under ``audio_path`` (train-clean-100, dev-clean, ...):
read ``*.trans.txt`` transcripts, decode audio, compute features, map characters with the
28-symbol alphabet, sort utterances by frame count (SortaGrad) and write
  * a store (``<out>/<partition>.feats`` + ``.index.npz``) for the native mmap loader, and
  * optionally reference-compatible TFRecords: train split into ``train_<len//100>``
    bins with sparse bins (< 20 utts) dropped, dev/test as one sorted file
    (src/preprocess_LibriSpeech.py:143-176).
Audio decoding: ``.wav`` via scipy, ``.npy`` arrays; ``.flac`` needs the optional
``soundfile`` module (not installed in this image) and is reported clearly if missing.
"""
from __future__ import annotations

import argparse
import glob
import os
from typing import Dict, List, Tuple

import numpy as np

from .. import ALPHABET
from .featurizer import compute_features
from .store import StoreWriter

CHAR_TO_IX = {ch: i for i, ch in enumerate(ALPHABET)}


def encode_transcript(text: str) -> List[int]:
    return [CHAR_TO_IX[c] for c in text.upper() if c in CHAR_TO_IX]


def read_audio(path: str) -> Tuple[np.ndarray, int]:
    ext = os.path.splitext(path)[1].lower()
    if ext == ".wav":
        from scipy.io import wavfile
        sr, data = wavfile.read(path)
        data = data.astype(np.float64)
        if data.ndim > 1:
            data = data.mean(1)
        return data, int(sr)
    if ext == ".npy":
        return np.load(path, allow_pickle=False).astype(np.float64), 16000
    if ext == ".flac":
        try:
            import soundfile as sf  # type: ignore
        except ImportError:
            raise RuntimeError("decoding .flac needs the 'soundfile' package; convert to .wav first")
        data, sr = sf.read(path)
        return np.asarray(data, np.float64), int(sr)
    raise ValueError("unsupported audio file %s" % path)


def scan_partition(part_dir: str) -> List[Tuple[str, str]]:
    """[(audio_path, transcript)] from LibriSpeech ``<spk>/<chapter>/*.trans.txt`` files."""
    items = []
    for tf in sorted(glob.glob(os.path.join(part_dir, "**", "*.txt"), recursive=True)):
        d = os.path.dirname(tf)
        with open(tf) as f:
            for line in f:
                parts = line.strip().split(" ", 1)
                if len(parts) != 2:
                    continue
                uid, text = parts
                for ext in (".flac", ".wav", ".npy"):
                    p = os.path.join(d, uid + ext)
                    if os.path.exists(p):
                        items.append((p, text))
                        break
    return items


def process_partition(part_dir: str, out_prefix: str, features: str = "mfcc",
                      tfrecord_dir: str = "", is_train: bool = False, min_bin: int = 20) -> Dict[str, int]:
    utts = []
    for path, text in scan_partition(part_dir):
        audio, sr = read_audio(path)
        feats = compute_features(audio, sr, features)
        utts.append((feats, encode_transcript(text), text))
    utts.sort(key=lambda u: u[0].shape[0])                 # SortaGrad order
    w = StoreWriter(out_prefix, utts[0][0].shape[1] if utts else 161)
    for feats, lab, text in utts:
        w.add(feats, lab, text)
    w.close()
    if tfrecord_dir:
        from ..runtime import native
        N = native.load()
        name = os.path.basename(out_prefix)
        os.makedirs(os.path.join(tfrecord_dir, name), exist_ok=True)
        if is_train:
            bins: Dict[int, list] = {}
            for feats, lab, _ in utts:
                bins.setdefault(feats.shape[0] // 100, []).append(
                    N.make_sequence_example(feats.shape[0], feats, np.asarray(lab, np.int64), "feats"))
            for k, recs in bins.items():
                if len(recs) >= min_bin:
                    N.write_records(os.path.join(tfrecord_dir, name, "train_%d.tfrecords" % k), recs)
        else:
            recs = [N.make_sequence_example(f.shape[0], f, np.asarray(l, np.int64), "feats") for f, l, _ in utts]
            N.write_records(os.path.join(tfrecord_dir, name, name + ".tfrecords"), recs)
    return {"utterances": len(utts), "frames": int(sum(u[0].shape[0] for u in utts))}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--audio_path", default="../data/LibriSpeech/audio")
    ap.add_argument("--out_dir", default="../data/LibriSpeech/processed")
    ap.add_argument("--features", default="mfcc", choices=["mfcc", "spectrogram"])
    ap.add_argument("--tfrecords", action="store_true")
    a = ap.parse_args(argv)
    for part in sorted(glob.glob(os.path.join(a.audio_path, "*"))):
        if not os.path.isdir(part):
            continue
        name = os.path.basename(part)
        stats = process_partition(part, os.path.join(a.out_dir, name), a.features,
                                  a.out_dir if a.tfrecords else "", is_train=name.startswith("train"))
        print(name, stats)


if __name__ == "__main__":
    main()
