"""Audio featurizer (offline preprocessing).

Reference: src/preprocess_LibriSpeech.py:24-42 — DC removal, peak normalisation, then
python_speech_features.mfcc(winlen=0.025, winstep=0.01, numcep=161, nfilt=322, nfft=512,
lowfreq=0, preemph=0.97, ceplifter=22, appendEnergy=True). python_speech_features is not
installed here, so this is an independent numpy implementation of the same pipeline
(rectangular window, power spectrum /nfft, triangular mel filterbank, log, orthonormal
DCT-II, sinusoidal lifter, c0 replaced by log frame energy). Quirk Q11: the reference's
"mfcc" has 161 cepstra from 322 filters; a linear spectrogram with 161 bins (nfft=320) is
offered as the DS2-paper alternative.
"""
from __future__ import annotations

import math

import numpy as np


def _frames(signal: np.ndarray, frame_len: int, frame_step: int) -> np.ndarray:
    n = len(signal)
    num = 1 if n <= frame_len else 1 + int(math.ceil((n - frame_len) / float(frame_step)))
    pad = (num - 1) * frame_step + frame_len
    sig = np.concatenate([signal, np.zeros(pad - n)])
    idx = np.arange(frame_len)[None, :] + frame_step * np.arange(num)[:, None]
    return sig[idx]


def _hz2mel(hz):
    return 2595.0 * np.log10(1.0 + hz / 700.0)


def _mel2hz(mel):
    return 700.0 * (10.0 ** (mel / 2595.0) - 1.0)


def mel_filterbank(nfilt: int, nfft: int, sample_rate: int, lowfreq: float = 0.0,
                   highfreq: float = None) -> np.ndarray:
    highfreq = highfreq or sample_rate / 2.0
    mels = np.linspace(_hz2mel(lowfreq), _hz2mel(highfreq), nfilt + 2)
    bins = np.floor((nfft + 1) * _mel2hz(mels) / sample_rate).astype(int)
    fb = np.zeros((nfilt, nfft // 2 + 1))
    for j in range(nfilt):
        for i in range(bins[j], bins[j + 1]):
            fb[j, i] = (i - bins[j]) / max(1, (bins[j + 1] - bins[j]))
        for i in range(bins[j + 1], bins[j + 2]):
            fb[j, i] = (bins[j + 2] - i) / max(1, (bins[j + 2] - bins[j + 1]))
    return fb


def _dct2_ortho(x: np.ndarray) -> np.ndarray:
    n = x.shape[-1]
    k = np.arange(n)
    basis = np.cos(np.pi * (2 * k[None, :] + 1) * k[:, None] / (2.0 * n))   # [n_out, n_in]
    out = x @ basis.T
    out[..., 0] *= math.sqrt(1.0 / (4 * n)) * 2
    out[..., 1:] *= math.sqrt(1.0 / (2 * n)) * 2
    return out


def _lifter(cep: np.ndarray, L: int) -> np.ndarray:
    if L <= 0:
        return cep
    n = np.arange(cep.shape[1])
    return cep * (1 + (L / 2.0) * np.sin(np.pi * n / L))


def mfcc(signal: np.ndarray, sample_rate: int, winlen: float = 0.025, winstep: float = 0.01,
         numcep: int = 161, nfilt: int = 322, nfft: int = 512, lowfreq: float = 0.0,
         highfreq: float = None, preemph: float = 0.97, ceplifter: int = 22,
         append_energy: bool = True) -> np.ndarray:
    sig = np.asarray(signal, dtype=np.float64)
    sig = np.append(sig[0], sig[1:] - preemph * sig[:-1])
    fr = _frames(sig, int(round(winlen * sample_rate)), int(round(winstep * sample_rate)))
    mag = np.abs(np.fft.rfft(fr, nfft))
    pspec = (mag ** 2) / nfft
    energy = np.sum(pspec, 1)
    energy = np.where(energy == 0, np.finfo(float).eps, energy)
    fb = mel_filterbank(nfilt, nfft, sample_rate, lowfreq, highfreq)
    feat = pspec @ fb.T
    feat = np.where(feat == 0, np.finfo(float).eps, feat)
    cep = _dct2_ortho(np.log(feat))[:, :numcep]
    cep = _lifter(cep, ceplifter)
    if append_energy:
        cep[:, 0] = np.log(energy)
    return cep.astype(np.float32)


def spectrogram(signal: np.ndarray, sample_rate: int, winlen: float = 0.02, winstep: float = 0.01,
                eps: float = 1e-14) -> np.ndarray:
    """Log linear spectrogram, Hamming window; 20 ms at 16 kHz -> nfft 320 -> 161 bins."""
    n = int(round(winlen * sample_rate))
    fr = _frames(np.asarray(signal, dtype=np.float64), n, int(round(winstep * sample_rate)))
    fr = fr * np.hamming(n)[None, :]
    p = np.abs(np.fft.rfft(fr, n)) ** 2
    return np.log(p + eps).astype(np.float32)


def compute_features(audio: np.ndarray, sample_rate: int, kind: str = "mfcc") -> np.ndarray:
    """DC removal + peak normalisation then features (src/preprocess_LibriSpeech.py:36-41)."""
    a = np.asarray(audio, dtype=np.float64)
    a = a - a.mean()
    peak = np.max(np.abs(a)) if a.size else 1.0
    a = a / (peak if peak > 0 else 1.0)
    if kind == "mfcc":
        return mfcc(a, sample_rate)
    if kind == "spectrogram":
        return spectrogram(a, sample_rate)
    raise ValueError(kind)
