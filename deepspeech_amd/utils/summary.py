"""Training/eval summaries without TensorFlow or tensorboard installed.

Reference: tf.summary scalars/histograms written by a FileWriter every 50 steps
(src/deepSpeech_train.py:349-351, :401-416; helper_routines.py:26-28 activation
histograms + sparsity) and the eval 'char_err_rate' scalar (src/deepSpeech_test.py:182-185).

:class:`EventWriter` emits TensorBoard-readable ``events.out.tfevents.*`` files (TFRecord
framing with masked CRC32C + hand-encoded ``Event``/``Summary``/``HistogramProto``
protobufs). One writer per run (the reference re-created a FileWriter every 50 steps, Q12).
:class:`JsonlWriter` writes the same values as JSON lines for scripts.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time
from typing import Dict, Optional

import numpy as np

# ---------------------------------------------------------------- crc32c / framing
_CRC_TABLE = None


def _crc32c(data: bytes) -> int:
    global _CRC_TABLE
    try:
        from ..runtime import native
        return int(native.load().crc32c(data))
    except Exception:
        pass
    if _CRC_TABLE is None:
        tbl = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (0x82F63B78 ^ (c >> 1)) if (c & 1) else (c >> 1)
            tbl.append(c)
        _CRC_TABLE = tbl
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    c = _crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def frame_record(data: bytes) -> bytes:
    hdr = struct.pack("<Q", len(data))
    return hdr + struct.pack("<I", _masked_crc(hdr)) + data + struct.pack("<I", _masked_crc(data))


# ---------------------------------------------------------------- protobuf encoding
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint((field << 3) | wt)


def _bytes_field(field: int, b: bytes) -> bytes:
    return _key(field, 2) + _varint(len(b)) + b


def _double_field(field: int, v: float) -> bytes:
    return _key(field, 1) + struct.pack("<d", v)


def _float_field(field: int, v: float) -> bytes:
    return _key(field, 5) + struct.pack("<f", v)


def _int_field(field: int, v: int) -> bytes:
    return _key(field, 0) + _varint(v)


def _histogram(values: np.ndarray) -> bytes:
    v = np.asarray(values, dtype=np.float64).ravel()
    if v.size == 0:
        v = np.zeros(1)
    counts, edges = np.histogram(v, bins=30)
    h = (_double_field(1, float(v.min())) + _double_field(2, float(v.max())) +
         _double_field(3, float(v.size)) + _double_field(4, float(v.sum())) +
         _double_field(5, float((v * v).sum())))
    h += _bytes_field(6, struct.pack("<%dd" % len(edges[1:]), *edges[1:]))
    h += _bytes_field(7, struct.pack("<%dd" % len(counts), *counts.astype(np.float64)))
    return h


def _histogram_from_stats(st) -> bytes:
    """HistogramProto of a utils.stats.HistStats (TF default buckets; empty buckets are merged
    into their right neighbour, as TF's EncodeToProto does)."""
    from .stats import limits
    lim = limits()
    nz = np.nonzero(st.counts)[0]
    h = (_double_field(1, st.min) + _double_field(2, st.max) + _double_field(3, st.num) +
         _double_field(4, st.sum) + _double_field(5, st.sum_sq))
    if nz.size:
        h += _bytes_field(6, struct.pack("<%dd" % nz.size, *lim[nz].tolist()))
        h += _bytes_field(7, struct.pack("<%dd" % nz.size, *st.counts[nz].astype(np.float64).tolist()))
    return h


def _event(step: int, summary: Optional[bytes] = None, file_version: Optional[str] = None) -> bytes:
    e = _double_field(1, time.time()) + _int_field(2, step)
    if file_version is not None:
        e += _bytes_field(3, file_version.encode())
    if summary is not None:
        e += _bytes_field(5, summary)
    return e


class EventWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        fname = "events.out.tfevents.%d.%s" % (int(time.time()), socket.gethostname())
        self.path = os.path.join(logdir, fname)
        self._f = open(self.path, "ab")
        self._f.write(frame_record(_event(0, file_version="brain.Event:2")))
        self._f.flush()

    def scalars(self, step: int, values: Dict[str, float]) -> None:
        s = b"".join(_bytes_field(1, _bytes_field(1, k.encode()) + _float_field(2, float(v)))
                     for k, v in values.items())
        self._f.write(frame_record(_event(step, summary=s)))
        self._f.flush()

    def histogram(self, step: int, tag: str, values) -> None:
        s = _bytes_field(1, _bytes_field(1, tag.encode()) + _bytes_field(5, _histogram(values)))
        self._f.write(frame_record(_event(step, summary=s)))

    def histogram_stats(self, step: int, tag: str, st) -> None:
        """Histogram from precomputed (device-side) statistics: utils.stats.HistStats."""
        s = _bytes_field(1, _bytes_field(1, tag.encode()) + _bytes_field(5, _histogram_from_stats(st)))
        self._f.write(frame_record(_event(step, summary=s)))

    def flush(self) -> None:
        self._f.flush()

    def close(self) -> None:
        self._f.close()


class JsonlWriter:
    def __init__(self, path: str):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        self._f = open(path, "a")

    def write(self, step: int, **values) -> None:
        rec = {"step": step, "time": time.time()}
        rec.update(values)
        self._f.write(json.dumps(rec) + "\n")
        self._f.flush()

    def close(self) -> None:
        self._f.close()


def _parse(buf: bytes):
    """Minimal protobuf walker: [(field, wire_type, value)] (value = int / bytes)."""
    out, i = [], 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 1:
            v, i = buf[i:i + 8], i + 8
        elif wt == 5:
            v, i = buf[i:i + 4], i + 4
        elif wt == 2:
            n, i = _read_varint(buf, i)
            v, i = buf[i:i + n], i + n
        else:
            raise ValueError("wire type %d" % wt)
        out.append((f, wt, v))
    return out


def _read_varint(buf: bytes, i: int):
    v, shift = 0, 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            return v, i


def read_events(path: str):
    """Parse scalars back from an event file (used by tests): [(step, tag, value)]."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        rec = data[i + 12: i + 12 + n]
        i += 12 + n + 4
        fields = _parse(rec)
        step = next((v for f, wt, v in fields if f == 2 and wt == 0), 0)
        for f, wt, summ in fields:
            if f != 5:
                continue
            for vf, _, val in _parse(summ):
                if vf != 1:
                    continue
                vals = _parse(val)
                tag = next((v.decode() for ff, _, v in vals if ff == 1), "")
                for ff, wt2, v in vals:
                    if ff == 2 and wt2 == 5:
                        out.append((step, tag, struct.unpack("<f", v)[0]))
    return out


def read_histograms(path: str):
    """Parse histograms back from an event file (tests): [(step, tag, dict)] with min, max,
    num, sum, sum_sq, limits, counts."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        rec = data[i + 12: i + 12 + n]
        i += 12 + n + 4
        fields = _parse(rec)
        step = next((v for f, wt, v in fields if f == 2 and wt == 0), 0)
        for f, wt, summ in fields:
            if f != 5:
                continue
            for vf, _, val in _parse(summ):
                if vf != 1:
                    continue
                vals = _parse(val)
                tag = next((v.decode() for ff, _, v in vals if ff == 1), "")
                for ff, wt2, v in vals:
                    if ff == 5 and wt2 == 2:
                        h = {}
                        for hf, hwt, hv in _parse(v):
                            key = {1: "min", 2: "max", 3: "num", 4: "sum", 5: "sum_sq"}.get(hf)
                            if key:
                                h[key] = struct.unpack("<d", hv)[0]
                            elif hf in (6, 7):
                                arr = list(struct.unpack("<%dd" % (len(hv) // 8), hv))
                                h["limits" if hf == 6 else "counts"] = arr
                        out.append((step, tag, h))
    return out
