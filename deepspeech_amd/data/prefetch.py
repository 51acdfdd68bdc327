"""Background host->device batch prefetcher (the reference's queue runners feeding the
graph, src/deepSpeech_input.py:53-60 + src/deepSpeech_train.py:491, the MI355X way).

A producer thread pulls host batches from any source with ``.next()`` (synthetic walk,
C++ store loader), copies them into a small ring of REUSED pinned host buffers (no per-batch
``pin_memory()`` allocation: ~30 MB per 15-s batch), issues the host->device copies on a
dedicated copy stream and records an event. ``next()`` hands out the device tensors with
the consumer's stream waiting on that event, so batch production and upload overlap the
previous steps' kernels; the host only blocks when the ring is empty.
"""
from __future__ import annotations

import queue
import threading
import time
import warnings
from typing import Dict, Optional

import numpy as np
import torch


class _Pinned:
    """One pinned staging slot, grown on demand (never shrinks)."""

    def __init__(self):
        self.bufs: Dict[str, torch.Tensor] = {}
        self.event: Optional[torch.cuda.Event] = None      # last H2D out of this slot

    def stage(self, name: str, a: np.ndarray) -> torch.Tensor:
        a = np.ascontiguousarray(a)
        t = torch.from_numpy(a)
        buf = self.bufs.get(name)
        if buf is None or buf.numel() < t.numel() or buf.dtype != t.dtype:
            buf = torch.empty(max(t.numel(), 1), dtype=t.dtype).pin_memory()
            self.bufs[name] = buf
        view = buf[: t.numel()].view(t.shape)
        view.copy_(t)
        return view


class DevicePrefetcher:
    def __init__(self, source, device: torch.device, depth: int = 2):
        if device.type != "cuda":
            raise ValueError("DevicePrefetcher needs a GPU device")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.source = source
        self.device = device
        self.depth = max(1, depth)
        self.copy_stream = torch.cuda.Stream(device=device)
        self.slots = [_Pinned() for _ in range(self.depth + 1)]
        self.q: "queue.Queue" = queue.Queue(maxsize=self.depth)
        self._stop = threading.Event()
        self._err: Optional[BaseException] = None
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()

    def _run(self) -> None:
        k = 0
        try:
            torch.cuda.set_device(self.device)
            while not self._stop.is_set():
                hb = self.source.next()
                slot = self.slots[k % len(self.slots)]
                k += 1
                if slot.event is not None:
                    slot.event.synchronize()         # previous upload out of this slot done
                flat = hb.validate().flat_labels().astype(np.int32)
                host = {
                    "feats": slot.stage("feats", hb.feats.astype(np.float32, copy=False)),
                    "seq_lens": slot.stage("seq_lens", hb.seq_lens.astype(np.int32)),
                    "labels": slot.stage("labels", np.where(hb.labels < 0, 0, hb.labels).astype(np.int32)),
                    "label_lens": slot.stage("label_lens", hb.label_lens.astype(np.int32)),
                    "flat_labels": slot.stage("flat_labels", flat),
                }
                with torch.cuda.stream(self.copy_stream):
                    dev = {n: t.to(self.device, non_blocking=True) for n, t in host.items()}
                    ev = torch.cuda.Event()
                    ev.record(self.copy_stream)
                slot.event = ev
                while not self._stop.is_set():
                    try:
                        self.q.put((hb, dev, ev), timeout=0.1)
                        break
                    except queue.Full:
                        continue
        except BaseException as e:      # surfaced by next()
            self._err = e
            self.q.put(None)

    def next(self):
        """(host batch, device tensors) — the current stream waits for the upload."""
        item = self.q.get()
        if item is None:
            raise RuntimeError("prefetch thread failed") from self._err
        hb, dev, ev = item
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        for t in dev.values():
            t.record_stream(cur)
        return hb, dev

    def close(self, timeout_s: float = 60.0) -> bool:
        """Stop the producer. Returns True once its thread has exited; False (with a
        warning) if it is still inside ``source.next()`` or an upload wait after
        ``timeout_s`` — the caller must then NOT tear the source down under it."""
        self._stop.set()
        deadline = time.monotonic() + timeout_s
        while self._thread.is_alive() and time.monotonic() < deadline:
            try:                      # unblock a producer waiting on a full queue
                while True:
                    self.q.get_nowait()
            except queue.Empty:
                pass
            self._thread.join(timeout=0.1)
        if self._thread.is_alive():
            warnings.warn("DevicePrefetcher: producer thread still running after %.0f s; "
                          "leaving its source open" % timeout_s)
            return False
        return True
