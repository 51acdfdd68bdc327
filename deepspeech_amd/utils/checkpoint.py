"""Checkpoint / resume with the reference's directory contract.

Reference (src/deepSpeech_train.py:354-356, :383-398, :471, :504-513):
  train_dir/deepSpeech_parameters.json      json.dump(vars(ARGS))
  train_dir/model.ckpt-<step>               saver.save(..., global_step=step), max_to_keep=100
  train_dir/checkpoint                      TF state file naming the latest checkpoint
Saved set: model variables, Adam slots, global_step, weight-EMA shadows (eval restores
them: src/deepSpeech_test.py:217-220), BN moving stats.

Here every entry is keyed by its TF variable name and stored in TF orientation (conv
kernels HWIO), so checkpoints map 1:1 onto the reference graph's variables
(SURVEY.md §5.4). The default file format is TF's own Saver-V2 tensor bundle
(``model.ckpt-<step>.index`` + ``model.ckpt-<step>.data-00000-of-00001``, utils/tf_bundle.py):
``global_step``, ``beta1_power`` / ``beta2_power`` (Adam's non-slot variables), ``<var>/Adam``,
``<var>/Adam_1`` and ``<var>/ExponentialMovingAverage`` as TF 1.x names them, plus one extra
``deepspeech_amd/adam_t``. ``fmt="torch"`` writes the earlier single ``torch.save`` file instead;
restore and eval read either. Saving never blocks a GPU training thread (CheckpointManager:
device snapshot -> side-stream copy into pinned buffers -> writer thread, which streams the
bundle's data shard straight from the pinned buffer).
"""
from __future__ import annotations

import glob
import math
import os
import re
import threading
from typing import Callable, Dict, List, Optional, Tuple

import torch

from ..models.deepspeech2 import DeepSpeech2
from . import tf_bundle as TB

EMA_SUFFIX = "/ExponentialMovingAverage"
ADAM_M = "/Adam"
ADAM_V = "/Adam_1"


def _conv_to_tf(w: torch.Tensor) -> torch.Tensor:      # [O, I, H, W] -> [H, W, I, O]
    return w.permute(2, 3, 1, 0).contiguous()


def _conv_from_tf(w: torch.Tensor) -> torch.Tensor:    # [H, W, I, O] -> [O, I, H, W]
    return w.permute(3, 2, 0, 1).contiguous()


def _nhwc_col_perm(model: DeepSpeech2):
    """Column permutation between the compute layout of the first layer's input (NCHW
    flatten of conv2: feature c*F2 + f, src/deepSpeech_NCHW.py:166-168) and the NHWC graph's
    channels-last flatten (f*C + c, src/deepSpeech.py:163-167): (to_tf, from_tf) on W."""
    C = model.num_filters
    F2 = model.rnn_in // C
    nhwc_of = torch.arange(C * F2).view(C, F2).t().reshape(-1)     # nhwc column j <- nchw column
    inv = torch.empty_like(nhwc_of)
    inv[nhwc_of] = torch.arange(C * F2)

    def to_tf(w):
        return w.index_select(-1, nhwc_of.to(w.device)).contiguous()

    def from_tf(w):
        return w.index_select(-1, inv.to(w.device)).contiguous()
    return to_tf, from_tf


def tf_name_map(model: DeepSpeech2) -> List[Tuple[str, str, Callable, Callable]]:
    """[(tf_name, torch_name, to_tf, from_tf)] for every parameter and buffer.

    NCHW graph (default): src/deepSpeech_NCHW.py + custom_ops.stacked_brnn scopes.
    NHWC graph (layout 'nhwc', --nchw False): src/deepSpeech.py scopes — conv BN under 'bn'
    with the zero-debiased moment EMAs, the RNN as two MultiRNNCells under
    bidirectional_rnn/{fw,bw}/multi_rnn_cell/cell_<i> (rnn/multi_rnn_cell/... uni-dir), and
    the first layer's W in channels-last input order."""
    ident = lambda t: t  # noqa: E731
    nhwc = getattr(model, "layout", "nchw") == "nhwc"
    out = []
    for blk in ("conv1", "conv2"):
        out += [
            ("%s/weights" % blk, "%s.weight" % blk, _conv_to_tf, _conv_from_tf),
            ("%s/biases" % blk, "%s.bias" % blk, ident, ident),
        ]
        if nhwc:
            ema = "%s/bn/moments/Squeeze%s/ExponentialMovingAverage"
            out += [
                ("%s/bn/beta" % blk, "%s.bn_beta" % blk, ident, ident),
                ("%s/bn/gamma" % blk, "%s.bn_gamma" % blk, ident, ident),
                ((ema % (blk, "")) + "/biased", "%s.ema_mean_biased" % blk, ident, ident),
                ((ema % (blk, "_1")) + "/biased", "%s.ema_var_biased" % blk, ident, ident),
                ((ema % (blk, "")) + "/local_step", "%s.ema_steps" % blk, ident, ident),
            ]
        else:
            out += [
                ("%s/bn2/beta" % blk, "%s.bn_beta" % blk, ident, ident),
                ("%s/bn2/gamma" % blk, "%s.bn_gamma" % blk, ident, ident),
                ("%s/bn2/moving_mean" % blk, "%s.running_mean" % blk, ident, ident),
                ("%s/bn2/moving_variance" % blk, "%s.running_var" % blk, ident, ident),
            ]
    cell_scope = "CustomRNNCell2" if model.cell == "rnn_relu" else "GRUCell"
    perm = _nhwc_col_perm(model) if nhwc else None
    for i, layer in enumerate(model.rnn):
        for dname in (["fw", "bw"] if layer.bw is not None else ["fw"]):
            if nhwc:
                if layer.bw is not None:
                    scope = "bidirectional_rnn/%s/multi_rnn_cell/cell_%d/%s" % (dname, i, cell_scope)
                else:
                    scope = "rnn/multi_rnn_cell/cell_%d/%s" % (i, cell_scope)
            elif layer.bw is not None:
                scope = "rnn/brnn-%d/bidirectional_rnn/%s/%s" % (i, dname, cell_scope)
            else:
                scope = "rnn/rnn-%d/%s" % (i, cell_scope)
            tp = "rnn.%d.%s" % (i, dname)
            w_to, w_from = (perm if (perm is not None and i == 0) else (ident, ident))
            out += [("%s/W" % scope, tp + ".W", w_to, w_from),
                    ("%s/U" % scope, tp + ".U", ident, ident),
                    ("%s/%s" % (scope, "B" if model.cell == "rnn_relu" else "b_i"), tp + ".b", ident, ident),
                    ("%s/sbn/moving_mean" % scope, tp + ".sbn_mean", ident, ident),
                    ("%s/sbn/moving_variance" % scope, tp + ".sbn_var", ident, ident)]
            if model.cell == "gru":
                out.append(("%s/b_h" % scope, tp + ".b_h", ident, ident))
    out += [("softmax_linear/weights", "fc_weight", ident, ident),
            ("softmax_linear/biases", "fc_bias", ident, ident)]
    return out


def model_to_tf(model: DeepSpeech2) -> Dict[str, torch.Tensor]:
    sd = dict(model.named_parameters())
    sd.update(dict(model.named_buffers()))
    return {tf: to_tf(sd[tn].detach()) for tf, tn, to_tf, _ in tf_name_map(model)}


def _in_dims(model: DeepSpeech2) -> List[int]:
    return [layer.fw.W.shape[1] for layer in model.rnn]


def normalize_layout(model: DeepSpeech2, tensors: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Accept the MKL-DNN single-blob RNN layout (engine=mkldnn_rnn / cudnn_rnn checkpoints,
    src/mkldnn_rnn_op.py:16-45) by unpacking its blobs into the per-matrix names."""
    from .mkldnn_blob import from_mkldnn_layout, is_mkldnn_checkpoint
    if is_mkldnn_checkpoint(tensors):
        return from_mkldnn_layout(tensors, model.num_hidden, _in_dims(model))
    return tensors


def load_model_from_tf(model: DeepSpeech2, tensors: Dict[str, torch.Tensor], strict: bool = True,
                       use_ema: bool = False) -> List[str]:
    """Copy TF-named tensors into the model; with use_ema, prefer '<name>/ExponentialMovingAverage'."""
    tensors = normalize_layout(model, tensors)
    sd = dict(model.named_parameters())
    sd.update(dict(model.named_buffers()))
    missing = []
    with torch.no_grad():
        for tf, tn, _, from_tf in tf_name_map(model):
            key = tf + EMA_SUFFIX if (use_ema and (tf + EMA_SUFFIX) in tensors) else tf
            if key not in tensors:
                missing.append(tf)
                continue
            src = from_tf(tensors[key].to(torch.float32))
            dst = sd[tn]
            if tuple(src.shape) != tuple(dst.shape):
                raise ValueError("shape mismatch for %s: %s vs %s" % (tf, tuple(src.shape), tuple(dst.shape)))
            dst.copy_(src.to(dst.dtype))
    if strict and missing:
        raise KeyError("checkpoint lacks %s" % missing[:5])
    return missing


def _arena_slots(trainer) -> Dict[str, torch.Tensor]:
    """Adam m/v and EMA shadows keyed by TF slot names."""
    out = {}
    model = trainer.model
    names = {tn: (tf, to_tf) for tf, tn, to_tf, _ in tf_name_map(model)}
    arena, opt = trainer.arena, trainer.opt
    vm, vv = arena.views(opt.m), arena.views(opt.v)
    ve = arena.views(opt.ema) if opt.ema is not None else None
    for tn in arena.names:
        tf, to_tf = names[tn]
        out[tf + ADAM_M] = to_tf(vm[tn])
        out[tf + ADAM_V] = to_tf(vv[tn])
        if ve is not None:
            out[tf + EMA_SUFFIX] = to_tf(ve[tn])
    return out


def _load_arena_slots(trainer, tensors: Dict[str, torch.Tensor]) -> None:
    model = trainer.model
    names = {tn: (tf, from_tf) for tf, tn, _, from_tf in tf_name_map(model)}
    arena, opt = trainer.arena, trainer.opt
    vm, vv = arena.views(opt.m), arena.views(opt.v)
    ve = arena.views(opt.ema) if opt.ema is not None else None
    with torch.no_grad():
        for tn in arena.names:
            tf, from_tf = names[tn]
            if tf + ADAM_M in tensors:
                vm[tn].copy_(from_tf(tensors[tf + ADAM_M]))
                vv[tn].copy_(from_tf(tensors[tf + ADAM_V]))
            if ve is not None and tf + EMA_SUFFIX in tensors:
                ve[tn].copy_(from_tf(tensors[tf + EMA_SUFFIX]))


def write_state_file(directory: str, latest: str, all_paths: List[str]) -> None:
    """TF's `checkpoint` text-proto state file."""
    lines = ['model_checkpoint_path: "%s"' % latest]
    lines += ['all_model_checkpoint_paths: "%s"' % p for p in all_paths]
    tmp = os.path.join(directory, "checkpoint.tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(directory, "checkpoint"))


def latest_checkpoint(directory: str) -> Optional[str]:
    """tf.train.get_checkpoint_state(dir).model_checkpoint_path equivalent."""
    state = os.path.join(directory, "checkpoint")
    if os.path.exists(state):
        with open(state) as f:
            for line in f:
                m = re.match(r'\s*model_checkpoint_path:\s*"(.*)"', line)
                if m:
                    p = m.group(1)
                    return p if os.path.isabs(p) else os.path.join(directory, p)
    cands = {}
    for p in glob.glob(os.path.join(directory, "model.ckpt-*")):
        m = re.match(r"^(.*model\.ckpt-(\d+))(\.index)?$", p)
        if m:
            cands[m.group(1)] = int(m.group(2))
    if not cands:
        return None
    return max(cands, key=cands.get)


def step_from_path(path: str) -> int:
    """global_step parsed from the file name (src/deepSpeech_train.py:393-397)."""
    return int(path.split("/")[-1].split("-")[-1])


class _HostSlot:
    """One pinned host copy of the optimizer-visible state: the arena's fp32 weights, Adam m
    and v, the EMA shadows (rows of ``flat``) and the model's buffers."""

    def __init__(self, rows: int, numel: int, bufs: Dict[str, torch.Tensor]):
        self.flat = torch.empty(rows, numel, dtype=torch.float32, pin_memory=True)
        self.bufs = {n: torch.empty(b.shape, dtype=b.dtype, pin_memory=True) for n, b in bufs.items()}
        self.bad = torch.empty(1, dtype=torch.int32, pin_memory=True)
        self.writing = False


class CheckpointManager:
    """model.ckpt-<step> files + the TF ``checkpoint`` state file (reference cadence: every 10
    steps, src/deepSpeech_train.py:354-356, :471).

    GPU saves never block the training thread:
      1. on the training stream, one device-to-device copy of the arena's weights, Adam m / v
         and EMA (plus the model buffers) into a device snapshot: ~0.3 ms per 0.74 GB (the
         headline model) at HBM speed, ordered after the saved step's optimizer update and
         before the next step's, so the snapshot is exactly step <step>'s state;
      2. on a side stream, the snapshot's copy into a pinned host slot, and an
         event; no host synchronisation on the training thread;
      3. a writer thread waits for that event, maps the arena onto the TF variable names and
         writes the file.
    The training thread never waits for the disk: a save requested while the writer is still
    busy with an earlier file takes no snapshot at all (no copies; counted in ``skipped``,
    logged once per stretch), so the file written next is the newest state at the first save
    after the writer frees up. ``force=True`` (the last step of a run) waits for the writer
    instead. The next save's device snapshot waits (on the stream, not the host) for the
    previous host copy to have read the device snapshot. A save whose step, or an earlier
    one, had a non-finite loss (the device-side watch, utils/stats.py) is not written.
    CPU trainers (and async_save=False) take the synchronous snapshot() path."""

    def __init__(self, directory: str, max_to_keep: int = 100, async_save: bool = True, fmt: str = "tf",
                 nan_policy: str = "abort"):
        if fmt not in ("tf", "torch"):
            raise ValueError("checkpoint format must be 'tf' (TF Saver-V2 bundle) or 'torch'")
        self.dir = directory
        self.max_to_keep = max_to_keep
        self.async_save = async_save
        self.fmt = fmt
        # a save after a non-finite loss is dropped only when that loss ends the run
        # (nan_policy "abort"); under "skip" the skipped updates left the weights finite
        self.nan_policy = nan_policy
        self.dropped: List[int] = []
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None
        os.makedirs(directory, exist_ok=True)
        self.kept: List[str] = []
        state = os.path.join(directory, "checkpoint")
        if os.path.exists(state):
            with open(state) as f:
                self.kept = [m.group(1) for m in (re.match(r'\s*all_model_checkpoint_paths:\s*"(.*)"', l) for l in f) if m]
        # asynchronous GPU path
        self._cv = threading.Condition()
        self._pending = None          # (slot, event, meta) waiting for the writer
        self._busy = False            # the writer is writing a file
        self._closed = False
        self._slots: List[_HostSlot] = []
        self._dev = None              # device snapshot: [rows, numel] + buffers + bad word
        self._stream = None
        self._d2h_done = None         # event: the last host copy has read the device snapshot
        self.skipped: List[int] = []  # saves requested while the writer was busy (no snapshot)
        self.write_s: List[float] = []    # seconds per file written (the effective save cadence)
        self.written: List[int] = []
        self._behind = False

    # ---- synchronous snapshot (CPU, tests, async_save=False) ------------------------------
    def snapshot(self, trainer) -> Dict[str, object]:
        out: Dict[str, object] = {}
        for k, v in model_to_tf(trainer.model).items():
            out[k] = v.detach().to("cpu", copy=True)
        for k, v in _arena_slots(trainer).items():
            out[k] = v.detach().to("cpu", copy=True)
        return self._finish(trainer.model, out, _meta(trainer))

    def _finish(self, model, out: Dict[str, object], meta: Dict[str, object]) -> Dict[str, object]:
        if getattr(model, "param_layout", "tf") == "mkldnn":
            # engine=mkldnn_rnn / cudnn_rnn: the reference's MkldnnRNNCell blob per direction
            from .mkldnn_blob import to_mkldnn_layout
            tens = to_mkldnn_layout({k: v for k, v in out.items() if isinstance(v, torch.Tensor)})
            out = {k: v for k, v in out.items() if not isinstance(v, torch.Tensor)}
            out.update(tens)
        out.update(meta)
        return out

    def save(self, trainer, step: int, force: bool = False) -> Optional[str]:
        """Checkpoint ``trainer`` as model.ckpt-<step>; returns the path, or None when the save
        was skipped because the writer is still busy (GPU, not forced)."""
        name = "model.ckpt-%d" % step
        path = os.path.join(self.dir, name)
        if hasattr(trainer, "flush"):
            trainer.flush()       # an optimizer update carried into the next step (Trainer)
        if self.async_save and trainer.arena.flat.is_cuda:
            return path if self._save_async(trainer, step, force) else None
        self.wait()
        if self.nan_policy == "abort" and hasattr(trainer, "first_nonfinite_step"):
            bad = trainer.first_nonfinite_step()
            if bad is not None and bad <= step:
                self._drop(step, bad)
                return None
        snap = self.snapshot(trainer)
        if self.async_save:
            self._thread = threading.Thread(target=self._write_guarded, args=(snap, step), daemon=True)
            self._thread.start()
        else:
            self._write(snap, step)
        return path

    # ---- file writing ----------------------------------------------------------------------
    def _drop(self, step: int, bad: int) -> None:
        self.dropped.append(step)
        print("checkpoint for step %d not written: non-finite loss at step %d (nan_policy abort)" % (step, bad),
              flush=True)

    def _write(self, snap: Dict[str, object], step: int) -> None:
        import time
        t0 = time.perf_counter()
        name = "model.ckpt-%d" % step
        path = os.path.join(self.dir, name)
        if self.fmt == "tf":
            TB.write_bundle(path, bundle_tensors(snap))
        else:
            tmp = path + ".tmp"
            torch.save(snap, tmp)
            os.replace(tmp, path)
        if name in self.kept:
            self.kept.remove(name)
        self.kept.append(name)
        while len(self.kept) > self.max_to_keep:
            old = os.path.join(self.dir, self.kept.pop(0))
            for f in [old] + TB.bundle_files(old):
                try:
                    os.remove(f)
                except FileNotFoundError:
                    pass
        write_state_file(self.dir, name, self.kept)
        self.written.append(step)
        self.write_s.append(time.perf_counter() - t0)

    def _write_guarded(self, snap, step) -> None:
        try:
            self._write(snap, step)
        except BaseException as e:  # surfaced by wait()
            self._error = e

    # ---- asynchronous GPU path -------------------------------------------------------------
    def _save_async(self, trainer, step: int, force: bool) -> bool:
        self._raise()
        with self._cv:
            if self._slots and (self._busy or self._pending is not None):
                if not force:
                    if not self._behind:
                        print("checkpoint writer busy: skipping saves from step %d until it is free" % step,
                              flush=True)
                    self._behind = True
                    self.skipped.append(step)
                    return False
                while self._busy or self._pending is not None:
                    self._cv.wait(timeout=1.0)
            self._behind = False
        arena, opt = trainer.arena, trainer.opt
        srcs = [arena.flat, opt.m, opt.v] + ([opt.ema] if opt.ema is not None else [])
        bufs = {n: b for n, b in trainer.model.named_buffers()}
        in_arena = set(arena.names)
        bufs.update({n: p.detach() for n, p in trainer.model.named_parameters() if n not in in_arena})
        dev = arena.flat.device
        if self._dev is None or self._dev[0].shape != (len(srcs), arena.numel):
            self.wait()
            self._dev = (torch.empty(len(srcs), arena.numel, device=dev, dtype=torch.float32),
                         {n: torch.empty_like(b) for n, b in bufs.items()},
                         torch.empty(1, device=dev, dtype=torch.int32))
            # one pinned slot: a snapshot is only taken while the writer is idle (see save)
            self._slots = [_HostSlot(len(srcs), arena.numel, bufs)]
            self._stream = torch.cuda.Stream(device=dev)
            self._d2h_done = None
            self._start_writer()
        dflat, dbufs, dbad = self._dev
        main = torch.cuda.current_stream(dev)
        if self._d2h_done is not None:
            main.wait_event(self._d2h_done)       # the previous host copy has read the snapshot
        for i, t in enumerate(srcs):
            dflat[i].copy_(t)
        for n, b in bufs.items():
            dbufs[n].copy_(b)
        dbad.copy_(trainer.watch.first_bad)
        with self._cv:
            slot = next(s for s in self._slots if not s.writing)
        side = self._stream
        side.wait_stream(main)
        with torch.cuda.stream(side):
            slot.flat.copy_(dflat, non_blocking=True)
            for n, b in dbufs.items():
                slot.bufs[n].copy_(b, non_blocking=True)
            slot.bad.copy_(dbad, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
        self._d2h_done = ev
        meta = _meta(trainer)
        meta["step"] = step
        meta["watch_base"] = int(trainer.watch._base)
        with self._cv:
            self._pending = (slot, ev, meta, trainer.model, list(zip(arena.names, arena.offsets)), len(srcs))
            self._cv.notify_all()
        return True

    def _start_writer(self) -> None:
        if self._thread is not None:
            return
        self._thread = threading.Thread(target=self._writer_loop, daemon=True)
        self._thread.start()

    def _writer_loop(self) -> None:
        while True:
            with self._cv:
                while self._pending is None and not self._closed:
                    self._cv.wait()
                if self._pending is None and self._closed:
                    return
                job, self._pending = self._pending, None
                slot = job[0]
                slot.writing = True
                self._busy = True
            try:
                self._write_job(*job)
            except BaseException as e:   # surfaced by wait() / the next save()
                self._error = e
            finally:
                with self._cv:
                    slot.writing = False
                    self._busy = False
                    self._cv.notify_all()

    def _write_job(self, slot: "_HostSlot", ev, meta, model, layout, rows) -> None:
        ev.synchronize()
        step = meta.pop("step")
        base = meta.pop("watch_base")
        bad = int(slot.bad[0])
        if self.nan_policy == "abort" and bad >= 0 and base + bad <= step:
            self._drop(step, base + bad)
            return
        # the bundle writer streams views of the pinned slot (it is not reused before this job
        # returns); torch.save would serialise a view's whole storage, so that format copies
        own = (lambda t: t) if self.fmt == "tf" else (lambda t: t.clone())
        names = {tn: (tf, to_tf) for tf, tn, to_tf, _ in tf_name_map(model)}
        params = dict(model.named_parameters())
        out: Dict[str, object] = {}
        suffixes = ["", ADAM_M, ADAM_V] + ([EMA_SUFFIX] if rows == 4 else [])
        for tn, (o, n) in layout:
            tf, to_tf = names[tn]
            shape = params[tn].shape
            for r, suf in enumerate(suffixes):
                out[tf + suf] = own(to_tf(slot.flat[r, o:o + n].view(shape)))
        for tf, tn, to_tf, _ in tf_name_map(model):
            if tn in slot.bufs:
                out[tf] = own(to_tf(slot.bufs[tn]))
        self._write(self._finish(model, out, meta), step)

    def _raise(self):
        if self._error is not None:
            e, self._error = self._error, None
            raise e

    def wait(self) -> None:
        """Block until every requested checkpoint is on disk (or surfaced its error)."""
        if self._slots:
            with self._cv:
                while self._pending is not None or self._busy:
                    self._cv.wait(timeout=1.0)
        elif self._thread is not None:
            self._thread.join()
            self._thread = None
        self._raise()

    def close(self) -> None:
        self.wait()
        if self._slots:
            with self._cv:
                self._closed = True
                self._cv.notify_all()
            if self._thread is not None:
                self._thread.join()
                self._thread = None


def _meta(trainer) -> Dict[str, object]:
    return {"global_step": int(trainer.global_step),
            "beta1_power": float(trainer.opt.b1 ** trainer.opt.t),
            "beta2_power": float(trainer.opt.b2 ** trainer.opt.t),
            "adam_t": int(trainer.opt.t),
            "format": "deepspeech_amd/tfnames/v1"}


ADAM_T = "deepspeech_amd/adam_t"


def bundle_tensors(snap: Dict[str, object]) -> Dict[str, torch.Tensor]:
    """Tensors of a TF bundle for a snapshot dict: its tensors plus the scalar variables TF's
    graph holds (global_step int64, Adam's beta1_power / beta2_power fp32) and adam_t."""
    out = {k: v for k, v in snap.items() if isinstance(v, torch.Tensor)}
    if "global_step" in snap:
        out["global_step"] = torch.tensor(int(snap["global_step"]), dtype=torch.int64)
    for k in ("beta1_power", "beta2_power"):
        if k in snap:
            out[k] = torch.tensor(float(snap[k]), dtype=torch.float32)
    if "adam_t" in snap:
        out[ADAM_T] = torch.tensor(int(snap["adam_t"]), dtype=torch.int64)
    return out


def _from_bundle(prefix: str) -> Dict[str, object]:
    data: Dict[str, object] = dict(TB.read_bundle(prefix))
    out: Dict[str, object] = {k: v for k, v in data.items()
                              if k not in ("global_step", "beta1_power", "beta2_power", ADAM_T)}
    out["format"] = "tf_bundle"
    if "global_step" in data:
        out["global_step"] = int(data["global_step"])
    for k in ("beta1_power", "beta2_power"):
        if k in data:
            out[k] = float(data[k])
    if ADAM_T in data:
        out["adam_t"] = int(data[ADAM_T])
    elif "beta1_power" in data and 0.0 < float(data["beta1_power"]) < 1.0:
        # a TF-written checkpoint: Adam's step count from beta1_power = 0.9^t (default beta1)
        out["adam_t"] = int(round(math.log(float(data["beta1_power"])) / math.log(0.9)))
    return out


def load_checkpoint_file(path: str) -> Dict[str, object]:
    """A checkpoint by path or prefix: a TF Saver-V2 bundle (``<path>.index`` exists: ours or
    TF-written) or a ``torch.save`` file (loaded with weights_only=True)."""
    if TB.bundle_exists(path):
        return _from_bundle(path)
    return torch.load(path, map_location="cpu", weights_only=True)


read_checkpoint = load_checkpoint_file


def restore(trainer, directory_or_file: str) -> Optional[int]:
    """Restore model + Adam slots + EMA + step; returns the global step (or None)."""
    path = directory_or_file
    if os.path.isdir(path):
        path = latest_checkpoint(path)
        if path is None:
            print("No checkpoint file found")
            return None
    data = load_checkpoint_file(path)
    if hasattr(trainer, "flush"):
        trainer.flush()          # a carried optimizer update lands before the restored state
    tensors = normalize_layout(trainer.model, {k: v for k, v in data.items() if isinstance(v, torch.Tensor)})
    load_model_from_tf(trainer.model, tensors, strict=True)
    _load_arena_slots(trainer, tensors)
    trainer.arena.mark_dirty()
    step = step_from_path(path)
    if data.get("format") and "global_step" in data:
        # snapshot() (and TF's Saver, whose global_step apply_gradients already advanced) stores trainer.global_step as it stood after the saved step
        # (Trainer.step already counted it), i.e. the index of the next step to run
        trainer.global_step = int(data["global_step"])
    else:
        # file-name fallback: the reference saves model.ckpt-<step> right after running
        # step <step> (src/deepSpeech_train.py:354-356), so <step>+1 runs next
        trainer.global_step = step + 1
    trainer.opt.t = int(data.get("adam_t", trainer.global_step))
    return step
