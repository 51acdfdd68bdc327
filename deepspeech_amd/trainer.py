"""One training step, shared by the CLI driver (train.py) and bench.py.

Reference step (src/deepSpeech_train.py:292-380 + :419-496): forward, mean CTC loss,
backward, Adam with staircase-decayed LR, weight EMA (0.9999, num_updates=global_step),
loss EMA (0.9), NaN assert.

MI355X step:
  arena.zero_grad(lazy)                   HIP engine: no memset (every fused op's first
                                          gradient write overwrites); ref engine: one memset
  logits = model(feats)                   MFMA conv + fused BN/clip -> persistent RNN
                                          layers -> FC GEMM
  loss = fused CTC(logits)                loss and dlogits in one kernel
  loss.backward()                         RCCL bucket all-reduces launch from grad hooks
  bucketer.finish()                       wait for the in-flight buckets
  optimizer.step()                        fused Adam + EMA, one kernel over the arena
No host synchronisation happens inside the step; the loss is returned as a device tensor.
"""
from __future__ import annotations

from dataclasses import dataclass, field
import os
import time
from typing import Dict, Optional

import torch

from .models import DeepSpeech2
from .ops import _ext
from .ops import ctc as _CTC
from .ops.optim import FusedAdamEMA, ParamArena, exponential_decay
from .parallel.grad_sync import GradBucketer, broadcast_params
from .utils import trace as TR
from .utils.stats import NonfiniteWatch


# host clock of the eager/graph decision (tests freeze it)
_clock = time.perf_counter


@dataclass
class LRSchedule:
    initial_lr: float
    decay_steps: int
    decay_rate: float
    staircase: bool = True

    def __call__(self, step: int) -> float:
        return exponential_decay(self.initial_lr, step, self.decay_steps, self.decay_rate, self.staircase)


def lr_schedule_from_args(args, steps_per_epoch: int) -> LRSchedule:
    """decay_steps = batches_per_epoch * num_epochs_per_decay (src/deepSpeech_train.py:239-241),
    with the epoch size taken from the ACTIVE dataset (quirk Q14)."""
    return LRSchedule(args.initial_lr, max(1, int(steps_per_epoch * args.num_epochs_per_decay)),
                      args.lr_decay_factor)


# Optimizer range of the head + layers >= 1 beside layer 0's BPTT when the weight gradients are
# not deferred, on a capped grid (same box, config 5 fp8, 2 rounds: off 21.77 / 21.39 ms/step,
# full grid 21.16 / 21.08, 192 blocks 21.04 / 20.99, 512 blocks 21.04 / 20.98)
_EARLY_UPPER = True
_UPPER_GRID = 512
# single device, weight gradients deferred to the grouped tail launch: that launch can apply Adam +
# EMA to the recurrent weights in its epilogue (csrc/gemm8.hip "Fused optimizer epilogue")
# instead of storing their gradients for a separate optimizer pass to read back. Bitwise the
# same update (tests/test_gemm_gpu.py), but measured slower at the headline (same box, round 4:
# 8.21 vs 8.04 ms/step): the grid's workgroups finish their tiles in lockstep, so every
# epilogue streams its 2.2 MB of optimizer state at the same moment (HBM-bound, +450 us on the
# group) instead of overlapping the MFMA work; off until that is staggered
_FUSED_OPT = False
# grid cap (blocks) of that early optimizer range: it streams beside the conv front-end's
# backward, whose latency-bound conv1 weight gradient it slowed 3x on the full grid (headline,
# same box, 4 rounds: 7.745-7.773 ms/step at 384 vs 7.788-7.817 uncapped and 7.793-7.821 at 512;
# another box 3 rounds: 384 -0.45 %, 256 -0.2 to -0.3 %). Only when the range is the whole head
# + recurrent stack (every weight gradient deferred to the grouped tail): config 5, whose upper
# range already ran beside layer 0's BPTT, measured +0.15-0.3 % with the cap on its remainder.
_EARLY_GRID = 384
# the same range when the upper part already ran beside layer 0's BPTT (0: uncapped)
_LOWER_GRID = 0
# grid cap (blocks) of the data-parallel per-bucket Adam + EMA ranges, which stream beside the
# BPTTs (0: uncapped). --force_dp at world 1, same box, 3 rounds: uncapped 7.754 / 7.747 / 7.705,
# 512 7.782 / 7.725 / 7.719, 256 7.771 / 7.790 / 7.814, 128 7.86-7.88 ms/step
_BUCKET_GRID = 0
# with defer_update, the beside dU GEMMs of the layers above the upper trigger go to the next
# step's forward too (ops/rnn.py WgradScheduler.carry_du)
_CARRY_DU = True
# carried optimizer chunks beside a forward recurrence: blocks per idle CU, and the unused LDS
# each block reserves so that it cannot share a CU with a recurrence workgroup (132 KB of LDS).
# Same box, 3 rounds: 1 block, no reservation 7.388-7.407 ms/step; 2 blocks + 32 KB 7.405-7.426;
# 4 blocks + 32 KB 7.432-7.435
_CARRY_BLOCKS_PER_CU = 1
_CARRY_LDS = 0
# capture step graphs on one stream (False: the weight-gradient side stream too; single-stream
# capture is not bitwise at H = 800, where the deferral needs the side stream)
_GRAPH_SINGLE_STREAM = False


def _check_hw_queues() -> None:
    """A DP step drives more HIP streams (main, weight-gradient side stream, bucket
    ordering stream, RCCL's own) than HIP's default 4 hardware queues: streams then share
    queues and the side stream serialises behind the BPTT (+6.6 % step time measured,
    profiles/r2_dp_readiness.md). utils/setenvs.py raises the floor to 8, but only if it runs
    before HIP initialises; warn loudly when it did not."""
    import os
    import warnings
    try:
        q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        q = 4
    if q < 8:
        warnings.warn("GPU_MAX_HW_QUEUES=%d (< 8): data-parallel streams share hardware queues; "
                      "call deepspeech_amd.utils.setenvs.setenvs() before anything initialises HIP" % q)


def _long_sequence(batch: Dict[str, torch.Tensor]) -> bool:
    """True when the batch's recurrence runs >= ops/rnn.py _PARTIAL_MIN_T steps."""
    from .models.deepspeech2 import conv_out_len
    from .ops import rnn as RNN
    return conv_out_len(int(batch["feats"].shape[1]))[1] >= RNN._PARTIAL_MIN_T


@dataclass
class _ShapeState:
    seen: int = 0
    graph: Optional["_StepGraph"] = None
    mode: Optional[str] = None               # "eager" / "graph" once decided
    host_s: list = field(default_factory=list)     # host enqueue seconds of the eager steps
    spans: list = field(default_factory=list)      # (start, end) events of undecided replays


@dataclass
class _StepGraph:
    graph: "torch.cuda.CUDAGraph"
    feats: torch.Tensor
    seq_lens: torch.Tensor
    labels: torch.Tensor
    label_lens: torch.Tensor
    loss: torch.Tensor
    ptrs: tuple = ()          # the state buffers the graph was captured on (Trainer._state_ptrs)


class Trainer:
    def __init__(self, model: DeepSpeech2, lr_schedule: LRSchedule, moving_avg_decay: Optional[float] = 0.9999,
                 world_size: int = 1, bucket_mb: float = 32.0, allreduce_bf16: bool = False,
                 nan_policy: str = "abort", collapse_repeated: bool = False, force_buckets: bool = False,
                 step_graphs=False, graph_warmup: int = 2, bucket_split_after=(), defer_update: bool = False,
                 dp_graphs: bool = False):
        self.model = model
        # data parallel: capture the bucketed step too (RCCL all-reduces and the per-bucket
        # optimizer ranges inside the shape's graph); opt-in, see graphs_active()
        self.dp_graphs = bool(dp_graphs)
        # carry the optimizer update of the FC head and recurrent layers >= 1 into the next
        # step's forward (see _body); readers of the weights between steps call flush()
        self.defer_update = bool(defer_update)
        if model.engine == "hip":
            from .ops.rnn import check_knobs
            check_knobs()            # timing-only kernel switches never reach a training run
        self._seed = {}            # (device, dtype) -> device scalar 1.0 (backward seed)
        # bf16 compute shadows of the weights only for the HIP engine (fused ops read them)
        self.arena = ParamArena(model, bf16_shadow=(model.engine == "hip"))
        self.opt = FusedAdamEMA(self.arena, lr=lr_schedule.initial_lr, ema_decay=moving_avg_decay)
        self.lr_schedule = lr_schedule
        self.world = world_size
        self.bucketer = GradBucketer(self.arena, bucket_mb=bucket_mb, compress_bf16=allreduce_bf16,
                                     world_size=world_size, force=force_buckets, split_after=bucket_split_after)
        if world_size > 1:
            broadcast_params(self.arena)
            self.arena.mark_dirty()
            if self.opt.ema is not None:
                self.opt.ema.copy_(self.arena.flat)
        # Deferring the input-weight gradients of layers >= 1 to the end of the BPTT chain
        # measured within noise on one GPU (profiles/r1_s3_negative_results.md) and, with
        # data parallelism, would hold ~40 % of the gradient bytes (every layer's W) back
        # until backward ends instead of releasing one bucket per layer for overlap: on for
        # the single-GPU path only (DS2_DEFER_DW=0/1 overrides)
        # (per arena: another Trainer / model in this process keeps its own setting)
        self.arena.wgrad.set_deferral(world_size == 1 and not self.bucketer.enabled)
        self.global_step = 0
        self.nan_policy = nan_policy
        self.collapse_repeated = collapse_repeated
        self.loss_ema: Optional[float] = None
        self.last_skip: Optional[torch.Tensor] = None
        # per-step divergence record on the device (read at host sync points, never skipped)
        self.watch = NonfiniteWatch(self.arena.flat.device)
        # data parallel: optimizer ranges per gradient bucket behind its all-reduce
        # (GradBucketer.set_optimizer); per_bucket_update=False keeps one update after finish()
        self.per_bucket_update = True
        # keep_grads: the fused optimizer epilogue also stores the gradients it consumed (set
        # when something reads arena.grad after a step: gradient summaries)
        self.keep_grads = False
        # single device: arena elements [0, split) — FC head and recurrent stack, laid out
        # before the conv front-end in gradient-production order — get their optimizer update
        # as soon as the recurrent weight gradients are issued (Trainer.step)
        self._early_split, self._early_params = 0, []
        self._layer_first = {}     # recurrent layer k -> arena index of its first parameter
        names = list(self.arena.names)
        first_conv = next((i for i, n in enumerate(names) if n.startswith("conv")), None)
        if self.arena.flat.is_cuda and first_conv:
            self._early_split = self.arena.offsets[first_conv][0]
            self._early_params = list(self.arena.params[:first_conv])
            for i, n in enumerate(names[:first_conv]):
                if n.startswith("rnn."):
                    self._layer_first.setdefault(int(n.split(".")[1]), i)
        if self.bucketer.enabled and self.arena.flat.is_cuda:
            _check_hw_queues()
        # step graphs (False, True or "auto"): the whole single-device step (forward, CTC,
        # backward, Adam + EMA) captured once per batch shape and replayed (see _graph_step)
        self.step_graphs = step_graphs
        self.graph_warmup = max(1, int(graph_warmup))
        self._shapes: Dict[tuple, "_ShapeState"] = {}
        # auto mode: shape key -> (chosen mode, best eager ms, best replay ms)
        self.graph_modes: Dict[tuple, tuple] = {}
        self._graph_pool = None
        self._chunk_cache = {}

    def upper_range(self, b: int):
        """(end, params) of the arena range holding the FC head and the recurrent layers >= b:
        everything laid out before layer b-1 (the arena is in gradient-production order). None
        when there is no such split (b < 1 or no layer b-1 in the arena)."""
        i = self._layer_first.get(b - 1) if b >= 1 else None
        if not i:
            return None
        return self.arena.offsets[i][0], list(self.arena.params[:i])

    def _chunks(self, hi: int):
        """[(lo, hi, params)] of arena range [0, hi) split per recurrent layer, in the order the
        next forward reads them: layer 1, 2, ..., the top layer, then the FC head."""
        key = ("chunks", hi)
        c = self._chunk_cache.get(key)
        if c is not None:
            return c
        starts = sorted((self.arena.offsets[i][0], k) for k, i in self._layer_first.items())
        layer_at = {s: k for s, k in starts}
        bounds = [0] + [s for s, _ in starts if 0 < s < hi] + [hi]
        out = []
        for lo, up in zip(bounds[:-1], bounds[1:]):
            params = [p for p, (o, n) in zip(self.arena.params, self.arena.offsets) if lo <= o < up]
            if up > lo:
                out.append((lo, up, params, layer_at.get(lo, -1)))
        c = self._chunk_cache[key] = list(reversed(out))
        return c

    def _carry_update(self, hi: int, lr_t: float, keep: float, gscale: float, dus=None) -> None:
        """Register the optimizer update of arena range [0, hi) (FC head + recurrent layers >= 1,
        whose gradients are final once layer 1's weight gradients are issued) with the arena, to
        be enqueued by the NEXT forward one chunk beside each recurrence (ops/rnn.py FusedBiLayer:
        layer k's chunk beside layer k-1's recurrence, the head's beside the top layer's), each
        projection waiting only for its own chunk. In this
        step's tail it ran beside the conv front-end's backward and the bottom layer's weight
        gradients, which it slowed (r5 profile: 387 us of HBM-bound work on the critical tail).
        Bitwise the same update (every element's Adam + EMA is independent of the launch split).

        ``dus``: layer -> the beside dU GEMM of that layer, carried too (ops/rnn.py
        WgradScheduler.carry_du): it runs right after the chunk of the layer below, so layer k's
        chunk is [Adam + EMA of layer k, dU GEMM of layer k+1] and each dU precedes its own
        layer's update on the side stream."""
        opt = self.opt
        dus = dict(dus or {})

        def chunk(lo, up):
            # beside a forward recurrence (grid = the CUs it leaves idle): _CARRY_BLOCKS_PER_CU
            # blocks per idle CU, each reserving LDS so none lands on a recurrence CU
            def fn(grid):
                if grid > 0:
                    opt.apply_range(lo, up, lr_t, keep, gscale, max_grid=grid * _CARRY_BLOCKS_PER_CU,
                                    lds_reserve=_CARRY_LDS if _CARRY_BLOCKS_PER_CU > 1 else 0)
                else:
                    opt.apply_range(lo, up, lr_t, keep, gscale)
            return fn
        chunks = self._chunks(hi)
        todo = []
        for lo, up, params, k in chunks:
            todo.append((chunk(lo, up), params))
            du = dus.pop(k + 1, None) if k >= 0 else None
            if du is not None:
                # its own (parameter-less) chunk right behind: the event readers of layer k wait
                # for is recorded before it, so the next projection does not wait for this GEMM
                todo.append((du, []))
        if dus:
            # a carried dU whose layer has no chunk below it (not expected): first, before any update
            first = list(dus.values())
            todo.insert(0, (lambda grid: [f(grid) for f in first], []))
        self.arena.set_pending_update(todo)

    def _carry_buckets(self, carried, lr_t: float, keep: float, gscale: float) -> None:
        """Data parallel: the Adam + EMA ranges of the gradient buckets inside the head + upper
        layers' arena range go to the next forward (one chunk per bucket, in the order the
        forward reads their weights: highest arena offset first), each waiting for its bucket's
        all-reduce event. Same update as the per-bucket range behind the collective."""
        opt = self.opt
        todo = []
        for lo, hi, ev in sorted(carried, key=lambda c: -c[0]):
            params = [p for p, (o, n) in zip(self.arena.params, self.arena.offsets) if lo <= o < hi]

            def fn(grid, lo=lo, hi=hi, ev=ev):
                torch.cuda.current_stream(self.arena.flat.device).wait_event(ev)
                if grid > 0:
                    opt.apply_range(lo, hi, lr_t, keep, gscale, max_grid=grid * _CARRY_BLOCKS_PER_CU,
                                    lds_reserve=_CARRY_LDS if _CARRY_BLOCKS_PER_CU > 1 else 0)
                else:
                    opt.apply_range(lo, hi, lr_t, keep, gscale)
            todo.append((fn, params))
        self.arena.set_pending_update(todo)

    def flush(self) -> None:
        """Complete an optimizer update carried into the next step (``defer_update``): after
        this, on the current stream, the weights, Adam moments, EMA and bf16 shadows are those
        of the last step. Call before anything reads them between steps: checkpoints, EMA
        swaps, eval, summaries, graph capture, and the end of a timed region."""
        self.arena.settle_updates()

    @property
    def lr(self) -> float:
        return self.lr_schedule(self.global_step)

    def graphs_active(self) -> bool:
        """True when :meth:`step` runs captured step graphs: HIP engine on a GPU, and either one
        device without gradient buckets, or data parallel over RCCL with ``dp_graphs``.

        A data-parallel capture records the step's collectives exactly as the eager step
        issues them: each bucket's all-reduce on the bucketer's ordering stream behind its
        members' producer events, its Adam + EMA range behind the collective, the main stream
        joined at the end. Bucket launch order is fixed per shape (autograd's hook order for a
        given graph), so every rank's graph issues the same collective sequence as its eager
        step, and ranks may even differ in eager / replay per shape (``auto``): the sequence on
        the communicator is the same. The communicator is initialised by the shape's eager
        warm-up steps before any capture. gloo cannot be captured: its process groups keep the
        eager step."""
        if not (bool(self.step_graphs) and self.arena.flat.is_cuda and self.model.engine == "hip"
                and not _FUSED_OPT and not getattr(self.model, "capture", False)):   # taps: eager
            return False
        if not self.bucketer.enabled:
            return self.world == 1
        return self.dp_graphs and self.bucketer.capturable()

    def step(self, batch: Dict[str, torch.Tensor]) -> torch.Tensor:
        # one Adam step count / EMA decay per training step, on the host, whatever runs it
        lr_t, keep = self.opt.prepare(self.lr, self.global_step)
        self.arena.ensure_bf16()      # outside any graph: a restore / EMA swap marks it dirty
        if self.graphs_active():
            loss = self._graph_step(batch, lr_t, keep)
        else:
            loss = self._body(batch, lr_t, keep)
        self.global_step += 1
        return loss

    # ---- captured steps ---------------------------------------------------------------
    @staticmethod
    def graph_key(batch: Dict[str, torch.Tensor]) -> tuple:
        """Shape key of a batch's step graph: features [N, T, F] and the label width rounded
        up to 16 (the CTC kernels read each utterance's own label length, so zero padding
        columns changes no result; rounding keeps one graph per length bucket)."""
        S = int(batch["labels"].shape[1])
        return tuple(batch["feats"].shape) + (max(16, -(-S // 16) * 16),)

    @staticmethod
    def _pad_labels(labels: torch.Tensor, width: int) -> torch.Tensor:
        if labels.shape[1] == width:
            return labels
        return torch.nn.functional.pad(labels, (0, width - labels.shape[1]))

    def _graph_step(self, batch: Dict[str, torch.Tensor], lr_t: float, keep: float) -> torch.Tensor:
        """One step of this batch's shape, eager or through the shape's step graph.

        The first ``graph_warmup`` steps of a new shape run eagerly (real training steps; they
        build the recurrence plans, workspaces and split-K counters the capture then reuses),
        the next one captures the step into a HIP graph and replays it. A replay copies the
        batch into the graph's static inputs, stages (lr_t, ema_keep) into the optimizer's
        device scalars and launches the graph: ~8 launches of host work instead of the eager
        step's ~90 kernel launches, autograd and stream bookkeeping, so the short SortaGrad
        buckets stop being host-bound (tools/host_overhead.py). ROCm replays a graph's
        cross-stream edges as barrier packets, which costs the long buckets the overlap of the
        weight-gradient side stream; with ``step_graphs="auto"`` each shape therefore compares
        the device time of its first two replays (events, queried when done: no host
        synchronisation) with the host enqueue time of its eager warm-up steps and keeps the
        graph only when the eager step is host-bound (``graph_modes``: mode, eager host ms,
        replay ms). Both paths give bitwise the same step. All shapes share one memory pool
        (replays never overlap, and each graph's outputs stay referenced)."""
        key = self.graph_key(batch)
        width = key[-1]
        st = self._shapes.get(key)
        if st is None:
            st = self._shapes[key] = _ShapeState()
        if st.mode == "eager" or (st.mode is None and st.seen < self.graph_warmup):
            st.seen += 1
            b = dict(batch)
            b["labels"] = self._pad_labels(batch["labels"], width)
            t0 = _clock()
            loss = self._body(b, lr_t, keep)
            st.host_s.append(_clock() - t0)
            return loss
        if st.graph is None:
            st.graph = self._capture(batch, width)
            if self.step_graphs != "auto":
                st.mode = "graph"
        if st.mode == "graph":
            return self._replay(st.graph, batch, width, lr_t, keep)
        # auto, undecided: replay between two events; decide once two replays have completed
        # (queried, never waited for): keep the graph when its device time beats the eager
        # step's host enqueue time — an eager step cannot finish faster than the host issues
        # it, while a GPU-bound eager step keeps the side-stream overlap a replay loses
        done = [(a, b) for a, b in st.spans if b.query()]
        if len(done) >= 2:
            tg = min(a.elapsed_time(b) for a, b in done)
            te = 1e3 * min(st.host_s)
            st.mode = "graph" if tg < 0.97 * te else "eager"
            self.graph_modes[key] = (st.mode, te, tg)
            st.spans = []
            if st.mode == "eager":
                st.graph = None
                if not any(o.graph is not None for o in self._shapes.values()):
                    # the last graph of the shared memory pool is gone, and with it the pool
                    # (PyTorch frees a private pool with its last graph): the next capture must
                    # not name the dead pool's handle (allocator assert at capture_begin)
                    self._graph_pool = None
                b = dict(batch)
                b["labels"] = self._pad_labels(batch["labels"], width)
                return self._body(b, lr_t, keep)
            return self._replay(st.graph, batch, width, lr_t, keep)
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        loss = self._replay(st.graph, batch, width, lr_t, keep, events=(a, b))
        st.spans.append((a, b))
        return loss

    def _state_ptrs(self) -> tuple:
        """Addresses of the buffers a captured step reads and writes in place (weights,
        gradients, bf16 shadows, Adam moments, EMA): a replay after any of them was re-allocated
        would write freed memory."""
        ts = (self.arena.flat, self.arena.grad, getattr(self.arena, "p16", None), self.opt.m, self.opt.v,
              self.opt.ema)
        return tuple(t.data_ptr() if t is not None else 0 for t in ts)

    def _replay(self, g: "_StepGraph", batch: Dict[str, torch.Tensor], width: int, lr_t: float,
                keep: float, events=None) -> torch.Tensor:
        if g.ptrs != self._state_ptrs():
            raise RuntimeError("step graph captured on re-allocated training state: call Trainer.drop_graphs()")
        self.flush()           # a graph never carries or consumes an update across steps
        feats, labels = batch["feats"], batch["labels"]
        pairs = [(g.feats, feats), (g.seq_lens, batch["seq_lens"]), (g.label_lens, batch["label_lens"]),
                 (g.labels, labels)]
        if all(s.is_cuda and s.dtype == d.dtype and s.is_contiguous() for d, s in pairs):
            # the graph's inputs and the optimizer's step constants in ONE launch
            # (csrc/fill.hip multi_copy_kernel; labels narrower than the captured width zero-padded)
            _ext.ext().multi_copy([g.feats.view(-1), g.seq_lens, g.label_lens, g.labels],
                                  [feats.reshape(-1), batch["seq_lens"], batch["label_lens"], labels],
                                  self.opt.hyper, [lr_t, keep])
        else:
            g.feats.copy_(feats, non_blocking=True)
            g.seq_lens.copy_(batch["seq_lens"], non_blocking=True)
            g.label_lens.copy_(batch["label_lens"], non_blocking=True)
            if labels.shape[1] == width:
                g.labels.copy_(labels, non_blocking=True)
            else:
                g.labels[:, labels.shape[1]:].zero_()
                g.labels[:, :labels.shape[1]].copy_(labels, non_blocking=True)
            self.opt.load_hyper(lr_t, keep)
        if events is not None:
            events[0].record()
        g.graph.replay()
        if events is not None:
            events[1].record()
        return g.loss.clone()

    def _capture(self, batch: Dict[str, torch.Tensor], width: int) -> "_StepGraph":
        dev = self.arena.flat.device
        self.flush()           # never capture the previous step's carried update into the graph
        static = {
            "feats": batch["feats"].clone(),
            "seq_lens": batch["seq_lens"].clone(),
            "labels": self._pad_labels(batch["labels"], width).clone(),
            "label_lens": batch["label_lens"].clone(),
        }
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        graph = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(dev)
        self.opt.device_hyper = True
        sch = self.arena.wgrad
        sch.single_stream = _GRAPH_SINGLE_STREAM
        try:
            # thread_local: the train driver's prefetch thread may pin / copy while we capture
            with torch.cuda.graph(graph, pool=self._graph_pool, capture_error_mode="thread_local"):
                loss = self._body(static, 0.0, 0.0)
        finally:
            self.opt.device_hyper = False
            sch.single_stream = False
        return _StepGraph(graph, static["feats"], static["seq_lens"], static["labels"], static["label_lens"], loss,
                          self._state_ptrs())

    def drop_graphs(self) -> None:
        """Forget every captured step (after anything that re-allocates the arena, optimizer
        state or model buffers the graphs were captured with)."""
        self._shapes.clear()
        self.graph_modes.clear()

    @property
    def _graphs(self) -> Dict[tuple, "_StepGraph"]:
        """Captured step graphs by shape key."""
        return {k: st.graph for k, st in self._shapes.items() if st.graph is not None}

    def _body(self, batch: Dict[str, torch.Tensor], lr_t: float, keep: float) -> torch.Tensor:
        """Forward, loss, backward and the optimizer update with a prepared (lr_t, keep): every
        launch of a training step and no host synchronisation (capturable)."""
        model = self.model
        model.train()
        self.arena.ensure_bf16()
        # the HIP engine delivers every gradient through the arena (first write overwrites),
        # so the per-step memset of the whole gradient buffer is skipped
        lazy = model.engine == "hip"
        if self.bucketer.enabled and lazy and self.arena.flat.is_cuda:
            # data parallel: sequences of < _PARTIAL_MIN_T recurrence steps take the single-device
            # schedule (every weight gradient in one grouped launch after the last BPTT, the
            # buckets' collectives behind it): their backward is too short for per-layer
            # overlap to pay for the capped beside grids (100 frames: 3.35 -> see
            # profiles/r6_dp.md); longer ones keep the per-layer GEMMs beside the BPTTs
            self.arena.wgrad.set_deferral(not _long_sequence(batch))
        self.arena.wgrad.discard()
        self.arena.zero_grad(lazy=lazy)
        with _CTC.loss_watch(self.watch) as lw:
            loss = model.forward_loss(batch["feats"], batch["seq_lens"], batch["labels"], batch["label_lens"])
        # a carried update whose weights no fused op awaited (another model path) completes
        # here, before backward writes this step's gradients over the ones it reads
        self.arena.settle_updates()
        if not lw.consumed:
            self.watch.update(loss)
        # a cached device 1.0 as the backward seed: autograd would launch a fill for ones_like
        one = self._seed.get((loss.device, loss.dtype))
        if one is None:
            one = self._seed[(loss.device, loss.dtype)] = torch.ones((), device=loss.device, dtype=loss.dtype)
        gscale = 1.0 / self.world
        per_bucket = self.bucketer.enabled and self.nan_policy != "skip" and self.per_bucket_update
        # (sequences of >= _PARTIAL_MIN_T recurrence steps only: beside a short recurrence the
        # carried ranges, capped to its idle CUs, outlast it and the projections wait for them)
        dp_carry = (per_bucket and self.defer_update and self.arena.flat.is_cuda and self._layer_first and
                    not torch.cuda.is_current_stream_capturing() and
                    _long_sequence(batch))
        if per_bucket:
            # DP-native ordering: each gradient bucket's Adam + EMA range runs on the
            # bucketer's ordering stream right behind its all-reduce (bitwise the same update);
            # with defer_update, the head's and upper layers' buckets carry theirs into the next
            # forward (GradBucketer carry_hi)
            up = self.upper_range(1) if dp_carry else None
            self.bucketer.set_optimizer(lambda lo, hi: self.opt.apply_range(lo, hi, lr_t, keep, gscale,
                                                                            max_grid=_BUCKET_GRID),
                                        carry_hi=up[0] if up else 0)
        early = (not per_bucket and self.nan_policy != "skip" and self._early_split > 0 and lazy and
                 self.arena.wgrad.grouped and self.arena.wgrad.defer_input)
        carry = early and self.defer_update and not torch.cuda.is_current_stream_capturing()
        carried = [0]
        carried_du = {}
        self.arena.wgrad.carry_du = carry and _CARRY_DU
        if early:
            # single device: the FC head's and recurrent stack's Adam + EMA range runs on the
            # weight-gradient stream right after the grouped tail GEMMs, beside the conv
            # front-end's backward (WgradScheduler.set_early_update); the front-end's range after
            split, sch = self._early_split, self.arena.wgrad
            if _FUSED_OPT:
                tensors, consts = self.opt.fused_constants(lr_t, keep, gscale)
                sch.set_fused_update(self.arena, tensors, consts, store_g=self.keep_grads)
            self.arena.wgrad.set_early_update(
                lambda: self.opt.apply_excluding(sch.early_upper_hi if sch.early_upper_done else 0, split,
                                                 sch.fused_ranges, lr_t, keep, gscale,
                                                 max_grid=_LOWER_GRID if sch.early_upper_done else _EARLY_GRID),
                self._early_params)
            if self._layer_first and _EARLY_UPPER:
                # the head and the layers whose weight gradients ran beside the BPTT (not in the
                # grouped tail launch): their range goes out beside the next BPTT, on a capped grid,
                # or (defer_update) beside the next step's first recurrence
                if carry:
                    def upper(hi, grid):
                        carried[0] = hi
                        carried_du.update(self.arena.wgrad.take_carried_du())
                else:
                    def upper(hi, grid):
                        self.opt.apply_range(0, hi, lr_t, keep, gscale, max_grid=grid)
                sch.set_early_upper(self.upper_range, upper, _UPPER_GRID)
        loss.backward(one)
        self.arena.wgrad.join()
        self.arena.wgrad.carry_du = False
        if lazy:
            self.arena.zero_unwritten()
        with TR.phase(TR.ALLREDUCE):
            carried_buckets = self.bucketer.take_carried() if per_bucket else []
            self.bucketer.finish()
            carried_buckets += self.bucketer.take_carried() if per_bucket else []
        if carried_buckets:
            self._carry_buckets(carried_buckets, lr_t, keep, gscale)
        if early:
            with TR.phase(TR.EMA):
                # the upper range [0, usplit) may have been applied beside layer 0's BPTT even
                # when the lower early range was skipped: never apply it twice
                sch = self.arena.wgrad
                lo = split if sch.early_done else (sch.early_upper_hi if sch.early_upper_done else 0)
                self.opt.apply_excluding(lo, self.arena.numel, sch.fused_ranges, lr_t, keep, gscale)
            if carried[0] > 0:
                self._carry_update(carried[0], lr_t, keep, gscale, carried_du)
        elif not per_bucket:
            skip = None
            if self.nan_policy == "skip":
                _, skip = self.opt.grad_norm_and_finite(gscale)
                self.last_skip = skip
            with TR.phase(TR.EMA):
                self.opt.apply_range(0, self.arena.numel, lr_t, keep, gscale, skip)
        return loss.detach()

    def first_nonfinite_step(self) -> Optional[int]:
        """Global step of the first non-finite loss so far (None if none). Reads one device
        word: call where the host synchronises anyway."""
        return self.watch.first_bad_step()

    def update_loss_ema(self, loss_value: float, decay: float = 0.9) -> float:
        """tf.train.ExponentialMovingAverage(0.9) of the loss (src/deepSpeech_train.py:175-188)."""
        if self.loss_ema is None:
            self.loss_ema = loss_value
        else:
            self.loss_ema = decay * self.loss_ema + (1 - decay) * loss_value
        return self.loss_ema

    # ---- EMA weights for eval (reference evaluates the shadow variables) -------------
    def swap_ema(self) -> None:
        self.flush()
        if self.opt.ema is None:
            return
        tmp = self.arena.flat.clone()
        self.arena.flat.copy_(self.opt.ema)
        self.opt.ema.copy_(tmp)
        self.arena.mark_dirty()
