"""Flat parameter arena + fused Adam/EMA optimizer.

Reference: tf.train.AdamOptimizer(lr) + ExponentialMovingAverage(decay, global_step)
(src/deepSpeech_train.py:430,457-465) with the staircase exponential-decay LR of
:231-250.

All trainable parameters live as views in ONE contiguous fp32 buffer (``flat``) with
gradients as views in ``grad``. That makes
  * the whole optimizer step one streaming kernel (csrc/optim.hip) on the GPU,
  * gradient all-reduce buckets plain contiguous slices (parallel/grad_sync.py),
  * zero_grad one memset.
The arena is laid out in REVERSE parameter registration order, which is the order
backward produces gradients (FC first, conv1 last), so early buckets fill first.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional, Tuple

import torch
import torch.nn as nn

from . import _ext


class ParamArena:
    """Flat fp32 master weights + fp32 gradients (+ optional bf16 compute shadows).

    Layout: ``groups`` (default: the model's ``arena_groups()`` if it has one, otherwise
    one group per parameter in reverse registration order). Members of a group are
    packed back to back with NO padding, so e.g. ``[W_fw; W_bw]`` of a bidirectional
    layer is one contiguous ``[2*G*H, in]`` matrix in all three buffers (the input
    projection of both directions is then ONE GEMM with no concat); groups start on
    ``align``-element (256 B) boundaries.

    Fused HIP ops write weight gradients straight into ``p.main_grad`` (a view of
    ``grad``) in fp32 and report them with :meth:`grad_done` — no bf16->fp32 casts, no
    autograd accumulation kernels — and read the weights from ``p.bf16`` (a view of the
    shadow that the fused optimizer rewrites after every update).
    """

    def __init__(self, model: nn.Module, align: int = 64, groups=None, bf16_shadow: bool = False):
        if groups is None and hasattr(model, "arena_groups"):
            groups = model.arena_groups()
        if groups is None:
            named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
            groups = [[np_] for np_ in reversed(named)]
        groups = [[(n, p) for n, p in g if p.requires_grad] for g in groups]
        groups = [g for g in groups if g]
        seen = {id(p) for g in groups for _, p in g}
        want = {id(p) for _, p in model.named_parameters() if p.requires_grad}
        if seen != want or sum(len(g) for g in groups) != len(want):
            raise ValueError("arena groups must cover every trainable parameter exactly once")
        self.names: List[str] = [n for g in groups for n, _ in g]
        self.params: List[nn.Parameter] = [p for g in groups for _, p in g]
        dev = self.params[0].device
        self.offsets: List[Tuple[int, int]] = []
        off = 0
        for g in groups:
            for _, p in g:
                self.offsets.append((off, p.numel()))
                off += p.numel()
            off = -(-off // align) * align
        self.numel = off
        self.flat = torch.zeros(off, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(off, device=dev, dtype=torch.float32)
        self.p16 = torch.zeros(off, device=dev, dtype=torch.bfloat16) if bf16_shadow else None
        self._index = {}
        self._ready_cbs = []
        # where / when this arena's weight-gradient GEMMs run (side stream, deferral, queues):
        # per arena, so independent models in one process never share that state
        from .rnn import WgradScheduler
        self.wgrad = WgradScheduler()
        # per-parameter "gradient written" events (enabled by the DP bucketer): recorded on
        # whatever stream enqueued the gradient write, so a collective waits for exactly
        # the producers of its bucket instead of joining whole streams
        self._ready_events: Optional[List[torch.cuda.Event]] = None
        self._written = set()
        self._held = set()         # gradients a queued (deferred) GEMM will report
        self._known_zero = set()
        for i, (p, (o, n)) in enumerate(zip(self.params, self.offsets)):
            self.flat[o:o + n].copy_(p.data.reshape(-1).float())
            p.data = self.flat[o:o + n].view_as(p)
            p.grad = self.grad[o:o + n].view_as(p)
            self._index[id(p)] = i
            if bf16_shadow:
                p.main_grad = self.grad[o:o + n].view_as(p)
                p.bf16 = self.p16[o:o + n].view_as(p)
                p._ds2_arena = self
        self._dirty = True
        self.ensure_bf16()
        # optimizer update carried into the next step (Trainer defer_update): chunks not issued
        # yet ([(fn, params)] in the order the next forward reads them), and the events of the
        # issued ones that readers of their weights still have to wait for
        self._pending_chunks: List[tuple] = []
        self._update_events: Dict[int, "torch.cuda.Event"] = {}
        self._event_pool: List["torch.cuda.Event"] = []
        self._event_next = 0
        self._gemm_beside = False          # a carried weight-gradient GEMM went out this step

    # ---- deferred optimizer update ----------------------------------------------------
    def set_pending_update(self, chunks) -> None:
        """Carry an optimizer update into the next forward: ``chunks`` = [(fn, params)] in the
        order the next forward reads their weights; ``fn(grid)`` enqueues one chunk's update on
        the current stream (grid: block cap, 0 = uncapped)."""
        self._pending_chunks = list(chunks)
        self._event_next = 0

    def has_pending_update(self) -> bool:
        return bool(self._pending_chunks) or bool(self._update_events)

    def _event(self) -> "torch.cuda.Event":
        if self._event_next == len(self._event_pool):
            self._event_pool.append(torch.cuda.Event())
        ev = self._event_pool[self._event_next]
        self._event_next += 1
        return ev

    def issue_pending_update(self, grid: int = 0, count: int = 1, gate=None) -> None:
        """Enqueue the next ``count`` chunks of the carried update on the weight-gradient side
        stream, behind everything the current stream has enqueued (a recurrent layer's
        projection): each then runs on the CUs that layer's persistent recurrence leaves idle,
        and the reader of its weights waits only for its own chunk (:meth:`await_params`).
        Chunks without parameters (a carried weight-gradient GEMM of the layer above) go out
        with the chunk before them. ``gate()``, if given, is enqueued on the side stream first
        (ops/rnn.py _gate: wait until the recurrence beside which the chunk runs is resident)."""
        if not self._pending_chunks:
            return
        while count < len(self._pending_chunks) and not self._pending_chunks[count][1]:
            count += 1
        take, self._pending_chunks = self._pending_chunks[:count], self._pending_chunks[count:]
        dev = self.flat.device
        side = self.wgrad.stream(dev) if dev.type == "cuda" else None
        if side is None:
            for fn, _ in take:
                fn(0)
            return
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            if gate is not None:
                gate()
            for fn, params in take:
                fn(grid)
                if not params:
                    self._gemm_beside = True
                    continue
                ev = self._event()
                ev.record(side)
                for p in params:
                    self._update_events[id(p)] = ev

    def carried_gemm_beside(self) -> bool:
        """True once a carried weight-gradient GEMM was issued beside this step's forward (it
        may still hold the CUs the recurrence left idle; ops/rnn.py _proj_grid)."""
        return self._gemm_beside

    def await_params(self, *params) -> None:
        """Make the current stream wait for the carried update of ``params`` (no-op when none
        is in flight); chunks holding any of them that were not issued yet are issued first.
        Every fused op that reads arena weights calls this before it reads them."""
        if not (self._update_events or self._pending_chunks):
            return
        ids = {id(p) for p in params if p is not None}
        last = -1
        for j, (_, ps) in enumerate(self._pending_chunks):
            if any(id(p) in ids for p in ps):
                last = j
        if last >= 0:
            self.issue_pending_update(0, last + 1)
        cur = None
        waited = set()
        for i in ids:
            ev = self._update_events.pop(i, None)
            if ev is not None and id(ev) not in waited:
                if cur is None:
                    cur = torch.cuda.current_stream(self.flat.device)
                cur.wait_event(ev)
                waited.add(id(ev))

    def settle_updates(self) -> None:
        """Complete the carried update from the current stream's point of view: issue the
        chunks nothing issued yet here, and wait for every chunk still in flight. After this
        the master weights, bf16 shadows, Adam moments and EMA are those of the last step."""
        take, self._pending_chunks = self._pending_chunks, []
        self._gemm_beside = False
        for fn, _ in take:
            fn(0)
        if self._update_events:
            cur = torch.cuda.current_stream(self.flat.device)
            for ev in {id(e): e for e in self._update_events.values()}.values():
                cur.wait_event(ev)
            self._update_events.clear()

    # ---- bf16 shadow ------------------------------------------------------------
    def mark_dirty(self) -> None:
        """Call after changing master weights outside the fused optimizer (restore, EMA swap)."""
        self._dirty = True

    def ensure_bf16(self) -> None:
        if self.p16 is not None and self._dirty:
            self.p16.copy_(self.flat)
        self._dirty = False

    def group_view(self, params, buf: str = "p16") -> Optional[torch.Tensor]:
        """Contiguous 1-D view of ``buf`` spanning ``params`` if they are packed back to back
        in this order, else None."""
        idx = [self._index.get(id(p)) for p in params]
        if any(i is None for i in idx):
            return None
        start = self.offsets[idx[0]][0]
        pos = start
        for i in idx:
            o, n = self.offsets[i]
            if o != pos:
                return None
            pos = o + n
        b = {"p16": self.p16, "grad": self.grad, "flat": self.flat}[buf]
        return None if b is None else b[start:pos]

    # ---- gradients ----------------------------------------------------------------
    def zero_grad(self, lazy: bool = False) -> None:
        """Start a new gradient step. ``lazy``: skip the memset of the whole arena — valid
        when every gradient is delivered by the fused ops (first write overwrites, later
        writes accumulate); call :meth:`zero_unwritten` before anything reads the arena."""
        if not lazy:
            self.grad.zero_()
        self._written.clear()
        self._held.clear()
        if self._ready_events is not None:
            self._ready_next = 0
            self._ready_events = [None] * len(self.params)
        # re-attach in case an op replaced a .grad (e.g. set_to_none elsewhere)
        for p, (o, n) in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + n].data_ptr():
                p.grad = self.grad[o:o + n].view_as(p)

    def zero_unwritten(self) -> None:
        """Zero the gradient of every parameter no op has written this step (lazy zeroing)."""
        for p, (o, n) in zip(self.params, self.offsets):
            if id(p) not in self._written:
                self.grad[o:o + n].zero_()

    def known_zero(self, p) -> bool:
        """True if ``p``'s gradient slice holds zeros that no op has overwritten since
        :meth:`set_known_zero` (a structurally-zero gradient needs no per-step memset)."""
        return id(p) in self._known_zero

    def set_known_zero(self, p) -> None:
        self._known_zero.add(id(p))

    def hold_report(self, *params) -> None:
        """These gradients are produced by a GEMM queued for later (weight-gradient deferral):
        autograd's post-accumulate hook, which fires when the op returns, must not count them
        as ready; the queued GEMM reports them (:meth:`grad_done`) once it is enqueued."""
        for p in params:
            if p is not None:
                self._held.add(id(p))

    def held(self, p) -> bool:
        return id(p) in self._held

    def mark_written(self, *params) -> None:
        """Count these gradients as produced this step without reporting them (a GEMM carried
        into the next step writes them; lazy zeroing must not clear their slots meanwhile)."""
        for p in params:
            if p is not None:
                self._written.add(id(p))
                self._known_zero.discard(id(p))

    def first_write(self, p) -> bool:
        """True if ``p``'s gradient has not been written yet this step (fused ops then
        overwrite instead of accumulate)."""
        return id(p) not in self._written

    def grad_done(self, *params) -> None:
        """Report gradients written straight into ``main_grad`` (fires bucket hooks). Call
        right after enqueueing the write, on the stream that carries it."""
        idx = []
        for p in params:
            if p is None:
                continue
            self._written.add(id(p))
            self._known_zero.discard(id(p))
            idx.append(self._index[id(p)])
        # one ready event for the whole call (the same enqueued work produced them all)
        self.record_ready(*idx)
        for i in idx:
            for cb in self._ready_cbs:
                cb(i)

    def on_grad_ready(self, cb) -> None:
        self._ready_cbs.append(cb)

    def enable_ready_events(self) -> None:
        if self.grad.is_cuda and self._ready_events is None:
            # per parameter: the event of the record that covered it this step, drawn from a pool
            # reused every step (a wait enqueued earlier keeps the record it saw)
            self._ready_events = [None] * len(self.params)
            self._ready_pool = []
            self._ready_next = 0
            self._ready_seq = 0
            self._ready_at = [(0, 0)] * len(self.params)   # (record order, stream) per parameter

    def ready_events_covering(self, idx) -> list:
        """The fewest ready events whose completion implies every parameter in ``idx`` is
        written: per recording stream, the latest-recorded member (streams run in order)."""
        last = {}
        for i in idx:
            if self._ready_events[i] is None:      # marked written, produced by a later launch
                continue
            seq, st = self._ready_at[i]
            if st not in last or seq > last[st][0]:
                last[st] = (seq, i)
        return [self._ready_events[i] for _, i in last.values()]

    def record_ready(self, *idx: int) -> None:
        """Mark the gradients of parameters ``idx`` as produced by the work enqueued so far on
        the current stream: ONE event record for all of them (each record is a marker packet
        in the stream's queue)."""
        if self._ready_events is None or not idx:
            return
        if self._ready_next == len(self._ready_pool):
            self._ready_pool.append(torch.cuda.Event())
        ev = self._ready_pool[self._ready_next]
        self._ready_next += 1
        ev.record()
        self._ready_seq += 1
        at = (self._ready_seq, torch.cuda.current_stream(self.grad.device).cuda_stream)
        for i in idx:
            self._ready_events[i] = ev
            self._ready_at[i] = at

    def ready_event(self, i: int) -> Optional["torch.cuda.Event"]:
        return self._ready_events[i] if self._ready_events is not None else None

    def views(self, buf: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {n: buf[o:o + c].view_as(p) for n, p, (o, c) in zip(self.names, self.params, self.offsets)}

    def param_range(self, name: str) -> Tuple[int, int]:
        i = self.names.index(name)
        return self.offsets[i]


def arena_of(p) -> Optional["ParamArena"]:
    return getattr(p, "_ds2_arena", None) if p is not None else None


def emit_grad(p, g: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """Deliver gradient ``g`` of parameter ``p`` from a fused op's backward.

    Arena-managed parameter: written (first producer this step) or accumulated into
    ``p.main_grad`` in fp32, reported ready, and None is returned to autograd.
    Otherwise ``g`` is returned for autograd to accumulate as usual."""
    if g is None or p is None:
        return None
    a = arena_of(p)
    if a is None:
        return g.to(p.dtype) if g.dtype != p.dtype else g
    mg = p.main_grad
    if a.first_write(p):
        mg.copy_(g.view_as(mg))
    else:
        mg.add_(g.view_as(mg))
    a.grad_done(p)
    return None


def mm_into(p, a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
            max_grid: int = 0) -> Optional[torch.Tensor]:
    """Weight gradient ``a @ b`` (bf16 operands, fp32 accumulation) for parameter ``p``.

    Arena-managed: the GEMM writes fp32 straight into ``p.main_grad`` (``out`` may name a
    larger group view of the gradient arena covering several packed parameters) and
    returns None; otherwise returns the fp32 product."""
    from . import gemm as G
    arena = arena_of(p)
    if arena is None:
        if G.enabled("wgrad") and a.is_cuda:
            r = torch.empty(a.shape[0], b.shape[1], device=a.device, dtype=torch.float32)
            if G.matmul(a, b, r):
                return r
        try:
            return torch.mm(a, b, out_dtype=torch.float32)
        except (RuntimeError, TypeError):
            return torch.mm(a.float(), b.float())
    dst = out if out is not None else p.main_grad.view(a.shape[0], b.shape[1])
    if G.enabled("wgrad") and G.matmul(a, b, dst, accumulate=not arena.first_write(p), max_grid=max_grid):
        return None
    if arena.first_write(p):
        try:
            torch.mm(a, b, out_dtype=torch.float32, out=dst)
        except (RuntimeError, TypeError):
            dst.copy_(torch.mm(a.float(), b.float()))
    else:
        dst.add_(torch.mm(a.float(), b.float()))
    return None


def exponential_decay(initial_lr: float, step: int, decay_steps: int, decay_rate: float,
                      staircase: bool = True) -> float:
    """tf.train.exponential_decay (src/deepSpeech_train.py:245-249)."""
    p = step / float(max(1, decay_steps))
    if staircase:
        p = math.floor(p)
    return initial_lr * (decay_rate ** p)


class FusedAdamEMA:
    """Adam (TF epsilon-hat form) + weight EMA over a ParamArena."""

    def __init__(self, arena: ParamArena, lr: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 ema_decay: Optional[float] = 0.9999, bf16_copy: bool = False):
        self.arena = arena
        self.lr = lr
        self.b1, self.b2 = betas
        self.eps = eps
        self.ema_decay = ema_decay
        dev = arena.flat.device
        self.m = torch.zeros_like(arena.flat)
        self.v = torch.zeros_like(arena.flat)
        self.ema = arena.flat.clone() if ema_decay is not None else None
        self.p16 = arena.p16 if arena.p16 is not None else (
            torch.empty(arena.numel, device=dev, dtype=torch.bfloat16) if bf16_copy else None)
        self.t = 0          # number of applied updates (Adam bias-correction power)
        self.use_hip = dev.type == "cuda"
        if self.p16 is not None and self.use_hip and arena.p16 is None:
            _ext.ext().cast_bf16(arena.flat, self.p16)
        self._norm_part = None
        self._bad = None
        # device {lr_t, ema_keep} read by the kernels instead of their scalar arguments while
        # ``device_hyper`` is set (a captured step: Trainer step graphs); load_hyper() writes it
        self.hyper = torch.zeros(2, device=dev, dtype=torch.float32) if self.use_hip else None
        self.device_hyper = False

    def load_hyper(self, lr_t: float, keep: float) -> None:
        """Stage this update's (lr_t, ema_keep) into :attr:`hyper` on the current stream (an
        async copy from a fresh pinned host tensor, which the caching host allocator keeps
        alive until the copy has run). Both are rounded to fp32 exactly as the scalar kernel
        arguments are, so a replayed update is bitwise the eager one."""
        h = torch.tensor([lr_t, keep], dtype=torch.float32).pin_memory()
        self.hyper.copy_(h, non_blocking=True)

    def _hyper_arg(self):
        return self.hyper if self.device_hyper else None

    # TF ExponentialMovingAverage with num_updates: min(decay, (1+n)/(10+n))
    def ema_keep(self, global_step: int) -> float:
        return min(self.ema_decay, (1.0 + global_step) / (10.0 + global_step))

    def grad_norm_and_finite(self, gscale: float = 1.0) -> Tuple[torch.Tensor, torch.Tensor]:
        """(||g||_2, non-finite flag) as device tensors (no host sync)."""
        g = self.arena.grad
        if self.use_hip:
            C = _ext.ext()
            if self._norm_part is None:
                nb = int(C.grad_norm_blocks(g.numel()))
                self._norm_part = torch.empty(nb, device=g.device, dtype=torch.float32)
                self._bad = torch.zeros(1, device=g.device, dtype=torch.int32)
            self._bad.zero_()
            C.grad_norm(g, gscale, self._norm_part, self._bad)
            return self._norm_part.sum().sqrt(), self._bad
        gg = g * gscale
        return gg.norm(), (~torch.isfinite(gg)).any().to(torch.int32).view(1)

    def prepare(self, lr: float, global_step: int) -> Tuple[float, float]:
        """Advance the Adam step count; (lr_t, ema_keep) of this update."""
        self.t += 1
        lr_t = lr * math.sqrt(1.0 - self.b2 ** self.t) / (1.0 - self.b1 ** self.t)
        keep = self.ema_keep(global_step) if self.ema is not None else 0.0
        return lr_t, keep

    @torch.no_grad()
    def apply_range(self, lo: int, hi: int, lr_t: float, keep: float, gscale: float = 1.0,
                    skip_flag: Optional[torch.Tensor] = None, max_grid: int = 0, lds_reserve: int = 0) -> None:
        """Adam + EMA of arena elements [lo, hi) with a prepared (lr_t, keep), on the current
        stream. Every element's update is independent and rounds the same way whatever the
        launch split, so ranges compose bitwise into the whole-arena update (the DP bucketer
        issues one range per gradient bucket)."""
        if hi <= lo:
            return
        a = self.arena
        sl = slice(lo, hi)
        if not self.use_hip:
            if skip_flag is not None and int(skip_flag.item()) != 0:
                return
            p, m, v = a.flat[sl], self.m[sl], self.v[sl]
            g = a.grad[sl] * gscale
            m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            p.sub_(lr_t * m / (v.sqrt() + self.eps))
            if self.ema is not None:
                e = self.ema[sl]
                e.copy_(p + keep * (e - p))
            if self.p16 is not None:
                self.p16[sl].copy_(p)
            return
        _ext.ext().adam_ema(a.flat[sl], a.grad[sl], self.m[sl], self.v[sl],
                            self.ema[sl] if self.ema is not None else None,
                            self.p16[sl] if self.p16 is not None else None,
                            lr_t, self.b1, self.b2, self.eps, gscale, keep, skip_flag, int(max_grid),
                            self._hyper_arg(), int(lds_reserve))

    @torch.no_grad()
    def apply_excluding(self, lo: int, hi: int, exclude, lr_t: float, keep: float, gscale: float = 1.0,
                        max_grid: int = 0) -> None:
        """Adam + EMA of arena elements [lo, hi) except the ``exclude`` ranges (already updated
        this step, e.g. by the grouped weight-gradient GEMM's fused epilogue): the remaining
        intervals in one launch (csrc/optim.hip adam_ema_ranges) when they fit its table."""
        todo, pos = [], lo
        for a, b in sorted(exclude):
            a, b = max(a, lo), min(b, hi)
            if b <= a:
                continue
            if a > pos:
                todo.append((pos, a))
            pos = max(pos, b)
        if pos < hi:
            todo.append((pos, hi))
        if not todo:
            return
        if self.use_hip and len(todo) > 1 and len(todo) <= 64 and all(a % 4 == 0 and b % 4 == 0 for a, b in todo):
            ar = self.arena
            _ext.ext().adam_ema_ranges(ar.flat, ar.grad, self.m, self.v, self.ema, self.p16,
                                       [x for r in todo for x in r], lr_t, self.b1, self.b2, self.eps, gscale, keep,
                                       self._hyper_arg())
            return
        for a, b in todo:
            self.apply_range(a, b, lr_t, keep, gscale, max_grid=max_grid)

    def fused_constants(self, lr_t: float, keep: float, gscale: float = 1.0):
        """(tensors, constants) of a fused-epilogue update (gemm.gemm8_group ``opt``)."""
        return ([self.arena.flat, self.m, self.v, self.ema, self.p16, self.arena.grad],
                [lr_t, self.b1, self.b2, self.eps, gscale, keep if self.ema is not None else 0.0])

    @torch.no_grad()
    def step(self, lr: float, global_step: int, gscale: float = 1.0,
             skip_flag: Optional[torch.Tensor] = None) -> None:
        """One Adam + EMA update of the whole arena."""
        lr_t, keep = self.prepare(lr, global_step)
        self.apply_range(0, self.arena.numel, lr_t, keep, gscale, skip_flag)

    def state_dict(self) -> Dict[str, object]:
        return {"m": self.m, "v": self.v, "ema": self.ema, "t": self.t}

    def load_state_dict(self, sd: Dict[str, object]) -> None:
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        if self.ema is not None and sd.get("ema") is not None:
            self.ema.copy_(sd["ema"])
        self.t = int(sd["t"])
