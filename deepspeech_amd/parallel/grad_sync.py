"""Bucketed gradient all-reduce overlapped with backward.

MI355X-first choices:
  * gradients already live in one flat fp32 arena (ops/optim.py), laid out in the order
    backward produces them, so a bucket is a contiguous slice: no pack/unpack copies;
  * a bucket is launched (async RCCL all-reduce) from a post-accumulate-grad hook the
    moment its last parameter's gradient lands, while BPTT of earlier layers continues.
    The recurrent layers finish their weight gradients one layer at a time, so bucket
    boundaries are snapped to layer (parameter) boundaries;
  * default bucket size 32 MB: each all-reduce is long enough to run at xGMI link rate
    (ring algorithms are per-link bound on the point-to-point mesh) but small enough that
    the last bucket (conv layers, ~0.1 MB) adds almost nothing after backward ends;
  * optional bf16 compression halves bytes on the links (sum in bf16, scaled in fp32
    afterwards by the optimizer's gscale = 1/world).
  * stream ordering without joins: every gradient write records an event on the stream
    that enqueued it (main stream for dx-adjacent work, the weight-gradient side stream
    for dW/dU), and a bucket's collective is issued from a dedicated ordering stream that
    waits on exactly its members' events. The main stream (running the next layer's
    BPTT) never waits on the side stream mid-backward; it waits for the collectives only
    in finish(), before the optimizer.
The SUM is averaged by the optimizer (``gscale``), so no extra division kernel runs.

Per-bucket optimizer (DP-native ordering, :meth:`GradBucketer.set_optimizer`): instead of
one Adam over the whole arena after the last collective, each bucket's Adam + EMA range is
issued on the ordering stream right behind its all-reduce, so the update of the early
buckets (FC head, top layers) streams while the lower layers' BPTT and the remaining
collectives run, and only the last bucket's range is left after backward. Every arena
element's update is independent and rounded the same way whatever the launch split, so
the result is bitwise the whole-arena update. A bucket's range is issued right behind its
own collective, ordered after everything the main stream has enqueued when the bucket
becomes ready. That is safe because every fused op enqueues its weight-reading work (the
recurrence, dx / dgrad GEMMs, the W^T shadow copies) on the main stream BEFORE it reports a
gradient of those weights, so when the last member of a bucket reports, every reader of the
bucket's weights is already ahead of the recorded point (ops/rnn.py FusedBiLayer._backward,
ops/frontend.py FusedHead._backward). (Round 3 issued a range only when the NEXT bucket
became ready, which held each update ~1 ms behind its all-reduce: profiles/r3_dp_buckets.md.)
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


class GradBucketer:
    def __init__(self, arena, bucket_mb: float = 32.0, compress_bf16: bool = False,
                 process_group=None, world_size: Optional[int] = None, force: bool = False,
                 split_after=()):
        """force: run the bucketed collectives even at world size 1 (needs an initialised
        process group; measures the DP machinery's own overhead on one GPU). split_after:
        parameter names that also end a bucket (tests pin bucket layouts with it)."""
        self.arena = arena
        self.pg = process_group
        self.compress = compress_bf16
        # world_size given by the caller wins (a world_size=1 trainer inside an initialised
        # process group keeps its gradients local)
        self.world = (world_size if world_size is not None else
                      (dist.get_world_size(process_group) if dist.is_initialized() else 1))
        limit = int(bucket_mb * 1024 * 1024 / 4)
        # snap buckets to parameter boundaries, in arena (= gradient production) order
        self.buckets: List[Tuple[int, int, List[int]]] = []
        cur: List[int] = []
        start = None
        for i, (off, n) in enumerate(arena.offsets):
            if start is None:
                start = off
            cur.append(i)
            end = off + n
            if end - start >= limit or arena.names[i] in split_after:
                self.buckets.append((start, arena.offsets[cur[-1]][0] + arena.offsets[cur[-1]][1], cur))
                cur, start = [], None
        if cur:
            self.buckets.append((start, arena.offsets[cur[-1]][0] + arena.offsets[cur[-1]][1], cur))
        # extend each bucket to the next bucket's start so alignment padding is covered too
        fixed = []
        for bi, (s, e, idx) in enumerate(self.buckets):
            e2 = self.buckets[bi + 1][0] if bi + 1 < len(self.buckets) else arena.numel
            fixed.append((s, e2, idx))
        self.buckets = fixed
        self.param_bucket = {}
        for bi, (_, _, idx) in enumerate(self.buckets):
            for i in idx:
                self.param_bucket[i] = bi
        self._pending: List[int] = []
        self._launched: List[bool] = []
        self._works = []
        self._shadow: List[Optional[torch.Tensor]] = [None] * len(self.buckets)
        self._handles = []
        self._opt = None                   # per-bucket optimizer: fn(lo, hi) on the current stream
        self._opt_pending: List[int] = []  # buckets whose collective is issued, update not yet
        self._carry_hi = 0                 # buckets inside arena [0, carry_hi): update carried
        self._carried: List[Tuple[int, int, "torch.cuda.Event"]] = []
        self._main_stream = None
        self.enabled = self.world > 1 or (force and dist.is_initialized())
        self._order_stream = None
        if self.enabled:
            arena.enable_ready_events()
            if arena.grad.is_cuda:
                self._order_stream = torch.cuda.Stream(device=arena.grad.device)
            # autograd-accumulated grads fire the tensor hook; fused ops that write
            # main_grad directly report through the arena
            for i, p in enumerate(arena.params):
                self._handles.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
            if hasattr(arena, "on_grad_ready"):
                arena.on_grad_ready(self._ready)
        self.prepare()

    def _ready(self, i: int) -> None:
        b = self.param_bucket[i]
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._launch(b)

    def _make_hook(self, i: int):
        # autograd runs a parameter's post-accumulate hook even when the producing op
        # returned no gradient for it (the fused ops deliver theirs through the arena and
        # return None): count each parameter once per step, whichever path reports first
        def hook(p):
            if getattr(self.arena, "_held", None) and id(p) in self.arena._held:
                return               # a deferred GEMM reports it (ParamArena.hold_report)
            written = getattr(self.arena, "_written", None)
            if written is not None:
                if id(p) in written:
                    return
                written.add(id(p))
            # autograd accumulated this gradient on the current stream (the engine runs the
            # hook under the producing op's stream)
            self.arena.record_ready(i)
            self._ready(i)
        return hook

    def prepare(self) -> None:
        self._pending = [len(idx) for (_, _, idx) in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._works = []
        self._opt = None
        self._opt_pending = []
        self._carry_hi = 0

    def set_optimizer(self, fn, carry_hi: int = 0) -> None:
        """Apply ``fn(lo, hi)`` (an optimizer update of arena elements [lo, hi), enqueued on
        the current stream) to each bucket right behind its collective, for THIS step only
        (:meth:`finish` clears it). Call before backward, on the stream that runs it (the
        ranges wait for that stream's progress; a hook may fire on a side stream).

        ``carry_hi`` (GPU): buckets lying wholly inside arena [0, carry_hi) (the FC head and the
        recurrent layers >= 1) get no update here; an event behind each one's collective is kept
        instead (:meth:`take_carried`) and the Trainer applies their updates beside the next
        step's forward recurrences, as on one device (Trainer defer_update): the per-bucket
        ranges then no longer stream beside the BPTTs."""
        if self.enabled:
            self._opt = fn
            if self.arena.grad.is_cuda:
                self._main_stream = torch.cuda.current_stream(self.arena.grad.device)
                self._carry_hi = int(carry_hi)

    def capturable(self) -> bool:
        """True when this bucketer's collectives can be captured into a HIP graph (RCCL
        process group, GPU gradients; gloo runs its collectives on the host)."""
        if not (self.enabled and self.arena.grad.is_cuda and self._order_stream is not None):
            return False
        try:
            return dist.get_backend(self.pg) == "nccl"
        except (RuntimeError, ValueError):
            return False

    def take_carried(self) -> List[Tuple[int, int, "torch.cuda.Event"]]:
        """(lo, hi, event behind the collective) of the buckets whose update was carried."""
        c, self._carried = self._carried, []
        return c

    def _flush_updates(self) -> None:
        """Issue the pending buckets' optimizer ranges behind their collectives (ordering
        stream), after the main stream's work enqueued so far (see module docstring). The
        wait is an event the main stream records now: waiting on the stream object itself is
        the same marker, taken at this point of the main stream's queue."""
        if not self._opt_pending:
            return
        os_ = self._order_stream
        if os_ is not None:
            os_.wait_stream(self._main_stream)
        pend, self._opt_pending = self._opt_pending, []
        waits = dict(self._works)
        for b in pend:
            s, e, _ = self.buckets[b]
            if os_ is None:
                if waits[b] is not None:
                    waits[b].wait()
                if self.compress:
                    self.arena.grad[s:e].copy_(self._shadow[b])
                self._opt(s, e)
                continue
            with torch.cuda.stream(os_):
                if waits[b] is not None:
                    waits[b].wait()              # the ordering stream waits for the collective
                if self.compress:
                    self.arena.grad[s:e].copy_(self._shadow[b])
                if e <= self._carry_hi:
                    ev = torch.cuda.Event()
                    ev.record(os_)               # the reduced gradient is final here
                    self._carried.append((s, e, ev))
                else:
                    self._opt(s, e)

    def _launch(self, b: int) -> None:
        if self._launched[b]:
            return
        self._launched[b] = True
        s, e, idx = self.buckets[b]
        g = self.arena.grad[s:e]
        os_ = self._order_stream
        if os_ is None:
            self._works.append((b, self._collective(b, g)))
            if self._opt is not None:
                self._opt_pending.append(b)
                self._flush_updates()
            return
        # the collective (ProcessGroupNCCL waits on the CURRENT stream at issue time) is
        # issued from the ordering stream, which waits on each member's producer event:
        # gradients written on the side stream and on the main stream alike, nothing else
        # one wait per producing stream (its latest-recorded member): every queued wait is a
        # barrier packet the command processor handles in order, and they add up (measured
        # with the per-layer optimizer ranges: one wait per member cost ~0.2 ms/step)
        written = [i for i in idx if id(self.arena.params[i]) in self.arena._written]
        for ev in self.arena.ready_events_covering(written):
            os_.wait_event(ev)
        with torch.cuda.stream(os_):
            self._works.append((b, self._collective(b, g)))
        if self._opt is not None:
            self._opt_pending.append(b)
            self._flush_updates()                # this bucket's readers are enqueued already

    def _collective(self, b: int, g: torch.Tensor):
        # under HIP-graph capture (Trainer dp_graphs) the blocking form: the issuing (ordering)
        # stream itself is ordered behind the collective, and there is no Work to wait on. An
        # async_op collective issued from a side stream during capture crashes this image's
        # ProcessGroupNCCL at issue (tools/probe_rccl_graph.py: "async" / "side_async_norec"
        # segfault, "side_sync" / "main_async" / "sync" capture and replay correctly)
        capturing = g.is_cuda and torch.cuda.is_current_stream_capturing()
        t = g
        if self.compress:
            sh = self._shadow[b]
            if sh is None or sh.numel() != g.numel():
                sh = torch.empty(g.numel(), device=g.device, dtype=torch.bfloat16)
                self._shadow[b] = sh
            sh.copy_(g)
            t = sh
        if capturing:
            dist.all_reduce(t, group=self.pg)
            return None
        return dist.all_reduce(t, group=self.pg, async_op=True)

    def finish(self) -> None:
        """Launch buckets whose params got no gradient (in index order on every rank),
        then wait for all all-reduces of this step."""
        if not self.enabled:
            return
        if self._order_stream is not None and not all(self._launched):
            # buckets still open hold parameters that got no gradient this step: their
            # slices were zeroed on the current stream (Trainer: zero_unwritten)
            self._order_stream.wait_stream(torch.cuda.current_stream(self.arena.grad.device))
        for b in range(len(self.buckets)):
            if not self._launched[b]:
                self._launch(b)
        if self._opt is not None:
            self._flush_updates()
            if self._order_stream is not None:
                # the next forward reads the updated weights / bf16 shadows
                self._main_stream.wait_stream(self._order_stream)
            self.prepare()
            return
        if self._order_stream is not None and any(w is None for _, w in self._works):
            # captured blocking collectives ordered the ordering stream only
            torch.cuda.current_stream(self.arena.grad.device).wait_stream(self._order_stream)
        for b, w in self._works:
            if w is not None:
                w.wait()
            if self.compress:
                s, e, _ = self.buckets[b]
                self.arena.grad[s:e].copy_(self._shadow[b])
        self.prepare()

    @property
    def updates_in_finish(self) -> bool:
        """True while a per-bucket optimizer is set for the running step."""
        return self._opt is not None

    def remove(self) -> None:
        for h in self._handles:
            h.remove()
        self._handles = []


def broadcast_params(arena, src: int = 0, process_group=None) -> None:
    """Make every rank start from rank 0's weights (one collective on the flat arena)."""
    if dist.is_initialized() and dist.get_world_size(process_group) > 1:
        dist.broadcast(arena.flat, src=src, group=process_group)
