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

import math
import os
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from .models import DeepSpeech2
from .ops.optim import FusedAdamEMA, ParamArena, exponential_decay
from .parallel.grad_sync import GradBucketer, broadcast_params
from .utils import trace as TR
from .utils.stats import NonfiniteWatch


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


class Trainer:
    def __init__(self, model: DeepSpeech2, lr_schedule: LRSchedule, moving_avg_decay: Optional[float] = 0.9999,
                 world_size: int = 1, bucket_mb: float = 32.0, allreduce_bf16: bool = False,
                 nan_policy: str = "abort", collapse_repeated: bool = False, force_buckets: bool = False):
        self.model = model
        self._seed = {}            # (device, dtype) -> device scalar 1.0 (backward seed)
        # bf16 compute shadows of the weights only for the HIP engine (fused ops read them)
        self.arena = ParamArena(model, bf16_shadow=(model.engine == "hip"))
        self.opt = FusedAdamEMA(self.arena, lr=lr_schedule.initial_lr, ema_decay=moving_avg_decay)
        self.lr_schedule = lr_schedule
        self.world = world_size
        self.bucketer = GradBucketer(self.arena, bucket_mb=bucket_mb, compress_bf16=allreduce_bf16,
                                     world_size=world_size, force=force_buckets)
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
        # Per-layer optimizer (1 GPU, HIP engine). The arena is laid out in gradient-production
        # order, and a recurrent layer's weights are never read again once its last weight
        # gradient is written (the dx GEMM reading W_l is issued before dW_l, whose side-stream
        # GEMM waits behind it). At the end of backward the main stream (conv front-end
        # backward + dU_0) finishes before the side stream's deferred dW GEMMs, so instead
        # of one whole-arena launch after both streams join, the main stream updates each
        # layer's arena range as soon as that range's gradients are final: its own range
        # [U_0, b_h0, conv] at once, then [W_0, b_0], [FC + layer L-1], [layer L-2], ... in
        # the order the side stream finishes them — memory-bound updates beside the
        # remaining compute-bound GEMMs. Measured slower on MI355X and therefore OFF by
        # default (DS2_SPLIT_ADAM=1 enables it): same-box A/B 8.80-8.87 vs 8.68-8.71 ms/step
        # (tools/host_overhead.py; one wait per range and stream; a per-parameter wait list
        # was 9.0, a third "optimizer" stream 9.2). profiles/r1_s3_negative_results.md.
        self._bounds = None
        names = self.arena.names
        if (os.environ.get("DS2_SPLIT_ADAM", "0") == "1" and model.engine == "hip"
                and self.arena.flat.is_cuda and not self.bucketer.enabled and "rnn.0.fw.U" in names):
            L = len(model.rnn)
            cuts = [names.index("rnn.%d.fw.W" % i) for i in range(L - 2, -1, -1) if "rnn.%d.fw.W" % i in names]
            cuts.append(names.index("rnn.0.fw.U"))
            if cuts == sorted(cuts) and cuts[0] > 0:
                self._bounds = [0] + cuts + [len(names)]
                self.arena.enable_ready_events()

        # Overlapped optimizer (1 GPU, HIP engine, DS2_OVERLAP_OPT): at the end of a step only
        # layer 0 + the conv front-end are updated; the update of the arena prefix [FC +
        # layers L-1..1] is prepared with the same (lr_t, EMA decay) and runs during the next
        # forward, beside layer 0's recurrence (ops.optim.DeferredUpdate). Same arithmetic,
        # same order of reads and writes of every weight; flush_optimizer() completes it for
        # any reader between steps (checkpoint, EMA swap, eval, the bench's last step).
        self._defer_hi = None
        self._defer_grid = int(os.environ.get("DS2_OVERLAP_OPT_GRID", "48"))
        if (os.environ.get("DS2_OVERLAP_OPT", "0") == "1" and self._bounds is None and model.engine == "hip"
                and self.arena.flat.is_cuda and not self.bucketer.enabled and len(model.rnn) >= 2
                and "rnn.0.fw.W" in names
                and all(getattr(l, "seq_bn", "frozen") in ("frozen", "none") for l in model.rnn)):
            self._defer_hi = self.arena.offsets[names.index("rnn.0.fw.W")][0]

    def flush_optimizer(self) -> None:
        """Complete any deferred optimizer update (call before reading weights, EMA or Adam
        state outside step())."""
        self.arena.flush_update()

    @property
    def _split_at(self):
        return None if self._bounds is None else self._bounds[-2]

    def _optimizer_parts(self):
        """(lo, hi, stream, events) ranges for FusedAdamEMA.step, or None (single launch).
        Call after the backward is fully queued (and after zero_unwritten)."""
        a = self.arena
        b = self._bounds
        if b is None:
            return None
        parts = []
        nr = len(b) - 1
        for r in range(nr):
            members = []
            for i in range(b[r], b[r + 1]):
                if id(a.params[i]) in a._written:
                    members.append(i)
                elif r < nr - 1:
                    return None        # zeroed / autograd-accumulated on the main stream
            waits = a.ready_events_covering(members)
            lo = a.offsets[b[r]][0]
            hi = a.offsets[b[r + 1]][0] if b[r + 1] < len(a.params) else a.numel
            parts.append((lo, hi, None, waits))
        # issue order: the main stream's own range, W_0 (the side stream's first tail GEMM),
        # then FC + layer L-1, L-2, ... (the deferred dW GEMMs' order)
        order = [nr - 1, nr - 2] + list(range(nr - 2))
        return [parts[r] for r in order]

    @property
    def lr(self) -> float:
        return self.lr_schedule(self.global_step)

    def step(self, batch: Dict[str, torch.Tensor]) -> torch.Tensor:
        model = self.model
        model.train()
        self.arena.ensure_bf16()
        # the HIP engine delivers every gradient through the arena (first write overwrites),
        # so the per-step memset of the whole gradient buffer is skipped
        lazy = model.engine == "hip"
        self.arena.wgrad.discard()
        self.arena.zero_grad(lazy=lazy)
        loss = model.forward_loss(batch["feats"], batch["seq_lens"], batch["labels"], batch["label_lens"])
        # normally consumed inside the forward (layer 1); never let backward overwrite the
        # gradients a pending update still has to read
        self.arena.flush_update()
        self.watch.update(loss)
        # a cached device 1.0 as the backward seed: autograd would launch a fill for ones_like
        one = self._seed.get((loss.device, loss.dtype))
        if one is None:
            one = self._seed[(loss.device, loss.dtype)] = torch.ones((), device=loss.device, dtype=loss.dtype)
        loss.backward(one)
        parts = None
        if self._bounds is not None and self.nan_policy != "skip":
            self.arena.wgrad.drain()
            if lazy:
                self.arena.zero_unwritten()
            parts = self._optimizer_parts()
            if parts is None and lazy:
                lazy = False           # already zeroed
        if parts is not None:
            with TR.phase(TR.EMA):
                self.opt.step(self.lr, self.global_step, gscale=1.0 / self.world, parts=parts)
            self.arena.wgrad.join()
            self.global_step += 1
            return loss.detach()
        self.arena.wgrad.join()
        if lazy:
            self.arena.zero_unwritten()
        with TR.phase(TR.ALLREDUCE):
            self.bucketer.finish()
        gscale = 1.0 / self.world
        skip = None
        if self.nan_policy == "skip":
            _, skip = self.opt.grad_norm_and_finite(gscale)
            self.last_skip = skip
        with TR.phase(TR.EMA):
            if self._defer_hi is not None and skip is None:
                from .ops.optim import DeferredUpdate
                lr_t, keep = self.opt.prepare(self.lr, self.global_step)
                self.opt.apply_range(self._defer_hi, self.arena.numel, lr_t, keep, gscale)
                self.arena.pending_update = DeferredUpdate(self.opt, 0, self._defer_hi, lr_t, keep, gscale,
                                                           self._defer_grid)
            else:
                self.opt.step(self.lr, self.global_step, gscale=gscale, skip_flag=skip)
        self.global_step += 1
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
        self.flush_optimizer()
        if self.opt.ema is None:
            return
        tmp = self.arena.flat.clone()
        self.arena.flat.copy_(self.opt.ema)
        self.opt.ema.copy_(tmp)
        self.arena.mark_dirty()
