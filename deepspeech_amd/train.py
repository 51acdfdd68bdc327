"""Training driver, CLI-compatible with the reference's deepSpeech_train.py.

  python -m deepspeech_amd.train --batch_size 32 --no-shuffle --max_steps 40000 \
      --num_rnn_layers 7 --num_hidden 1760 --num_filters 32 --initial_lr 1e-4 \
      --train_dir ../models/librispeech/train --data_dir ../data/LibriSpeech/processed/ \
      [--dummy True] [--cell gru] [--engine hip]
  multi-GPU: python -m deepspeech_amd.train --gpus 8 ...   (or under torch.distributed.run)

Reference flow (src/deepSpeech_train.py:419-528): wipe/create train_dir, dump the flags to
deepSpeech_parameters.json, build graph, Adam + staircase LR + weight EMA, restore or
init, loop: step, NaN check, throughput line every 10 steps (after step 10), summaries
every 50 steps, checkpoint every 10 steps + last, --debug traces at step 20.
"""
from __future__ import annotations

import glob
import os
import sys
import time
from datetime import datetime
from typing import Optional

import numpy as np
import torch

from . import config as C
from .data.synthetic import DummyBucketWalk, FixedShapeBatches, to_device
from .models import DeepSpeech2
from .ops import reference as R
from .parallel.dist import init_distributed, shutdown
from .trainer import Trainer, lr_schedule_from_args
from .utils import checkpoint as CK
from .utils.summary import EventWriter, JsonlWriter

OUR_FILES = ("model.ckpt-*", "checkpoint", "events.out.tfevents.*", "deepSpeech_parameters.json",
             "metrics.jsonl", "profiling.json", "profile_*.txt")


def clean_train_dir(path: str) -> None:
    """The reference deletes train_dir unless it is the --checkpoint dir
    (src/deepSpeech_train.py:504-507). We remove only the files this driver writes."""
    os.makedirs(path, exist_ok=True)
    for pat in OUR_FILES:
        for f in glob.glob(os.path.join(path, pat)):
            if os.path.isfile(f):
                os.remove(f)


def collapse_batch_labels(batch):
    """preprocess_collapse_repeated=True (src/deepSpeech_NCHW.py:225), applied on the host."""
    labs = batch.labels.copy()
    lens = batch.label_lens.copy()
    for i in range(labs.shape[0]):
        c = R.collapse_repeated(labs[i, : lens[i]].tolist())
        labs[i, :] = -1
        labs[i, : len(c)] = c
        lens[i] = len(c)
    batch.labels, batch.label_lens = labs, lens
    return batch


def build_data(args, ctx, train_dir):
    """Returns (source with .next(), steps_per_epoch)."""
    if args.dummy:
        if args.dummy_frames > 0:
            # fixed-length synthetic batches (bench.py's shape) instead of the reference's walk
            from .data.synthetic import FixedShapeBatches
            src = FixedShapeBatches(args.batch_size, max_frames=args.dummy_frames, seed=args.seed + ctx.rank, pool=4)
            return src, 1000
        src = DummyBucketWalk(args.batch_size, seed=args.seed + ctx.rank)
        return src, src.steps_per_epoch()
    from .data.store import StoreBatches, find_partition_files, find_store, tfrecords_to_store
    if not args.data_dir:
        raise ValueError("Please supply a data_dir (or --dummy True)")
    prefix = find_store(args.data_dir, "train")
    if prefix is None:
        files = find_partition_files(args.data_dir, "train")
        if not files:
            raise ValueError("no training data (store or TFRecords) under %s" % args.data_dir)
        prefix = os.path.join(train_dir, "cache", "train")
        if ctx.is_main and not os.path.exists(prefix + ".index.npz"):
            tfrecords_to_store(files, prefix)
        ctx.barrier()
    src = StoreBatches(prefix, args.batch_size, rank=ctx.rank, world=ctx.world_size,
                       max_frames=args.max_frames, sortagrad_epochs=args.sortagrad_epochs if not args.shuffle else 0,
                       shuffle=True, seed=args.seed)
    return src, src.steps_per_epoch()


def write_debug_reports(prof, model, args, dev) -> None:
    """--debug outputs (reference src/deepSpeech_train.py:358-380: chrome trace + tfprof
    params / flops / timing logs): profiling.json, params.log, flops.log, profile_ops.txt
    and the per-layer breakdown profile_layers.txt (deepspeech_amd/utils/prof.py)."""
    from .utils import prof as P
    d = args.train_dir
    trace = os.path.join(d, "profiling.json")
    prof.export_chrome_trace(trace)
    with open(os.path.join(d, "profile_ops.txt"), "w") as f:
        f.write(prof.key_averages().table(sort_by="self_cuda_time_total" if dev.type == "cuda"
                                          else "self_cpu_time_total", row_limit=80))
    with open(os.path.join(d, "params.log"), "w") as f:
        tot = 0
        for n, p in model.named_parameters():
            f.write("%-40s %-20s %d\n" % (n, tuple(p.shape), p.numel()))
            tot += p.numel()
        f.write("total trainable params: %d\n" % tot)
    with open(os.path.join(d, "flops.log"), "w") as f:
        for name, fl in model.flops_breakdown(args.batch_size, 1000).items():
            f.write("%-24s %.3f GFLOP (fwd, per batch of %d x 10 s)\n" % (name, fl / 1e9, args.batch_size))
    out, _ = P.analyse(P.load_events(trace))
    with open(os.path.join(d, "profile_layers.txt"), "w") as f:
        f.write(P.format_table(out) + "\n")


def resume_dir(args) -> Optional[str]:
    """Directory to resume from: --checkpoint (reference semantics), or train_dir itself under
    --resume auto / an elastic restart (torchrun --max-restarts) when it holds a checkpoint."""
    if args.checkpoint is not None:
        return args.checkpoint
    restarted = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or 0) > 0
    if (args.resume == "auto" or restarted) and CK.latest_checkpoint(args.train_dir) is not None:
        return args.train_dir
    return None


def write_summaries(events, step: int, trainer, model, args, lv: float, ema: float) -> None:
    """Reference add_summaries (src/deepSpeech_train.py:401-416: learning rate, gradient and
    variable histograms) + _activation_summary (src/helper_routines.py:15-28). Histograms are
    computed on the device (csrc/stats.hip), one pass per tensor; tags use the TF variable
    names of the checkpoint layout."""
    from .utils.stats import histogram
    events.scalars(step, {"ctc_loss(raw)": lv, "ctc_loss": ema, "learning_rate": trainer.lr})
    tfname = {tn: tf for tf, tn, _, _ in CK.tf_name_map(model)}
    grads = trainer.arena.views(trainer.arena.grad)
    for n, p in model.named_parameters():
        tag = tfname.get(n, n)
        events.histogram_stats(step, tag, histogram(p.detach()))
        if n in grads:
            events.histogram_stats(step, tag + "/gradients", histogram(grads[n]))
    if args.activation_summaries:
        for name, t in model.act_taps.items():
            st = histogram(t)
            events.histogram_stats(step, name + "/activations", st)
            events.scalars(step, {name + "/sparsity": st.zero_fraction})
    model.act_taps.clear()
    events.flush()


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = C.parse_train_args(argv)
    from .parallel.launch import check_world, maybe_spawn_cmd
    # --gpus N > 1 without torchrun: N child ranks of this same command line; this process never
    # touches the GPU and returns the job's code
    code = maybe_spawn_cmd(args.gpus, [sys.executable, "-u", "-m", "deepspeech_amd.train"] + argv)
    if code is not None:
        return code
    world = check_world(args.gpus)
    from .utils.setenvs import setenvs
    setenvs(platform=args.platform if args.platform in ("mi355x", "knl", "bdw") else "mi355x")   # before HIP init
    ctx = init_distributed(args.device)
    if ctx.world_size != world:
        raise SystemExit("world size %d does not match --gpus / WORLD_SIZE %d" % (ctx.world_size, world))
    dev = ctx.device
    engine = C.resolve_engine(args.engine, dev)
    dtype = C.resolve_dtype(args.dtype, args.use_fp16, dev)
    torch.manual_seed(args.seed)
    np.random.seed(args.seed + ctx.rank)
    if ctx.is_main:
        print("debug: ", args.debug)
        print("nchw: ", args.nchw)
        print("dummy: ", args.dummy)
        print("engine: ", args.engine, "->", engine, "| dtype:", dtype, "| world:", ctx.world_size)
        if args.train_dir != args.checkpoint and resume_dir(args) is None:
            clean_train_dir(args.train_dir)
        C.dump_param_json(args, args.train_dir)
        print("Running on platform: ", args.platform)
    ctx.barrier()

    model = DeepSpeech2(**C.model_kwargs_from_args(args)).to(dev)
    model.set_engine(engine, dtype, fp8=(args.dtype == "fp8" and engine == "hip"))
    # --engine mkldnn_rnn / cudnn_rnn (reference: MkldnnRNNCell, src/deepSpeech_NCHW.py:173-176)
    # checkpoints keep the MKL-DNN single-blob RNN parameters (utils/mkldnn_blob.py)
    if args.engine in ("mkldnn_rnn", "cudnn_rnn") and model.cell == "rnn_relu" and model.layout == "nchw":
        model.param_layout = "mkldnn"
    data, steps_per_epoch = build_data(args, ctx, args.train_dir)
    trainer = Trainer(model, lr_schedule_from_args(args, steps_per_epoch), args.moving_avg_decay,
                      world_size=ctx.world_size, bucket_mb=args.bucket_mb,
                      allreduce_bf16=args.allreduce_dtype == "bf16", nan_policy=args.nan_policy,
                      step_graphs={"auto": "auto", "on": True, "off": False}[args.step_graphs],
                      defer_update=True, dp_graphs=args.dp_step_graphs)
    start = 0
    rdir = resume_dir(args)
    if rdir is not None:
        print("has checkpoint", rdir)
        step = CK.restore(trainer, rdir)
        if step is not None:
            start = trainer.global_step
            trainer.watch.reset(start)
    else:
        print("does not have checkpoint")
    if ctx.is_main:
        for n, p in model.named_parameters():
            print("Variable: ", n, tuple(p.shape))
        print("parameters: %d" % model.num_params())

    ckpt = (CK.CheckpointManager(args.train_dir, args.max_to_keep, args.async_checkpoint, fmt=args.checkpoint_format,
                                 nan_policy=args.nan_policy) if ctx.is_main else None)
    events = EventWriter(args.train_dir) if ctx.is_main else None
    metrics = JsonlWriter(os.path.join(args.train_dir, "metrics.jsonl")) if ctx.is_main else None
    durations = []
    audio_hist = []
    t_last = time.time()
    steps_since = 0
    audio_since = 0.0
    loss = None
    prof = None
    # per-step device time from events recorded after each step (no per-step sync); read at
    # the host sync points -> p50/p95 step time and achieved TFLOP/s in metrics.jsonl
    step_events = []           # (event, analytic training FLOPs of the step)
    ev_prev = None
    first_attempt = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or 0) == 0
    sum_on = ctx.is_main and (not args.dummy or args.summaries_on_dummy) and args.summary_every > 0
    trainer.keep_grads = sum_on          # gradient histograms read arena.grad after the step

    def check_divergence():
        bad = trainer.first_nonfinite_step()
        if bad is not None and args.nan_policy == "abort":
            raise FloatingPointError("Model diverged with loss = NaN (step %d)" % bad)
        return bad

    class _Src:       # host batches, labels collapsed like TF preprocess_collapse_repeated
        def next(self):
            hb_ = data.next()
            return collapse_batch_labels(hb_) if args.ctc_collapse_repeated else hb_
    src = _Src()
    # GPU: batches are produced and uploaded by a background thread through a pinned ring
    # (data/prefetch.py), overlapping the previous steps' kernels
    prefetch = None
    if dev.type == "cuda" and os.environ.get("DS2_PREFETCH", "1") == "1":
        from .data.prefetch import DevicePrefetcher
        prefetch = DevicePrefetcher(src, dev, depth=2)

    for step in range(start, args.max_steps):
        t0 = time.time()
        if prefetch is not None:
            hb, batch = prefetch.next()
        else:
            hb = src.next()
            batch = None
        data_time = time.time() - t0
        if args.debug and step == 20:
            from torch.profiler import ProfilerActivity, profile
            from .utils import trace as TR
            TR.enable(True)
            prof = profile(activities=[ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if dev.type == "cuda" else []),
                           record_shapes=False)
            prof.__enter__()
        if batch is None:
            batch = to_device(hb, dev)
        model.capture = sum_on and step % args.summary_every == 0
        loss = trainer.step(batch)
        model.capture = False
        if dev.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            fl = sum(model.flops_per_step(1, int(t)) for t in np.asarray(hb.seq_lens).tolist())
            step_events.append((ev, fl))
        if args.fault_inject_step == step and ctx.rank == args.fault_inject_rank and first_attempt:
            print("fault injection at step %d on rank %d" % (step, ctx.rank), flush=True)
            os._exit(17)
        steps_since += 1
        audio_since += hb.audio_seconds
        if prof is not None:
            trainer.flush()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            prof.__exit__(None, None, None)
            from .utils import trace as TR
            TR.enable(False)
            if ctx.is_main:
                write_debug_reports(prof, model, args, dev)
            prof = None
        do_log = (step > 10 and step % args.log_every == 0) or step + 1 == args.max_steps
        do_sum = sum_on and step % args.summary_every == 0
        # checkpoints need no host synchronisation (utils/checkpoint.py: device snapshot + side-
        # stream copy + writer thread); --checkpoint_every 0 saves the last step only
        do_ckpt = ctx.is_main and ((args.checkpoint_every > 0 and step % args.checkpoint_every == 0)
                                   or step + 1 == args.max_steps)
        if do_log or do_sum:
            lv = float(loss.item())          # host sync point
            if engine == "hip":
                from .ops import rnn as RNN
                RNN.check_errors()
            check_divergence()               # every step's loss was checked on the device
            step_ms = []
            step_fl = 0.0
            for ev, fl in step_events:
                if ev_prev is not None:
                    step_ms.append(ev_prev.elapsed_time(ev))
                    step_fl += fl
                ev_prev = ev
            step_events = []
            now = time.time()
            dur = (now - t_last) / max(1, steps_since)
            if step >= 10:
                durations.append(dur)
                audio_hist.append(audio_since / max(1e-9, now - t_last))
            t_last, steps_since, audio_since = now, 0, 0.0
            ema = trainer.update_loss_ema(lv)
            if do_log and ctx.is_main and durations:
                sec_batch = float(np.mean(durations))
                ex_sec = args.batch_size * ctx.world_size / sec_batch
                aps = float(np.mean(audio_hist)) * ctx.world_size
                if args.dummy:
                    print("%s: step %d, loss = %.2f (%.1f examples/sec; %.3f sec/batch; %.3f dummy sec/batch; "
                          "%.1f audio-sec/sec)" % (datetime.now(), step, lv, ex_sec, sec_batch, data_time, aps),
                          flush=True)
                else:
                    print("%s: step %d, loss = %.2f (%.1f examples/sec; %.3f sec/batch; %.1f audio-sec/sec)"
                          % (datetime.now(), step, lv, ex_sec, sec_batch, aps), flush=True)
            if ctx.is_main:
                rec = dict(loss=lv, loss_ema=ema, lr=trainer.lr)
                if step_ms:
                    ms = np.asarray(step_ms)
                    rec.update(step_ms_p50=round(float(np.percentile(ms, 50)), 4),
                               step_ms_p95=round(float(np.percentile(ms, 95)), 4),
                               tflops=round(step_fl * ctx.world_size / (ms.sum() / 1e3) / 1e12, 3))
                metrics.write(step, **rec)
            if do_sum:
                trainer.flush()              # variable histograms read the updated weights
                write_summaries(events, step, trainer, model, args, lv, ema)
        if do_ckpt:
            trainer.flush()                  # the snapshot is step <step>'s full update
            if ckpt.save(trainer, step, force=step + 1 == args.max_steps) is None:
                # the writer was still busy with an earlier file: no snapshot (CheckpointManager)
                metrics.write(step, event="checkpoint_skipped", checkpoints_written=len(ckpt.written))
    trainer.flush()
    if loss is not None:
        float(loss.item())
        check_divergence()
    if ckpt is not None:
        ckpt.close()
        if ckpt.written:
            # the effective save cadence of the run
            metrics.write(args.max_steps - 1, event="checkpoint_summary", checkpoints_written=len(ckpt.written),
                          checkpoints_skipped=len(ckpt.skipped), checkpoints_dropped=len(ckpt.dropped),
                          checkpoint_write_s_mean=round(sum(ckpt.write_s) / len(ckpt.write_s), 4))
    if events is not None:
        events.close()
    source_free = prefetch.close() if prefetch is not None else True
    if source_free and hasattr(data, "close"):
        data.close()              # never under a producer thread that is still reading it
    shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
