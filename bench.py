#!/usr/bin/env python3
"""Headline benchmark: DeepSpeech2 (2x conv + 5x BiGRU-800) bf16 training throughput.

Metric (BASELINE.json): audio-sec/sec training throughput of the whole job, on synthetic
LibriSpeech-shaped spectrogram batches with random-init weights (no dataset/checkpoint
is available offline). Every step is a full training step: forward, CTC loss, backward,
RCCL gradient all-reduce (N > 1), fused Adam + weight EMA.

  python bench.py --gpus N --steps K --warmup W
  (N > 1: either bench.py starts the N ranks itself, or an outer launcher does:
   python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...;
   a --gpus that disagrees with the launcher's WORLD_SIZE is an error)

Batch: 32 utterances per GPU (the reference's headline batch, src/train.sh:42), each
padded to 1000 frames (10 s) with per-utterance lengths in (900, 1000] frames (one
100-frame bucket, as bucket_by_sequence_length does in src/deepSpeech_input.py:53-60) and
~15 characters/second of labels. audio-seconds = sum of true lengths / 100 (10 ms frames).
Scaling is weak: per-GPU work is fixed as N grows.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# platform environment (RCCL channel budget, kernel-argument placement, high-priority
# collectives) before torch is imported: deepspeech_amd/utils/setenvs.py
from deepspeech_amd.utils.setenvs import setenvs  # noqa: E402

setenvs([])


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU) on this node; without an outer launcher (torchrun) "
                        "bench.py starts them itself (parallel/launch.py). Default: the launcher's "
                        "WORLD_SIZE, else 1")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch_size", type=int, default=32, help="utterances per GPU")
    p.add_argument("--frames", type=int, default=1000, help="padded utterance length (10 ms frames)")
    p.add_argument("--num_hidden", type=int, default=800)
    p.add_argument("--num_rnn_layers", type=int, default=5)
    p.add_argument("--num_filters", type=int, default=32)
    p.add_argument("--cell", type=str, default="gru")
    p.add_argument("--engine", type=str, default="hip", choices=["hip", "ref"])
    p.add_argument("--bucket_mb", type=float, default=32.0)
    p.add_argument("--allreduce_bf16", action="store_true")
    p.add_argument("--profile_dir", type=str, default="", help="write a torch.profiler trace here")
    p.add_argument("--force_dp", action="store_true",
                   help="run the data-parallel machinery (process group, gradient buckets, "
                        "collectives on the ordering stream) even on one GPU, to time its overhead")
    p.add_argument("--step_graphs", action="store_true",
                   help="time the captured step (HIP step graphs; with --force_dp / N > 1 the "
                        "bucketed step, Trainer dp_graphs) instead of the eager one: the short "
                        "SortaGrad lengths (--frames 100) are host-bound eagerly")
    p.add_argument("--dp_graphs", action="store_true",
                   help="data parallel: the epoch walk's per-shape step graphs capture the bucketed "
                        "step too (Trainer dp_graphs)")
    p.add_argument("--no_infer", action="store_true",
                   help="skip the streaming-inference RTF measured after the training timing "
                        "(BASELINE metric's inference half; rank 0, outside the timed region)")
    p.add_argument("--infer_seconds", type=float, default=10.0, help="audio per stream of the RTF runs")
    p.add_argument("--no_walk", action="store_true",
                   help="skip the SortaGrad epoch walk measured after the headline timing")
    p.add_argument("--walk_scale", type=int, default=1,
                   help="epoch-walk size: the reference dummy epoch's bucket counts x this (reference: 10)")
    p.add_argument("--no_defer_update", action="store_true",
                   help="apply every step's whole optimizer update inside that step instead of carrying "
                        "the head's and upper layers' range into the next forward (A/B)")
    p.add_argument("--no_carry_du", action="store_true",
                   help="with the carried update, keep the upper layers' dU GEMMs beside the next BPTT (A/B)")
    p.add_argument("--no_gate", action="store_true",
                   help="side-stream work beside a persistent recurrence without the residency gate (A/B)")
    p.add_argument("--no_proj_beside", action="store_true",
                   help="A/B: projections keep the whole grid while a carried dU GEMM runs beside")
    p.add_argument("--carry_blocks", type=int, default=0,
                   help="blocks per idle CU of the carried optimizer chunks (A/B; 0: the default)")
    p.add_argument("--fp8", action="store_true",
                   help="BASELINE config 5's fp8 mode: MX-fp8 e4m3 input projections, an e4m3 forward "
                        "recurrence (U and hidden-state exchange) and an fp8 BPTT (e4m3 U^T, E8M0-scaled "
                        "gate gradients); weight gradients and the front-end stay bf16. NOT the "
                        "headline bf16 number")
    return p.parse_args()


def main():
    args = parse()
    from deepspeech_amd.parallel.launch import check_world, maybe_spawn
    # --gpus N > 1 without torchrun: N child ranks of this same command; this process never
    # touches the GPU and exits with the job's code
    code = maybe_spawn(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    if code is not None:
        sys.exit(code)
    world = check_world(args.gpus)
    import torch
    from deepspeech_amd.parallel.dist import init_distributed, shutdown
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.trainer import Trainer, LRSchedule
    from deepspeech_amd.ops import rnn as RNN

    ctx = init_distributed("auto", force_group=args.force_dp)
    assert ctx.world_size == world, (ctx.world_size, world)
    dev = ctx.device
    if dev.type != "cuda" and args.engine == "hip":
        args.engine = "ref"
    torch.manual_seed(1234)
    model = DeepSpeech2(num_filters=args.num_filters, num_hidden=args.num_hidden,
                        num_rnn_layers=args.num_rnn_layers, cell=args.cell, bidirectional=True,
                        stack_fix=True, seq_bn="frozen").to(dev)
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    model.set_engine(args.engine, dtype, fp8=bool(args.fp8 and args.engine == "hip"))
    if args.no_carry_du:
        import deepspeech_amd.trainer as _T
        _T._CARRY_DU = False
    if args.no_gate:
        RNN._RESIDENCY_GATE = False
    if args.no_proj_beside:
        RNN._PROJ_BESIDE = False
    if args.carry_blocks:
        import deepspeech_amd.trainer as _T
        _T._CARRY_BLOCKS_PER_CU, _T._CARRY_LDS = args.carry_blocks, 32768
    trainer = Trainer(model, LRSchedule(1e-4, 10 ** 9, 0.9), moving_avg_decay=0.9999,
                      world_size=ctx.world_size, bucket_mb=args.bucket_mb,
                      allreduce_bf16=args.allreduce_bf16, force_buckets=args.force_dp,
                      defer_update=not args.no_defer_update, dp_graphs=args.dp_graphs or args.step_graphs,
                      step_graphs=bool(args.step_graphs))
    feed = FixedShapeBatches(args.batch_size, max_frames=args.frames, seed=1000 + ctx.rank, pool=4)
    batches = [to_device(feed.next(), dev) for _ in range(4)]
    audio_per_step = [float(b["seq_lens"].sum().item()) / 100.0 for b in batches]
    # analytic training FLOPs at each utterance's TRUE length (not the padded frame count)
    flops_per_step = [sum(model.flops_per_step(1, int(t)) for t in b["seq_lens"].tolist()) for b in batches]

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for i in range(args.warmup):
        trainer.step(batches[i % len(batches)])
    trainer.flush()
    sync()
    if dev.type == "cuda":
        RNN.check_errors()
    ctx.barrier()
    sync()
    prof = None
    if args.profile_dir and ctx.is_main:
        from torch.profiler import profile, ProfilerActivity
        prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA])
        prof.__enter__()
    t0 = time.perf_counter()
    audio = 0.0
    flops = 0.0
    loss = None
    for i in range(args.steps):
        loss = trainer.step(batches[i % len(batches)])
        audio += audio_per_step[i % len(batches)]
        flops += flops_per_step[i % len(batches)]
    # the last step's optimizer update carried into a next forward (Trainer defer_update)
    # is enqueued here, INSIDE the timed region: every timed step's update is measured
    trainer.flush()
    sync()
    ctx.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(args.profile_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(args.profile_dir, "bench_trace.json"))
        with open(os.path.join(args.profile_dir, "bench_ops.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
    if dev.type == "cuda":
        RNN.check_errors()
    elapsed = ctx.all_reduce_max(elapsed)
    total_audio = ctx.all_reduce_sum(audio)
    ms = 1000.0 * elapsed / args.steps
    value = total_audio / elapsed
    flops = ctx.all_reduce_sum(flops)
    lossv = float(loss.float().item()) if loss is not None else float("nan")
    # device memory high-water mark of the headline steps (caching allocator; this rank)
    peak_gib = torch.cuda.max_memory_allocated(dev) / 2 ** 30 if dev.type == "cuda" else None
    walk = None
    if not args.no_walk and dev.type == "cuda":
        walk = epoch_walk(trainer, ctx, dev, args.batch_size, args.walk_scale)
    shutdown(ctx)
    infer = None
    if ctx.is_main and not args.no_infer:
        infer = streaming_rtf(dev, args.engine, args.infer_seconds)
    if ctx.is_main:
        out = {
            "metric": "audio-sec/sec training throughput (whole node), DS2 BiGRU",
            "value": round(value, 2),
            "unit": "audio-sec/sec",
            "n_gpus": ctx.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("fp8(proj+fwd recurrence)+bf16" if args.fp8 else "bf16") if dtype == torch.bfloat16 else "fp32",
            "data": "synthetic (LibriSpeech-shaped spectrograms, random-init weights)",
            "config": {
                "model": "DeepSpeech2 2xconv(32) + %dx%s-%d bidirectional + CTC" % (
                    args.num_rnn_layers, "BiGRU" if args.cell == "gru" else "BiRNN", args.num_hidden),
                "global_batch": args.batch_size * ctx.world_size,
                "seq_len": args.frames,
                "parallelism": "dp%d" % ctx.world_size,
                "engine": args.engine,
            },
            "per_gpu_audio_sec_per_sec": round(value / ctx.world_size, 2),
            "utterances_per_sec": round(args.batch_size * ctx.world_size * args.steps / elapsed, 2),
            "achieved_tflops": round(flops / elapsed / 1e12, 2),
            "final_loss": round(lossv, 4),
        }
        if peak_gib is not None:
            out["peak_mem_gib"] = round(peak_gib, 2)
        if walk is not None:
            out["epoch_walk"] = walk
        if infer is not None:
            out["inference"] = infer
        print(json.dumps(out), flush=True)


def epoch_walk(trainer, ctx, dev, batch_size: int, scale: int):
    """SortaGrad epoch throughput, measured AFTER and outside
    the headline timing: one dummy epoch in the reference's order — buckets of 100..1500
    frames ascending, each bucket's batch count from src/deepSpeech_dummy.py:9-11 (x scale;
    the reference uses 10), data/synthetic.py DummyBucketWalk — with the batches staged on
    the device beforehand (the reference's dummy mode times data generation separately,
    src/deepSpeech_train.py:309-312). The same trainer continues training; on one GPU it runs
    the captured-step path with per-shape eager / replay selection (Trainer step_graphs
    "auto"). A first pass captures and decides every shape untimed; the second pass is timed
    (barrier + synchronize on both sides, max over ranks; audio summed over ranks). An eager
    pass follows for comparison."""
    import torch
    from deepspeech_amd.data.synthetic import DummyBucketWalk, to_device
    walk = DummyBucketWalk(batch_size, seed=77 + ctx.rank, scale_factor=scale)
    n = walk.steps_per_epoch()
    host = [walk.next() for _ in range(n)]
    batches = [to_device(b, dev) for b in host]
    audio = sum(b.audio_seconds for b in host)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def timed():
        sync()
        ctx.barrier()
        sync()
        t0 = time.perf_counter()
        for b in batches:
            trainer.step(b)
        trainer.flush()
        sync()
        ctx.barrier()
        sync()
        return ctx.all_reduce_max(time.perf_counter() - t0)

    total_audio = ctx.all_reduce_sum(audio)
    res = {"what": "one dummy epoch in SortaGrad order (100..1500-frame buckets ascending, "
                   "src/deepSpeech_dummy.py counts x %d), audio-sec/sec whole job" % scale,
           "steps": n, "audio_s": round(total_audio, 1)}
    prev = trainer.step_graphs
    if trainer.graphs_active() or (dev.type == "cuda" and ctx.world_size == 1):
        trainer.step_graphs = "auto"
    for b in batches:                     # untimed: plans, captures, per-shape decisions
        trainer.step(b)
    el = timed()
    res["audio_s_per_s"] = round(total_audio / el, 1)
    res["ms"] = round(1e3 * el, 1)
    if trainer.graph_modes:
        res["modes"] = {str(k[1]): m[0] for k, m in sorted(trainer.graph_modes.items())}
    trainer.step_graphs = False
    el_e = timed()
    res["eager_audio_s_per_s"] = round(total_audio / el_e, 1)
    trainer.step_graphs = prev
    return res


def streaming_rtf(dev, engine: str, seconds: float):
    """Streaming-inference real-time factor (BASELINE metric's second half; north-star config
    4: 2 x conv + 5 x uni-GRU-800 + CTC, greedy and prefix-beam-16 decoding), measured AFTER
    and outside the training timing. RTF = compute seconds / audio seconds per stream, 0.5 s
    chunks, 1 and 32 concurrent streams (a chunk of all streams is one launch sequence, HIP
    graph replay), synthetic features and random-init weights (infer.py). Reference eval path:
    src/deepSpeech_test.py:112-136 (whole-utterance greedy decode)."""
    import torch
    from deepspeech_amd.infer import rtf
    from deepspeech_amd.models import DeepSpeech2
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=32, num_hidden=800, num_rnn_layers=5, cell="gru", bidirectional=False).to(dev)
    m.set_engine(engine, torch.bfloat16 if engine == "hip" else torch.float32)
    if dev.type != "cuda":
        seconds = min(seconds, 2.0)
    rtf(m, seconds=1.0, chunk_s=0.5, batch=1)          # warm-up: plans, kernels, graph capture
    res = {"model": "DS2 2xconv(32) + 5x uni-GRU-800 + CTC", "chunk_s": 0.5, "audio_s_per_stream": seconds,
           "unit": "RTF = compute s / audio s per stream (lower is better)"}
    for B in (1, 32):
        for dec in ("greedy", "beam"):
            r, _ = rtf(m, seconds=seconds, chunk_s=0.5, batch=B, decoder=dec, beam_width=16)
            key = "rtf_%s%s_streams%d" % (dec, "16" if dec == "beam" else "", B)
            res[key] = round(r, 6)
            res["x_realtime_total_%s%s_streams%d" % (dec, "16" if dec == "beam" else "", B)] = \
                round(B / r, 1) if r > 0 else None
    return res


if __name__ == "__main__":
    main()
