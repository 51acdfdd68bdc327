"""Command-line flags for the train / eval entrypoints.

Every flag name and default of the reference is kept so existing launch lines work
unchanged (reference: src/deepSpeech_train.py:37-128, src/deepSpeech_test.py:32-74).
MI355X-specific flags are added on top (cell type, dtype, stacking fix, engine
mapping, distributed knobs).

Reference-engine mapping: the reference's ``engine`` values select a
TF kernel family; here they map onto our two engines:
  * ``ref``  – pure PyTorch ops (CPU golden model / debugging)
  * ``hip``  – hand-written gfx950 kernels (persistent RNN, CTC, fused BN, fused Adam)
``tf``/``mkl``/``mkldnn_rnn``/``cudnn_rnn`` are accepted as aliases and resolve to
``hip`` when a GPU is present and ``ref`` otherwise.
"""
from __future__ import annotations

import argparse
import json
import os
from typing import Any, Dict, Optional

ENGINE_ALIASES = ("tf", "mkl", "mkldnn_rnn", "cudnn_rnn")

# Architecture keys restored from deepSpeech_parameters.json on resume
# (reference: src/deepSpeech_train.py:114-127) plus our extensions.
RESUME_KEYS = (
    "num_hidden", "num_rnn_layers", "rnn_type", "num_filters", "use_fp16",
    "temporal_stride", "initial_lr", "engine", "nchw",
    # extensions
    "cell", "stack_fix", "seq_bn", "dtype", "ctc_collapse_repeated",
)
EVAL_KEYS = (
    "num_hidden", "num_rnn_layers", "rnn_type", "num_filters", "use_fp16",
    "moving_avg_decay", "nchw",
    "cell", "stack_fix", "seq_bn", "ctc_collapse_repeated",
)


def str2bool(v: Any) -> bool:
    """distutils.util.strtobool replacement (the reference uses it for bool flags)."""
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("y", "yes", "t", "true", "on", "1"):
        return True
    if s in ("n", "no", "f", "false", "off", "0"):
        return False
    raise argparse.ArgumentTypeError("invalid truth value %r" % (v,))


def _add_model_flags(p: argparse.ArgumentParser) -> None:
    p.add_argument("--cell", type=str, default="rnn_relu", choices=["rnn_relu", "gru"],
                   help="recurrent cell: rnn_relu (reference CustomRNNCell2) or gru")
    p.add_argument("--stack_fix", type=str2bool, default=True,
                   help="stack RNN layers correctly (False reproduces reference quirk Q1)")
    p.add_argument("--seq_bn", type=str, default="frozen", choices=["frozen", "batch", "none"],
                   help="sequence-wise BN on W.x: frozen (reference parity, moving stats "
                        "never updated), batch (DS2 paper), none")
    p.add_argument("--ctc_collapse_repeated", type=str2bool, default=True,
                   help="TF preprocess_collapse_repeated: repeated labels ('LL') are merged before "
                        "the CTC loss, as the reference always does (src/deepSpeech_NCHW.py:225, "
                        "quirk Q5); False = standard CTC")


def build_train_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="DeepSpeech2 training on MI355X")
    # ---- reference flags (names + defaults kept) -----------------------------------
    p.add_argument("--train_dir", type=str, default="../models/librispeech/train",
                   help="Directory to write event logs and checkpoints")
    p.add_argument("--platform", type=str, default="mi355x",
                   help="running platform (knl/bdw accepted for compatibility)")
    p.add_argument("--data_dir", type=str, default="", help="Path to the audio data directory")
    p.add_argument("--max_steps", type=int, default=20000, help="Number of batches to run")
    p.add_argument("--log_device_placement", type=str2bool, default=False)
    p.add_argument("--batch_size", type=int, default=32,
                   help="Number of inputs to process in a batch per GPU")
    p.add_argument("--temporal_stride", type=int, default=1, help="Stride along time (unused, Q8)")
    g = p.add_mutually_exclusive_group(required=False)
    g.add_argument("--shuffle", dest="shuffle", action="store_true")
    g.add_argument("--no-shuffle", dest="shuffle", action="store_false")
    p.set_defaults(shuffle=True)
    g = p.add_mutually_exclusive_group(required=False)
    g.add_argument("--use_fp16", dest="use_fp16", action="store_true")
    g.add_argument("--use_fp32", dest="use_fp16", action="store_false")
    p.set_defaults(use_fp16=False)
    p.add_argument("--keep_prob", type=float, default=0.5, help="dropout keep prob (unused, Q8)")
    p.add_argument("--num_hidden", type=int, default=1024, help="Number of hidden nodes")
    p.add_argument("--num_rnn_layers", type=int, default=2, help="Number of recurrent layers")
    p.add_argument("--checkpoint", type=str, default=None,
                   help="Continue training from checkpoint directory")
    p.add_argument("--rnn_type", type=str, default="bidirectional",
                   help="unidirectional (uni-dir) or bidirectional")
    p.add_argument("--initial_lr", type=float, default=0.00001)
    p.add_argument("--num_filters", type=int, default=32)
    p.add_argument("--moving_avg_decay", type=float, default=0.9999)
    p.add_argument("--num_epochs_per_decay", type=int, default=5)
    p.add_argument("--lr_decay_factor", type=float, default=0.9)
    p.add_argument("--intra_op", type=int, default=44, help="kept for compatibility")
    p.add_argument("--inter_op", type=int, default=1, help="kept for compatibility")
    p.add_argument("--engine", type=str, default="tf",
                   help="ref | hip (aliases: tf, mkl, mkldnn_rnn, cudnn_rnn)")
    p.add_argument("--debug", type=str2bool, default=False,
                   help="write a chrome trace + per-layer profile at step 20")
    p.add_argument("--nchw", type=str2bool, default=True,
                   help="True: the reference's NCHW graph (src/deepSpeech_NCHW.py); False: its NHWC graph "
                        "(src/deepSpeech.py: moments+EMA conv BN, per-direction RNN stacks)")
    p.add_argument("--dummy", type=str2bool, default=False,
                   help="Use synthetic data rather than LibriSpeech data")
    # ---- extensions ---------------------------------------------------------------
    _add_model_flags(p)
    p.add_argument("--dtype", type=str, default="auto", choices=["auto", "fp32", "bf16", "fp8"],
                   help="compute dtype (auto: bf16 on GPU, fp32 on CPU; use_fp16 maps to bf16)")
    p.add_argument("--synthetic", dest="dummy", action="store_true", help="alias of --dummy True")
    p.add_argument("--sortagrad_epochs", type=int, default=1,
                   help="epochs presented in length-sorted order before shuffling")
    p.add_argument("--checkpoint_every", type=int, default=10, help="steps between checkpoints")
    p.add_argument("--max_to_keep", type=int, default=100)
    p.add_argument("--summary_every", type=int, default=50)
    p.add_argument("--log_every", type=int, default=10)
    p.add_argument("--nan_policy", type=str, default="abort", choices=["abort", "skip"])
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--device", type=str, default="auto", help="auto | cpu | cuda")
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU) on this node; without an outer launcher (torchrun) the driver "
                        "starts them itself (parallel/launch.py). Default: the launcher's WORLD_SIZE, else 1")
    p.add_argument("--async_checkpoint", type=str2bool, default=True)
    p.add_argument("--checkpoint_format", type=str, default="tf", choices=["tf", "torch"],
                   help="tf: TF Saver-V2 bundle (model.ckpt-<step>.index + .data-00000-of-00001, "
                        "readable by the reference's tf.train.Saver); torch: one torch.save file")
    p.add_argument("--step_graphs", type=str, default="auto", choices=["auto", "on", "off"],
                   help="single-GPU HIP engine: replay each batch shape's captured training step "
                        "(HIP graph) instead of launching it eagerly; auto: time both once per "
                        "shape and keep the faster (trainer.py _graph_step)")
    p.add_argument("--dp_step_graphs", type=str2bool, default=False,
                   help="data parallel over RCCL: --step_graphs also captures the bucketed step "
                        "(all-reduces and per-bucket optimizer ranges inside the graph; trainer.py "
                        "graphs_active). Checked bitwise at world size 1; off by default until "
                        "measured at world size > 1")
    p.add_argument("--bucket_mb", type=float, default=32.0,
                   help="gradient all-reduce bucket size (MB) for data parallel")
    p.add_argument("--allreduce_dtype", type=str, default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--dummy_frames", type=int, default=0,
                   help="--dummy True: fixed-length synthetic batches of this many frames (bench.py's "
                        "headline shape: 1000) instead of the reference's bucket walk (0)")
    p.add_argument("--max_frames", type=int, default=1800,
                   help="drop utterances longer than this (frames)")
    p.add_argument("--fault_inject_step", type=int, default=-1,
                   help="testing only: kill rank --fault_inject_rank at this step (first attempt of "
                        "an elastic job only, so a torchrun restart runs through)")
    p.add_argument("--fault_inject_rank", type=int, default=0)
    p.add_argument("--resume", type=str, default="none", choices=["none", "auto"],
                   help="auto: continue from the latest checkpoint in train_dir instead of wiping it "
                        "(implied when torchrun restarts the job: TORCHELASTIC_RESTART_COUNT > 0)")
    p.add_argument("--activation_summaries", type=str2bool, default=True,
                   help="activation histograms + sparsity at conv1/conv2/rnn/logits on summary steps")
    p.add_argument("--summaries_on_dummy", type=str2bool, default=False,
                   help="write summaries in --dummy mode too (the reference skips them there)")
    return p


def build_eval_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="DeepSpeech2 evaluation (CER) on MI355X")
    p.add_argument("--eval_dir", type=str, default="../models/librispeech/eval")
    p.add_argument("--checkpoint_dir", type=str, default="../models/librispeech/train")
    p.add_argument("--eval_data", type=str, default="val", help="'test' | 'val' | 'train'")
    p.add_argument("--batch_size", type=int, default=1)
    p.add_argument("--eval_interval_secs", type=int, default=60 * 5)
    p.add_argument("--data_dir", type=str, default="../data/LibriSpeech/processed/")
    p.add_argument("--run_once", type=str2bool, default=False)
    p.add_argument("--engine", type=str, default="tf")
    p.add_argument("--nchw", type=str2bool, default=True)
    # extensions
    p.add_argument("--dummy", type=str2bool, default=False, help="evaluate on synthetic data")
    p.add_argument("--decoder", type=str, default="greedy", choices=["greedy", "beam"])
    p.add_argument("--beam_width", type=int, default=16)
    p.add_argument("--use_ema", type=str2bool, default=True,
                   help="evaluate the EMA (shadow) weights like the reference")
    p.add_argument("--num_examples", type=int, default=0, help="override eval set size")
    p.add_argument("--device", type=str, default="auto")
    p.add_argument("--dtype", type=str, default="auto", choices=["auto", "fp32", "bf16"])
    p.add_argument("--display", type=str2bool, default=True)
    return p


def load_param_json(directory: str) -> Dict[str, Any]:
    with open(os.path.join(directory, "deepSpeech_parameters.json"), "r") as f:
        return json.load(f)


def apply_resume_params(args: argparse.Namespace, params: Dict[str, Any], keys) -> None:
    for k in keys:
        if k in params:
            setattr(args, k, params[k])


def parse_train_args(argv=None) -> argparse.Namespace:
    args = build_train_parser().parse_args(argv)
    if args.checkpoint is not None:
        # reference: src/deepSpeech_train.py:114-127 — architecture comes from the json
        apply_resume_params(args, load_param_json(args.checkpoint), RESUME_KEYS)
    return args


def parse_eval_args(argv=None) -> argparse.Namespace:
    args = build_eval_parser().parse_args(argv)
    params = load_param_json(args.checkpoint_dir)
    apply_resume_params(args, params, EVAL_KEYS)
    # reference-defaults for keys that may be missing in a json written by another tool
    for k, v in (("cell", "rnn_relu"), ("stack_fix", True), ("seq_bn", "frozen"),
                 ("ctc_collapse_repeated", True), ("moving_avg_decay", 0.9999)):
        if not hasattr(args, k):
            setattr(args, k, v)
    return args


def resolve_device(name: str):
    import torch
    if name == "auto":
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    return torch.device(name)


def resolve_engine(engine: str, device) -> str:
    """Map reference engine names onto {ref, hip}."""
    if engine in ("ref", "hip"):
        if engine == "hip" and device.type != "cuda":
            raise ValueError("engine=hip requires a GPU device")
        return engine
    if engine in ENGINE_ALIASES:
        return "hip" if device.type == "cuda" else "ref"
    raise ValueError("unknown engine %r" % engine)


def resolve_dtype(dtype: str, use_fp16: bool, device):
    import torch
    if dtype == "auto":
        if device.type == "cuda" or use_fp16:
            return torch.bfloat16 if device.type == "cuda" else torch.float32
        return torch.float32
    return {"fp32": torch.float32, "bf16": torch.bfloat16, "fp8": torch.bfloat16}[dtype]


def model_kwargs_from_args(args) -> Dict[str, Any]:
    bidir = str(getattr(args, "rnn_type", "bidirectional")) not in ("uni-dir", "unidirectional", "uni")
    return dict(
        num_filters=args.num_filters,
        num_hidden=args.num_hidden,
        num_rnn_layers=args.num_rnn_layers,
        cell=getattr(args, "cell", "rnn_relu"),
        bidirectional=bidir,
        stack_fix=getattr(args, "stack_fix", True),
        seq_bn=getattr(args, "seq_bn", "frozen"),
        layout="nchw" if str2bool(getattr(args, "nchw", True)) else "nhwc",
    )


def dump_param_json(args: argparse.Namespace, directory: str) -> str:
    """reference: src/deepSpeech_train.py:511-513 (json.dump(vars(ARGS)))."""
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, "deepSpeech_parameters.json")
    with open(path, "w") as f:
        json.dump(vars(args), f, sort_keys=True, indent=4, default=str)
    return path


def get_rnn_seqlen_py(seq_len: int) -> int:
    """Scalar version of get_rnn_seqlen (reference src/deepSpeech.py:38-48)."""
    import math
    t1 = math.ceil((seq_len - 19) / 2.0)
    return int(math.ceil((t1 - 9) / 2.0))


def maybe_int(x: Optional[str]) -> Optional[int]:
    return None if x is None else int(x)
