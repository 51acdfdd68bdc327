"""Evaluation driver (CER), CLI-compatible with the reference's deepSpeech_test.py.

  python -m deepspeech_amd.test --eval_data test --checkpoint_dir ../models/librispeech/train \
      --data_dir ../data/LibriSpeech/processed/ --run_once True [--decoder beam]

Reference flow (src/deepSpeech_test.py:139-241): architecture from the checkpoint dir's
deepSpeech_parameters.json, restore the EMA (shadow) weights, log-softmax + greedy CTC
decode over get_rnn_seqlen lengths, CER = Levenshtein(label, pred)/len(label) per
utterance averaged over the set (2048 train / 2703 val / 2620 test examples), print the
pairs, write a 'char_err_rate' summary, loop every eval_interval_secs unless run_once.
Eval-mode BN uses running statistics (quirk Q4 fixed).
"""
from __future__ import annotations

import math
import os
import shutil
import sys
import time
from datetime import datetime
from typing import List

import numpy as np
import torch

from . import ALPHABET, BLANK
from . import config as C
from .data.synthetic import DummyBucketWalk, to_device
from .models import DeepSpeech2
from .ops import reference as R
from .utils import checkpoint as CK
from .utils.summary import EventWriter, JsonlWriter

NUM_EXAMPLES = {"train": 2048, "val": 2703, "test": 2620}
IX_TO_CHAR = {i: c for i, c in enumerate(ALPHABET)}


def ids_to_text(ids) -> str:
    return "".join(IX_TO_CHAR.get(int(i), "") for i in ids)


def levenshtein(a, b) -> int:
    try:
        from .runtime import native
        N = native.load()
        if isinstance(a, str):
            return int(N.levenshtein(a, b))
        return int(N.levenshtein_ids(list(a), list(b)))
    except RuntimeError:
        prev = list(range(len(b) + 1))
        for i in range(1, len(a) + 1):
            cur = [i] + [0] * len(b)
            for j in range(1, len(b) + 1):
                cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (a[i - 1] != b[j - 1]))
            prev = cur
        return prev[-1]


def decode(logits: torch.Tensor, lens: torch.Tensor, decoder: str, beam_width: int) -> List[List[int]]:
    from .ops import decode as D
    if decoder == "greedy":
        if logits.is_cuda:
            return D.greedy_decode(logits, lens)          # csrc/decode.hip
        lp = torch.log_softmax(logits.float(), dim=-1)
        try:
            from .runtime import native
            best = lp.argmax(-1).to(torch.int32).cpu().numpy()
            return native.load().greedy_collapse(best, lens.cpu().numpy().astype(np.int32), BLANK)
        except RuntimeError:
            return R.greedy_decode(lp, lens)
    return D.beam_decode(logits, lens, beam_width, BLANK, -10.0)


def eval_once(model, args, data, num_iter: int, display: bool) -> float:
    model.eval()
    cers = []
    with torch.no_grad():
        for step in range(num_iter):
            hb = data.next()
            b = to_device(hb, model.fc_weight.device)
            logits, lens = model(b["feats"], b["seq_lens"])
            preds = decode(logits, lens, args.decoder, args.beam_width)
            if model.engine == "hip":
                # decode() synchronised already: surface a recurrence timeout (undefined
                # outputs) for this batch instead of reporting a CER computed from them
                from .ops import rnn as RNN
                RNN.check_errors()
            for i, p in enumerate(preds):
                lab = hb.labels[i, : hb.label_lens[i]].tolist()
                ref_s, hyp_s = ids_to_text(lab), ids_to_text(p)
                cers.append(levenshtein(ref_s, hyp_s) / max(1, len(ref_s)))
                if display and i < 2:
                    print(ref_s + " vs " + hyp_s)
    return float(np.mean(cers)) * 100.0 if cers else float("nan")


def build_eval_data(args):
    if args.dummy:
        return DummyBucketWalk(args.batch_size, seed=4321)
    from .data.store import StoreBatches, find_partition_files, find_store, tfrecords_to_store
    prefix = find_store(args.data_dir, args.eval_data)
    if prefix is None:
        files = find_partition_files(args.data_dir, args.eval_data)
        if not files:
            raise ValueError("no %s data under %s" % (args.eval_data, args.data_dir))
        prefix = os.path.join(args.eval_dir, "cache", args.eval_data)
        if not os.path.exists(prefix + ".index.npz"):
            tfrecords_to_store(files, prefix)
    return StoreBatches(prefix, args.batch_size, shuffle=True, sortagrad_epochs=0, max_frames=10 ** 9)


def main(argv=None) -> int:
    args = C.parse_eval_args(argv)
    dev = C.resolve_device(args.device)
    engine = C.resolve_engine(args.engine, dev)
    dtype = C.resolve_dtype(args.dtype, False, dev)
    print("nchw: ", args.nchw)
    print("engine: ", args.engine, "->", engine)
    if os.path.isdir(args.eval_dir):
        shutil.rmtree(args.eval_dir)        # reference wipes eval_dir (src/deepSpeech_test.py:238-240)
    os.makedirs(args.eval_dir, exist_ok=True)
    model = DeepSpeech2(**C.model_kwargs_from_args(args)).to(dev)
    model.set_engine(engine, dtype)
    data = build_eval_data(args)
    n = args.num_examples or NUM_EXAMPLES.get(args.eval_data, 2048)
    num_iter = int(math.ceil(n / args.batch_size))
    events = EventWriter(args.eval_dir)
    jl = JsonlWriter(os.path.join(args.eval_dir, "eval.jsonl"))
    while True:
        path = CK.latest_checkpoint(args.checkpoint_dir)
        if path is None:
            print("No checkpoint file found")
        else:
            tensors = {k: v for k, v in CK.load_checkpoint_file(path).items() if isinstance(v, torch.Tensor)}
            CK.load_model_from_tf(model, tensors, strict=True, use_ema=args.use_ema)
            step = CK.step_from_path(path)
            cer = eval_once(model, args, data, num_iter, args.display)
            print("%s: char_err_rate = %.3f %%" % (datetime.now(), cer), flush=True)
            events.scalars(step, {"char_err_rate": cer})
            jl.write(step, char_err_rate=cer, checkpoint=os.path.basename(path))
        if args.run_once:
            break
        time.sleep(args.eval_interval_secs)
    events.close()
    if hasattr(data, "close"):
        data.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
