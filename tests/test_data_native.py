"""Input pipeline, native runtime (loader / TFRecord / decoders), featurizer, summaries."""
import itertools
import math
import os

import numpy as np
import pytest
import torch

from deepspeech_amd import BLANK, NUM_CLASSES
from deepspeech_amd.config import get_rnn_seqlen_py
from deepspeech_amd.data import synthetic as S
from deepspeech_amd.runtime import native

N = native.load()


def test_dummy_bucket_walk_follows_reference_tables():
    g = S.DummyBucketWalk(batch_size=4, seed=0, scale_factor=1)
    seen = []
    for _ in range(g.steps_per_epoch()):
        b = g.next()
        assert b.feats.shape[1:] == (b.seq_lens[0], 161)
        assert (b.labels < NUM_CLASSES - 1).all()           # Q6 fixed: no blank in labels
        L = int(b.label_lens[0]); lab = b.labels[0, :L]
        assert L + int((lab[1:] == lab[:-1]).sum()) <= get_rnn_seqlen_py(int(b.seq_lens[0]))
        seen.append(int(b.seq_lens[0]))
    # ascending bucket walk of utt_lengths with counts*scale*batch utterances per bucket
    assert seen[0] == 100 and seen[-1] == 1500
    assert g.utterances_per_epoch == sum(S.COUNTS) * 4


def test_fixed_shape_batches():
    f = S.FixedShapeBatches(8, max_frames=1000, seed=0, pool=2)
    b = f.next()
    assert b.feats.shape == (8, 1000, 161) and b.seq_lens.max() == 1000 and b.seq_lens.min() > 900
    assert (b.feats[np.arange(8), np.minimum(b.seq_lens, 999)][b.seq_lens < 1000] == 0).all()
    assert 14 < b.label_lens.mean() / (b.seq_lens.mean() / 100) < 16


def test_plan_batches_sorted_and_distributed():
    rng = np.random.default_rng(0)
    lens = rng.integers(100, 1800, size=400).astype(np.int32)
    plan = N.plan_batches(lens, np.zeros(400, np.int32), 8, 100, 1800, True, 0, 2, True)
    # sorted: nondecreasing bucket order; the 2 batches of a step share a bucket
    buckets = [lens[b[0]] // 100 for b in plan]
    assert buckets == sorted(buckets)
    for i in range(0, len(plan) - 1, 2):
        assert lens[plan[i][0]] // 100 == lens[plan[i + 1][0]] // 100
    assert all(len(b) == 8 for b in plan)
    assert len(set(itertools.chain(*plan))) == sum(len(b) for b in plan)   # no duplicates
    shuf = N.plan_batches(lens, np.zeros(400, np.int32), 8, 100, 1800, False, 1, 1, True)
    assert [lens[b[0]] // 100 for b in shuf] != sorted(lens[b[0]] // 100 for b in shuf)
    # infeasible / too long utterances are dropped
    mf = np.full(400, 10 ** 6, np.int32)
    assert N.plan_batches(lens, mf, 8, 100, 1800, True, 0, 1, True) == []


def _make_store(tmp_path, n=40, seed=0):
    from deepspeech_amd.data.store import StoreWriter
    rng = np.random.default_rng(seed)
    w = StoreWriter(str(tmp_path / "train-clean"))
    utts = []
    for i in range(n):
        T = int(rng.integers(150, 600))
        f = rng.standard_normal((T, 161)).astype(np.float32)
        lab = rng.integers(0, 28, size=int(rng.integers(5, 20))).astype(np.int32)
        w.add(f, lab)
        utts.append((f, lab))
    return w.close(), utts


def test_store_and_threaded_loader(tmp_path):
    from deepspeech_amd.data.store import StoreBatches
    prefix, utts = _make_store(tmp_path)
    sb = StoreBatches(prefix, batch_size=4, num_threads=3, sortagrad_epochs=1, shuffle=False)
    seen = 0
    for _ in range(5):
        b = sb.next()
        assert b.feats.shape[0] == 4 and b.feats.shape[2] == 161
        for i in range(4):
            T, L = int(b.seq_lens[i]), int(b.label_lens[i])
            match = [j for j, (f, l) in enumerate(utts) if f.shape[0] == T and len(l) == L and (l == b.labels[i, :L]).all()]
            assert match, "batch row not found in store"
            assert np.array_equal(b.feats[i, :T], utts[match[0]][0])
            assert (b.feats[i, T:] == 0).all()
            seen += 1
    sb.close()
    assert seen == 20


def test_tfrecord_roundtrip_reference_format(tmp_path):
    from deepspeech_amd.data.store import StoreIndex, store_to_tfrecords, tfrecords_to_store
    prefix, utts = _make_store(tmp_path, n=6)
    path = store_to_tfrecords(prefix, str(tmp_path / "dev.tfrecords"))
    recs = N.read_records(path, True)
    assert len(recs) == 6
    seq_len, labels, feats = N.parse_sequence_example(recs[2], "feats")
    assert seq_len == utts[2][0].shape[0] and np.array_equal(feats, utts[2][0])
    assert np.array_equal(labels, utts[2][1])
    p2 = tfrecords_to_store([path], str(tmp_path / "again"))
    ix = StoreIndex.load(p2)
    assert ix.lengths.tolist() == [u[0].shape[0] for u in utts]
    # CRC check catches corruption
    raw = bytearray(open(path, "rb").read())
    raw[30] ^= 0xFF
    open(tmp_path / "bad.tfrecords", "wb").write(bytes(raw))
    with pytest.raises(RuntimeError):
        N.read_records(str(tmp_path / "bad.tfrecords"), True)


def test_crc32c_known_vector():
    assert N.crc32c(b"123456789") == 0xE3069283


def test_levenshtein_and_greedy():
    assert N.levenshtein("KITTEN", "SITTING") == 3
    assert N.levenshtein_ids([1, 2, 3], [1, 3]) == 1
    best = np.array([[1, 1, BLANK, 1, 2, 2, BLANK]], np.int32).T     # [T, N=1]
    assert N.greedy_collapse(best, np.array([7], np.int32), BLANK) == [[1, 1, 2]]
    assert N.greedy_collapse(best, np.array([3], np.int32), BLANK) == [[1]]


def _brute_force_ctc_best(lp, blank):
    T, K = lp.shape
    scores = {}
    for path in itertools.product(range(K), repeat=T):
        out, prev = [], None
        for c in path:
            if c != prev and c != blank:
                out.append(c)
            prev = c
        p = sum(lp[t, c] for t, c in enumerate(path))
        key = tuple(out)
        scores[key] = np.logaddexp(scores.get(key, -np.inf), p)
    return max(scores.items(), key=lambda kv: kv[1])


def test_prefix_beam_search_exact_for_wide_beam():
    rng = np.random.default_rng(3)
    for _ in range(3):
        lp = np.log(rng.dirichlet(np.ones(3), size=5)).astype(np.float32)
        bs = N.PrefixBeamSearch(64, 2, -1e9)
        bs.feed(lp)
        best, score = bs.results()[0]
        ref, rscore = _brute_force_ctc_best(lp.astype(np.float64), 2)
        assert tuple(best) == ref and abs(score - rscore) < 1e-4
        # streaming: feeding in chunks gives the same result
        bs2 = N.PrefixBeamSearch(64, 2, -1e9)
        bs2.feed(lp[:2]); bs2.feed(lp[2:])
        assert bs2.best() == list(ref)


def test_beam_search_batch_threads_and_streaming_match_single():
    rng = np.random.default_rng(11)
    T, B, K = 40, 6, 29
    lp = np.log(rng.dirichlet(np.ones(K) * 0.3, size=(T, B))).astype(np.float32)   # [T, B, K]
    lens = np.array([40, 33, 17, 40, 1, 25], np.int32)
    single = []
    for b in range(B):
        bs = N.PrefixBeamSearch(8, 28, -8.0)
        bs.feed(np.ascontiguousarray(lp[: lens[b], b]))
        single.append(bs.best())
    for threads in (1, 4):
        assert N.beam_search_batch(lp, lens, 8, 28, -8.0, threads) == single
    # incremental (streaming) batch decoder: chunks of 15 frames, per-chunk valid lengths
    bb = N.BatchBeamSearch(B, 8, 28, -8.0, 3)
    for s in range(0, T, 15):
        chunk = np.ascontiguousarray(lp[s:s + 15])
        bb.feed(chunk, np.clip(lens - s, 0, chunk.shape[0]).astype(np.int32))
    assert bb.best() == single


def test_featurizer_mfcc_shape_and_dct():
    from scipy.fft import dct
    from deepspeech_amd.data import featurizer as FZ
    x = np.random.default_rng(0).standard_normal((4, 12))
    assert np.allclose(FZ._dct2_ortho(x), dct(x, type=2, axis=-1, norm="ortho"))
    sig = np.sin(np.arange(16000) * 2 * np.pi * 440 / 16000)
    m = FZ.compute_features(sig, 16000, "mfcc")
    assert m.shape == (99, 161) and np.isfinite(m).all()
    s = FZ.compute_features(sig, 16000, "spectrogram")
    assert s.shape[1] == 161


def test_preprocess_partition_wav(tmp_path):
    from scipy.io import wavfile
    from deepspeech_amd.data.preprocess import process_partition
    from deepspeech_amd.data.store import StoreIndex
    d = tmp_path / "audio" / "dev-clean" / "1" / "2"
    d.mkdir(parents=True)
    rng = np.random.default_rng(0)
    lines = []
    for i, text in enumerate(["HELLO WORLD", "A B", "DEEP SPEECH TWO"]):
        wavfile.write(str(d / ("1-2-%04d.wav" % i)), 16000,
                      (rng.standard_normal(16000 * (i + 1) // 2) * 1000).astype(np.int16))
        lines.append("1-2-%04d %s" % (i, text))
    (d / "1-2.trans.txt").write_text("\n".join(lines) + "\n")
    stats = process_partition(str(tmp_path / "audio" / "dev-clean"), str(tmp_path / "out" / "dev-clean"),
                              tfrecord_dir=str(tmp_path / "out"))
    assert stats["utterances"] == 3
    ix = StoreIndex.load(str(tmp_path / "out" / "dev-clean"))
    assert list(ix.lengths) == sorted(ix.lengths)            # SortaGrad order
    assert os.path.exists(tmp_path / "out" / "dev-clean" / "dev-clean.tfrecords")


def test_event_file_roundtrip(tmp_path):
    from deepspeech_amd.utils.summary import EventWriter, read_events
    w = EventWriter(str(tmp_path))
    w.scalars(5, {"loss": 1.5, "lr": 0.25})
    w.histogram(5, "w", np.arange(10.0))
    w.close()
    ev = read_events(w.path)
    assert (5, "loss", 1.5) in ev and (5, "lr", 0.25) in ev


def test_lr_schedule_staircase():
    from deepspeech_amd.ops.optim import exponential_decay
    assert exponential_decay(1e-4, 0, 10, 0.9) == 1e-4
    assert exponential_decay(1e-4, 9, 10, 0.9) == 1e-4
    assert abs(exponential_decay(1e-4, 25, 10, 0.9) - 1e-4 * 0.81) < 1e-12


def test_cpu_adam_matches_tf_formula():
    from deepspeech_amd.ops.optim import FusedAdamEMA, ParamArena
    lin = torch.nn.Linear(3, 1, bias=False)
    with torch.no_grad():
        lin.weight.copy_(torch.tensor([[1.0, 2.0, 3.0]]))
    arena = ParamArena(lin)
    opt = FusedAdamEMA(arena, betas=(0.9, 0.999), eps=1e-8, ema_decay=0.9999)
    g = torch.tensor([0.5, -1.0, 2.0])
    lin.weight.grad.copy_(g.view(1, 3))
    opt.step(lr=0.1, global_step=0)
    m = 0.1 * g
    v = 0.001 * g * g
    lr_t = 0.1 * math.sqrt(1 - 0.999) / (1 - 0.9)
    exp = torch.tensor([1.0, 2.0, 3.0]) - lr_t * m / (v.sqrt() + 1e-8)
    assert torch.allclose(lin.weight.view(-1), exp, atol=1e-6)
    keep = min(0.9999, 1 / 10)
    assert torch.allclose(opt.ema[:3], exp + keep * (torch.tensor([1.0, 2, 3]) - exp), atol=1e-6)
