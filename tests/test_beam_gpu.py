"""GPU CTC prefix beam search (csrc/beam.hip) against the native host decoder
(runtime/decoder.cpp PrefixBeamSearch, itself checked against a brute-force path sum in
tests/test_native.py): same best prefixes and beam scores, whole-utterance and chunked."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lp(T, B, K, sharp, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.log_softmax(sharp * torch.randn(T, B, K, generator=g), -1)


def _host(lp, lens, W, blank, prune):
    from deepspeech_amd.runtime import native
    N = native.load()
    out = []
    for b in range(lp.shape[1]):
        bs = N.PrefixBeamSearch(W, blank, prune)
        bs.feed(lp[: int(lens[b]), b].contiguous().numpy())
        out.append(bs.results())
    return out


@pytest.mark.parametrize("W,prune,sharp", [(16, -10.0, 2.0), (8, -3.0, 3.0), (32, -10.0, 1.0), (1, -10.0, 2.0)])
def test_gpu_beam_matches_host(cuda, W, prune, sharp):
    from deepspeech_amd.ops.decode import GpuBeamSearch
    T, B, K, blank = 60, 6, 29, 28
    lp = _lp(T, B, K, sharp, seed=W)
    lens = torch.tensor([60, 41, 1, 60, 17, 33], dtype=torch.int32)
    gs = GpuBeamSearch(B, W, blank, prune, cuda, frames_hint=8)       # forces trie growth too
    gs.feed(lp.to(cuda), lens.to(cuda))
    got = gs.results()
    want = _host(lp, lens, W, blank, prune)
    for b in range(B):
        assert len(got[b]) == len(want[b]), b
        assert got[b][0][0] == want[b][0][0], (b, got[b][0], want[b][0])
        g = sorted(s for _, s in got[b])
        h = sorted(s for _, s in want[b])
        np.testing.assert_allclose(g, h, rtol=2e-5, atol=2e-5)
        assert {tuple(p) for p, _ in got[b]} == {tuple(p) for p, _ in want[b]}


def test_gpu_beam_chunked_equals_whole(cuda):
    """Streaming: feeding chunks of 1..13 frames gives bitwise the whole-utterance beams."""
    from deepspeech_amd.ops.decode import GpuBeamSearch
    T, B, K, blank = 80, 4, 29, 28
    lp = _lp(T, B, K, 2.0, seed=7).to(cuda)
    whole = GpuBeamSearch(B, 16, blank, -10.0, cuda, frames_hint=T)
    whole.feed(lp)
    parts = GpuBeamSearch(B, 16, blank, -10.0, cuda, frames_hint=4)
    t = 0
    for n in (1, 13, 7, 13, 13, 2, 13, 13, 5):
        parts.feed(lp[t:t + n])
        t += n
    assert t == T
    assert whole.results() == parts.results()
    parts.reset()
    parts.feed(lp)
    assert parts.best() == whole.best()


def test_beam_decode_routes_to_gpu_and_streaming_recognizer(cuda):
    """ops.decode.beam_decode on device logits uses the GPU search; the streaming recogniser's
    beam transcript equals beam_decode over the whole stream's log-probs. (No host comparison
    here: a random-init model's near-uniform frames are full of near-ties, which the last ulp of
    expf / log1pf, device vs glibc, orders either way, and the searches then diverge; the host
    parity is pinned on distinct scores in test_gpu_beam_matches_host.)"""
    from deepspeech_amd.infer import StreamingRecognizer
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.ops.decode import beam_decode
    torch.manual_seed(0)
    m = DeepSpeech2(num_filters=32, num_hidden=128, num_rnn_layers=2, cell="gru", bidirectional=False).to(cuda)
    m.set_engine("hip", torch.bfloat16)
    rec = StreamingRecognizer(m, decoder="beam", beam_width=16, batch=2)
    assert rec.gbeams is not None
    feats = torch.randn(2, 50 * 6 + 38, m.freq_bins, device=cuda)
    for i in range(0, feats.shape[1], 50):
        rec.accept(feats[:, i:i + 50])
    got = rec.finish()
    lp = torch.cat(rec.logprobs, 0)
    lens = torch.full((2,), lp.shape[0], dtype=torch.int32)
    assert got == beam_decode(lp, lens, 16)
    assert all(len(g) > 0 for g in got)
