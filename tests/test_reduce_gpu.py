"""csrc/reduce.hip against fp32 PyTorch: the recurrent bias-gradient sums (col_sum) and the FC
head's bias gradient (fc_bias_grad), which replaced torch reduce / multiply / copy kernels in the
training step. Reference: src/custom_ops.py:68-71 (recurrent bias),
src/deepSpeech_NCHW.py:188-198 (softmax_linear/biases)."""
import pytest
import torch

from deepspeech_amd.ops import _ext

pytestmark = pytest.mark.gpu


def test_col_sum_multi_job(cuda):
    C = _ext.ext()
    torch.manual_seed(0)
    ins = [torch.randn(2, 4, 2400, device=cuda), torch.randn(2, 4, 2400, device=cuda), torch.randn(1, 16, 29 * 800,
                                                                                                  device=cuda)]
    outs = [torch.empty(2 * 2400, device=cuda), torch.randn(2 * 2400, device=cuda), torch.empty(29 * 800, device=cuda)]
    base = outs[1].clone()
    C.col_sum(ins, outs, [False, True, False])
    torch.cuda.synchronize()
    want = [ins[0].double().sum(1).reshape(-1), base.double() + ins[1].double().sum(1).reshape(-1),
            ins[2].double().sum(1).reshape(-1)]
    for o, w in zip(outs, want):
        assert torch.allclose(o.double(), w, rtol=1e-5, atol=1e-5), (o.double() - w).abs().max()
    # fixed summation order: bitwise reproducible
    again = [torch.empty_like(outs[0])]
    C.col_sum([ins[0]], again, [False])
    assert torch.equal(again[0], outs[0])


@pytest.mark.parametrize("M,K", [(7712, 29), (100, 29), (33, 7)])
def test_fc_bias_grad(cuda, M, K):
    C = _ext.ext()
    torch.manual_seed(1)
    G = torch.randn(M, 32, device=cuda).bfloat16()
    scale = torch.tensor([0.75], device=cuda)
    out = torch.empty(K, device=cuda)
    C.fc_bias_grad(G, K, scale, 1.0 / 32, out, False)
    want = G[:, :K].double().sum(0) * 0.75 / 32
    torch.cuda.synchronize()
    assert torch.allclose(out.double(), want, rtol=1e-5, atol=1e-5), (out.double() - want).abs().max()
    prev = out.clone()
    C.fc_bias_grad(G, K, scale, 1.0 / 32, out, True)
    assert torch.allclose(out.double(), prev.double() + want, rtol=1e-5, atol=1e-5)
