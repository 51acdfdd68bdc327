"""Hand-written MFMA GEMM family (csrc/gemm.hip) against fp32 PyTorch references.

Every operand layout (row/col) and epilogue (bf16 + alpha + bias, fp32 store, fp32
accumulate), every tile configuration, ragged M/N tails, a K that ends in half a k-tile
(K % 64 == 32) and a batched call. Operands are asymmetric random data so a transposed
or swapped store cannot pass.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from deepspeech_amd.ops import gemm as G  # noqa: E402

DEV = torch.device("cuda:0")
BF = torch.bfloat16


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("M,N,K", [(7712, 800, 800), (300, 328, 96), (517, 1040, 2400), (390, 192, 72)])
def test_linear_bias_alpha(cfg, M, N, K):
    torch.manual_seed(cfg * 7 + M)
    x = torch.randn(M, K, device=DEV).to(BF)
    W = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = torch.randn(N, device=DEV).to(BF)
    out = G.gemm(x, W, torch.empty(M, N, device=DEV, dtype=BF), M, N, K, False, False, 0, 0.75, b, cfg=cfg)
    ref = 0.75 * (x.float() @ W.float().t()) + b.float()
    assert _rel(out, ref) < 6e-3


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("M,N,K", [(7712, 800, 4800), (200, 256, 160), (333, 2400, 4800), (390, 192, 200)])
def test_mm_nn(cfg, M, N, K):
    torch.manual_seed(cfg + N)
    a = torch.randn(M, K, device=DEV).to(BF)
    b = (torch.randn(K, N, device=DEV) * 0.05).to(BF)
    out = G.gemm(a, b, torch.empty(M, N, device=DEV, dtype=BF), M, N, K, False, True, 0, 1.0, None, cfg=cfg)
    ref = a.float() @ b.float()
    assert _rel(out, ref) < 6e-3


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("M,N,K", [(4800, 800, 7712), (2400, 800, 7712), (136, 264, 96), (192, 64 * 4, 390),
                                   (136, 128, 8)])
def test_mm_tn_store_and_accumulate(cfg, M, N, K):
    torch.manual_seed(cfg + K)
    a = torch.randn(K, M, device=DEV).to(BF)
    b = torch.randn(K, N, device=DEV).to(BF)
    ref = a.float().t() @ b.float()
    out = torch.full((M, N), float("nan"), device=DEV)
    G.gemm(a, b, out, M, N, K, True, True, 1, 1.0, None, cfg=cfg)
    assert _rel(out, ref) < 2e-5 * K ** 0.5 + 1e-4
    if cfg >= 6:
        return          # persistent configurations: no read-modify-write epilogue
    G.gemm(a, b, out, M, N, K, True, True, 2, 0.5, None, cfg=cfg)
    assert _rel(out, 1.5 * ref) < 2e-5 * K ** 0.5 + 1e-4


def test_mm_tn_batched_strided_output():
    """Both directions' dU in one launch, written into a strided slice of a bigger buffer."""
    torch.manual_seed(3)
    K, M, N = 7712, 2400, 800
    a = torch.randn(2, K, M, device=DEV).to(BF)
    b = torch.randn(2, K, N, device=DEV).to(BF)
    big = torch.zeros(2, M, N + 64, device=DEV)
    out = big[:, :, 32:32 + N]
    G.mm_tn(a, b, out)
    ref = torch.bmm(a.float().transpose(1, 2), b.float())
    assert _rel(out, ref) < 2e-3
    assert float(big[:, :, :32].abs().max()) == 0.0 and float(big[:, :, 32 + N:].abs().max()) == 0.0


def test_row_stride_views():
    """Operands given as column slices of wider matrices (leading dimension > K)."""
    torch.manual_seed(5)
    M, K, N = 1000, 800, 2400
    xw = torch.randn(M, K + 64, device=DEV).to(BF)
    x = xw[:, 64:]
    W = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    out = G.linear(x, W)
    assert _rel(out, x.float() @ W.float().t()) < 6e-3
