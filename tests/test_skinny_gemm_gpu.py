"""Decode skinny GEMM (csrc/kernels/skinny_gemm.hip) vs an fp32 PyTorch reference: M <= 16 rows,
ragged N / K tails, strided activation rows, bias; and the ops.linear dispatch under no_grad."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _native():
    from shuffle_exchange_amd.ops import native
    native.require_hip()


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("N,K", [(16, 8), (100, 264), (4104, 4096), (1000, 14336), (33, 1032)])
@pytest.mark.parametrize("with_bias", [False, True])
def test_skinny_gemm_matches_fp32(M, N, K, with_bias):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    xs = torch.randn(M, K + 16, device="cuda", dtype=torch.bfloat16, generator=g)
    x = xs[:, :K]  # row stride K + 16
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16, generator=g) if with_bias else None
    y = torch.ops.sxe.skinny_gemm(x, w, b)
    ref = x.float() @ w.float().t() + (b.float() if b is not None else 0)
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-2, err


def test_linear_dispatches_skinny_under_no_grad():
    from shuffle_exchange_amd.ops.linear import linear
    w = torch.randn(256, 512, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(2, 3, 512, device="cuda", dtype=torch.bfloat16)
    with torch.no_grad():
        y = linear(x, w)
    assert y.shape == (2, 3, 256)
    torch.testing.assert_close(y.float(), (x.float() @ w.float().t()), atol=0.25, rtol=2e-2)
    xg = x.clone().requires_grad_()
    linear(xg, w).sum().backward()  # autograd path still works (F.linear)
    assert xg.grad is not None
