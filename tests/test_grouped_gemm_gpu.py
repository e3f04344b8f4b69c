"""Grouped expert GEMM tile variants (csrc/kernels/grouped_gemm.hip) against an fp32 PyTorch
reference: the 128 x 128 register-staged kernel and the LDS-DMA 256 x 256 kernel with 4 and 8 waves
(SXE_GG_TILE / SXE_GG_WN, read per call), ragged expert segments (empty, one row, tile tails), with
and without the fused per-row routing scale. All of them store transposed accumulators (one 8-byte
store per 4 columns), so an asymmetric weight catches a swapped row / column map."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from shuffle_exchange_amd.ops import native
    native.require_hip()


def _ref(x, w, offs, s):
    out = torch.zeros(x.shape[0], w.shape[1], device=x.device)
    o = offs.tolist()
    for e in range(w.shape[0]):
        a, b = o[e], o[e + 1]
        if b > a:
            out[a:b] = x[a:b].float() @ w[e].float().t()
    if s is not None:
        out = out * s.float()[:, None]
    return out


@pytest.mark.parametrize("tile,wn", [("128", None), ("256", "2"), ("256", "4")])
@pytest.mark.parametrize("counts", [[0, 300, 1, 257, 0, 77, 513, 2], [512, 256]])
@pytest.mark.parametrize("scale", [None, "fp32", "bf16"])
def test_grouped_gemm_tiles(tile, wn, counts, scale, monkeypatch):
    from shuffle_exchange_amd.ops import moe as moe_ops
    monkeypatch.setenv("SXE_GG_DISPATCH", "kernel")
    monkeypatch.setenv("SXE_GG_TILE", tile)
    if wn:
        monkeypatch.setenv("SXE_GG_WN", wn)
    torch.manual_seed(len(counts))
    E, N, K = len(counts), 512, 384
    R = sum(counts)
    x = torch.randn(R, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(E, N, K, device="cuda", dtype=torch.bfloat16) / 16
    offs = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device="cuda")
    s = None
    if scale:
        s = torch.rand(R, device="cuda", dtype=torch.float32 if scale == "fp32" else torch.bfloat16)
    y = moe_ops.grouped_gemm(x, w, offs, s)
    ref = _ref(x, w, offs, s)
    err = ((y.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, (tile, wn, err)


@pytest.mark.parametrize("tile", ["128", "256"])
def test_grouped_gemm_identity(tile, monkeypatch):
    """X = I per expert segment, W asymmetric small integers: Y rows are exactly the weight columns."""
    from shuffle_exchange_amd.ops import moe as moe_ops
    monkeypatch.setenv("SXE_GG_DISPATCH", "kernel")
    monkeypatch.setenv("SXE_GG_TILE", tile)
    E, N, K = 2, 256, 256
    x = torch.eye(K, device="cuda", dtype=torch.bfloat16).repeat(E, 1)
    w = ((torch.arange(E * N * K, device="cuda").reshape(E, N, K) % 7) - 3).to(torch.bfloat16)
    offs = torch.tensor([0, K, 2 * K], dtype=torch.int32, device="cuda")
    y = moe_ops.grouped_gemm(x, w, offs, None)
    ref = torch.cat([w[e].float().t() for e in range(E)])
    torch.testing.assert_close(y.float(), ref, rtol=0, atol=0)
