"""gfx950 block-scaled MX GEMM (csrc/kernels/mx_gemm.hip) against an fp32 PyTorch reference of the
same op: the operands are dequantised exactly (ops/mx.py) and multiplied in fp32, so the only
differences are the MFMA's fp32 accumulation order and the bf16 output rounding."""
import pytest
import torch

from shuffle_exchange_amd.ops import mx

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from shuffle_exchange_amd.ops import native
    native.require_hip()


def test_activation_quant_matches_reference():
    torch.manual_seed(0)
    x = (torch.randn(37, 512, device="cuda") * torch.logspace(-4, 4, 37, device="cuda")[:, None]).to(torch.bfloat16)
    x[3, 64:96] = 0
    q, s = torch.ops.sxe.mx_quant_fp8(x)
    rq, rs = mx.quantize(x.float().cpu(), "mxfp8")
    assert torch.equal(s.cpu(), rs)
    assert torch.equal(q.cpu(), rq)


@pytest.mark.parametrize("fmt", ["mxfp8", "mxfp6", "mxfp6_e2m3", "mxfp4"])
@pytest.mark.parametrize("M,N,K", [(1, 128, 128), (17, 384, 256), (300, 256, 1024), (1024, 1024, 512), (2048, 4096, 256)])
def test_mx_gemm_matches_fp32(fmt, M, N, K):
    torch.manual_seed(M + N + K)
    w = torch.randn(N, K, device="cuda") * 0.05
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    cs = torch.rand(N, device="cuda") + 0.5
    W = mx.MXWeight(w, fmt)
    q, s = torch.ops.sxe.mx_quant_fp8(x)
    y = torch.ops.sxe.mx_gemm(q, s, W.q, W.scale, mx.FORMATS[fmt][0], b, cs)
    ref = (mx.dequantize(q, s, "mxfp8", K) @ mx.dequantize(W.q, W.scale, fmt, K).t()) * cs + b.float()
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-3, err
    # no bias / scale path, through MXWeight.linear (<= 16 rows: weight-only skinny path, bf16
    # activations; more rows: MXFP8 activations on the block-scaled GEMM)
    y2 = W.linear(x)
    xa = x.float() if (M <= 16 and fmt != "mxfp6_e2m3") else mx.dequantize(q, s, "mxfp8", K)
    ref2 = xa @ W.dequantize(torch.float32).t()
    assert (y2.float() - ref2).abs().max().item() <= 1e-2 * ref2.abs().max().item() + 1e-3


def test_mx_gemm_asymmetric_identity():
    # A = I (exact in e4m3), B asymmetric integers (exact in every format): Y must be W itself,
    # which catches any row/column swap in the epilogue or operand maps
    K = N = 256
    x = torch.eye(K, device="cuda").to(torch.bfloat16)
    w = (torch.arange(N * K, device="cuda").reshape(N, K) % 7 - 3).float()
    for fmt in ["mxfp8", "mxfp6", "mxfp4"]:
        W = mx.MXWeight(w, fmt)
        y = W.linear(x)
        torch.testing.assert_close(y.float(), mx.dequantize(W.q, W.scale, fmt, K).t(), rtol=0, atol=0)


@pytest.mark.parametrize("bits", [6, 4])
@pytest.mark.parametrize("M,N,K", [(17, 128, 128), (300, 384, 1024), (2048, 1024, 512), (1030, 4096, 256)])
def test_fpx_weight_prefill_on_mx_gemm(bits, M, N, K, monkeypatch):
    """FPxWeight (FP6-LLM bit planes) with > 16 rows: the planes go straight into the block-scaled
    MFMA GEMM (exact e3m2 / e2m1 -> e4m3 transcode in registers, MXFP8 activations, per-row scale in
    the epilogue); reference = MXFP8(x) @ the fp32-decoded weight, no bf16 weight is materialised."""
    from shuffle_exchange_amd.ops.fp_quantizer import FPxWeight
    torch.manual_seed(bits + M + N)
    w = torch.randn(N, K, device="cuda") * 0.05
    W = FPxWeight(w.bfloat16(), bits)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    # the only way to a bf16 weight is FPxWeight.dequantize (fpxw_unpack): refuse it during linear
    real_deq = FPxWeight.dequantize

    def refuse(self, *a, **k):
        raise AssertionError("FPxWeight.linear materialised a dequantised weight")
    monkeypatch.setattr(FPxWeight, "dequantize", refuse)
    y = W.linear(x, b)
    monkeypatch.setattr(FPxWeight, "dequantize", real_deq)
    q, s = torch.ops.sxe.mx_quant_fp8(x)
    ref = mx.dequantize(q, s, "mxfp8", K) @ W.dequantize(torch.float32).t() + b.float()
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-3, err
    full = x.float() @ W.dequantize(torch.float32).t() + b.float()
    assert ((y.float() - full).norm() / full.norm()).item() < 0.05  # fp8 activations: a small, bounded change


@pytest.mark.parametrize("kind", ["mxfp8", "mxfp6", "mxfp4", "int8", "int4"])
@pytest.mark.parametrize("M,N,K", [(1, 128, 128), (5, 384, 1024), (16, 4096, 4096), (3, 1000, 512)])
def test_skinny_dequant_decode(kind, M, N, K):
    """<= 16-row GEMMs over MX / int weights (csrc/kernels/skinny_dq.hip): bf16 activations (weight
    only), codes decoded in registers; reference = x @ the fp32-decoded weight."""
    from shuffle_exchange_amd.ops.fp_quantizer import quantized_weight
    if kind.startswith("mx") and N % 128:
        N = 1024
    torch.manual_seed(M * 7 + N + K)
    w = torch.randn(N, K, device="cuda") * 0.05
    W = quantized_weight(w, kind)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    y = W.linear(x, b)
    wd = W.dequantize(torch.float32)
    ref = x.float() @ wd.t() + b.float()
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 2e-3, err


@pytest.mark.parametrize("tile", [1, 2, 5, 6, 7, 8, 9, 10])
@pytest.mark.parametrize("M,N,K", [(300, 256, 1024), (2048, 512, 384), (513, 768, 128), (256, 4096, 2048)])
def test_mx_gemm_tile_variants(tile, M, N, K, monkeypatch):
    """Every tile variant of the e4m3 path (SXE_MX_TILE, read per call) against the fp32 reference,
    with a bias and a per-column scale: ragged M, one / two / many K stages, N not a multiple of 256
    (variants needing 256 fall back)."""
    monkeypatch.setenv("SXE_MX_TILE", str(tile))
    torch.manual_seed(tile + M + N + K)
    w = torch.randn(N, K, device="cuda") * 0.05
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    cs = torch.rand(N, device="cuda") + 0.5
    W = mx.MXWeight(w, "mxfp8")
    q, s = torch.ops.sxe.mx_quant_fp8(x)
    y = torch.ops.sxe.mx_gemm(q, s, W.q, W.scale, mx.FORMATS["mxfp8"][0], b, cs)
    ref = (mx.dequantize(q, s, "mxfp8", K) @ mx.dequantize(W.q, W.scale, "mxfp8", K).t()) * cs + b.float()
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-3, (tile, err)
    y0 = torch.ops.sxe.mx_gemm(q, s, W.q, W.scale, mx.FORMATS["mxfp8"][0], None, None)
    ref0 = mx.dequantize(q, s, "mxfp8", K) @ mx.dequantize(W.q, W.scale, "mxfp8", K).t()
    assert (y0.float() - ref0).abs().max().item() <= 1e-2 * ref0.abs().max().item() + 1e-3


@pytest.mark.parametrize("tile", [1, 2, 6, 7, 8, 9, 10])
def test_mx_gemm_tile_identity(tile, monkeypatch):
    """X = I (exact in e4m3), W asymmetric small integers: Y must equal W^T exactly for every tile
    variant -- catches a transposed epilogue or a swapped operand / exponent map."""
    monkeypatch.setenv("SXE_MX_TILE", str(tile))
    K, N = 256, 512
    x = torch.eye(K, device="cuda").to(torch.bfloat16)
    w = (torch.arange(N * K, device="cuda").reshape(N, K) % 7 - 3).float()
    w[:, 128:] *= 4  # a second exponent per row: blocks 4.. differ from blocks 0..3
    W = mx.MXWeight(w, "mxfp8")
    q, s = torch.ops.sxe.mx_quant_fp8(x)
    y = torch.ops.sxe.mx_gemm(q, s, W.q, W.scale, mx.FORMATS["mxfp8"][0], None, None)
    torch.testing.assert_close(y.float(), mx.dequantize(W.q, W.scale, "mxfp8", K).t(), rtol=0, atol=0)
