"""FP quantizer (reference ops/fp_quantizer): FP8 e4m3 / FP6 e3m2 / FP4 e2m1 group-scaled round trips
(exact on representable values, bounded error otherwise), selective dequantize, and the FP8 GEMMs."""
import pytest
import torch


def test_value_tables_match_formats():
    from shuffle_exchange_amd.ops.fp_quantizer import _TABLES
    assert _TABLES[4].tolist() == [0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0]  # e2m1
    assert float(_TABLES[6].max()) == 28.0 and len(_TABLES[6]) == 32      # e3m2


@pytest.mark.parametrize("bits,mant,tol", [(8, 3, 0.04), (6, 2, 0.09), (4, 1, 0.2)])
def test_fp_quantize_roundtrip(bits, mant, tol):
    from shuffle_exchange_amd.ops.fp_quantizer import FP_Quantize
    torch.manual_seed(0)
    x = torch.randn(16, 256)
    fq = FP_Quantize(group_size=128)
    q = fq.quantize(x, q_bits=bits, q_mantisa_bits=mant)
    assert q.dtype == torch.uint8 and q.numel() == x.numel() * (bits if bits != 6 else 8) // 8
    y = fq.dequantize(q).float()
    assert y.shape == x.shape
    rel = ((y - x).norm() / x.norm()).item()
    assert rel < tol, rel
    # selective dequantize of rows 3 and 7
    sel = fq.selective_dequantize(q, torch.tensor([3, 7])).float()
    assert torch.allclose(sel, y[[3, 7]])


def test_fp4_exact_on_representable():
    from shuffle_exchange_amd.ops.fp_quantizer import FP_Quantize
    vals = torch.tensor([0.0, 0.5, -1.0, 1.5, 2.0, -3.0, 4.0, 6.0] * 16)
    fq = FP_Quantize(group_size=128)
    q = fq.quantize(vals, q_bits=4, q_mantisa_bits=1)
    assert torch.equal(fq.dequantize(q).float(), vals)


def test_fp8_linear_and_matmul_fp8_cpu():
    from shuffle_exchange_amd.ops.fp_quantizer import FP8Linear, matmul_fp8
    from shuffle_exchange_amd.ops.quantizer import quantize_fp8
    torch.manual_seed(0)
    lin = torch.nn.Linear(64, 32)
    x = torch.randn(8, 64)
    y = FP8Linear(lin)(x)
    assert ((y - lin(x)).norm() / lin(x).norm()).item() < 0.06
    w = torch.randn(64, 48)
    q, s = quantize_fp8(w.reshape(-1), 64)
    out = matmul_fp8(x.bfloat16(), q.view(64, 48), s, 64)
    assert ((out.float() - x @ w).norm() / (x @ w).norm()).item() < 0.05


def test_matmul_fp8_never_materialises_the_full_weight(monkeypatch):
    """Weight-only FP8 GEMM: the weight is dequantised in K slices of at most MATMUL_FP8_SLICE rows
    (the dequantize op is patched to refuse anything larger) and matches the full product."""
    import shuffle_exchange_amd.ops.fp_quantizer as fq
    from shuffle_exchange_amd.ops.quantizer import dequantize_fp8, quantize_fp8
    torch.manual_seed(0)
    K, N, g = 5000, 96, 64
    w, x = torch.randn(K, N), torch.randn(7, K).bfloat16()
    q, s = quantize_fp8(w.reshape(-1), g)
    ref = x.float() @ dequantize_fp8(q, s, g, dtype=torch.float32).view(K, N)
    real = fq.dequantize_fp8
    seen = []

    def guarded(qq, *a, **k):
        assert qq.numel() <= fq.MATMUL_FP8_SLICE * N, "full-size dequantised weight"
        seen.append(qq.numel())
        return real(qq, *a, **k)
    monkeypatch.setattr(fq, "dequantize_fp8", guarded)
    out = fq.matmul_fp8(x, q.view(K, N), s, g).float()
    assert len(seen) == -(-K // fq.MATMUL_FP8_SLICE)
    assert ((out - ref).abs().max() / ref.abs().max()).item() < 5e-3


@pytest.mark.gpu
def test_fp8_linear_gpu_on_mx_gemm():
    """W8A8 prefill on the block-scaled MX GEMM: equals MXFP8(x) @ (e4m3 codes x row scale)^T."""
    from shuffle_exchange_amd.ops import mx
    from shuffle_exchange_amd.ops.fp_quantizer import fp8_linear, quantize_weight_fp8_rowwise
    torch.manual_seed(1)
    M, N, K = 300, 384, 1024
    w = torch.randn(N, K, device="cuda") * 0.05
    wq, ws = quantize_weight_fp8_rowwise(w)
    x = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    y = fp8_linear(x, wq, ws, b).float()
    xq, xs = torch.ops.sxe.mx_quant_fp8(x)
    ref = mx.dequantize(xq, xs, "mxfp8", K) @ (wq.float() * ws.view(-1, 1)).t() + b.float()
    assert ((y - ref).abs().max() / ref.abs().max()).item() < 1e-2


@pytest.mark.gpu
def test_fp8_linear_gpu_scaled_mm():
    from shuffle_exchange_amd.ops.fp_quantizer import FP8Linear
    torch.manual_seed(0)
    lin = torch.nn.Linear(1024, 512).cuda().bfloat16()
    x = torch.randn(256, 1024, device="cuda", dtype=torch.bfloat16)
    ref = lin(x).float()
    y = FP8Linear(lin)(x).float()
    assert ((y - ref).norm() / ref.norm()).item() < 0.06


# ------------------------------------------------------------------ FP6 / FP4 weights (mxfp.hip)
@pytest.mark.parametrize("bits", [4, 6])
def test_fpx_weight_layout_roundtrip_cpu(bits):
    """The bit-plane GEMM layout decodes back to exactly the FP_Quantize values (per-row scale)."""
    from shuffle_exchange_amd.ops.fp_quantizer import FP_Quantize, FPxWeight
    torch.manual_seed(0)
    w = torch.randn(24, 256)
    fw = FPxWeight(w, bits)
    fq = FP_Quantize(group_size=256)
    ref = fq.dequantize(fq.quantize(w, q_bits=bits, q_mantisa_bits=2 if bits == 6 else 1)).float()
    torch.testing.assert_close(fw.dequantize(torch.float32), ref, rtol=0, atol=0)
    x = torch.randn(3, 256)
    torch.testing.assert_close(fw.linear(x), x @ ref.t(), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [4, 6])
def test_fpx_kernels_gpu(bits):
    """HIP quantize codes == the CPU value-table codes; HIP dequantize / unpack == CPU decode; the
    skinny FP6/FP4-weight GEMM == an fp32 GEMM on the decoded weight."""
    from shuffle_exchange_amd.ops import native
    from shuffle_exchange_amd.ops.fp_quantizer import FP_Quantize, FPxWeight
    native.require_hip()
    torch.manual_seed(0)
    mant = 2 if bits == 6 else 1
    x = torch.randn(64 * 1024) * 3
    qc, qg = FP_Quantize(512), FP_Quantize(512)
    codes_cpu = qc.quantize(x, q_bits=bits, q_mantisa_bits=mant)
    codes_gpu = qg.quantize(x.cuda(), q_bits=bits, q_mantisa_bits=mant)
    torch.testing.assert_close(qg.get_scales().cpu(), qc.get_scales(), rtol=0, atol=0)
    assert torch.equal(codes_gpu.cpu(), codes_cpu)
    torch.testing.assert_close(qg.dequantize(codes_gpu).float().cpu(), qc.dequantize(codes_cpu).float(), rtol=0, atol=0)
    for N, K in [(16, 128), (200, 4096), (1000, 1536)]:
        w = torch.randn(N, K) * 0.05
        fc, fg = FPxWeight(w, bits), FPxWeight(w.cuda().bfloat16(), bits)
        wd = FPxWeight(w.bfloat16(), bits).dequantize(torch.float32)
        # the unpack kernel emits bf16 (hipBLASLt operand): same fp32 product, same rounding
        torch.testing.assert_close(fg.dequantize(torch.bfloat16).cpu(), wd.bfloat16(), rtol=0, atol=0)
        for M in (1, 5, 16):
            xa = torch.randn(M, K).bfloat16()
            bias = torch.randn(N).bfloat16()
            y = fg.linear(xa.cuda(), bias.cuda()).float().cpu()
            ref = xa.float() @ wd.t() + bias.float()
            torch.testing.assert_close(y, ref, rtol=2e-2, atol=2e-2)
        assert fc.bits == bits
