"""int8 / int4 expert weights (ops/moe.QuantizedExperts): storage layout and the CPU path of
grouped_gemm_q / IntWeight (the GPU kernel is tests/test_grouped_gemm_q_gpu.py)."""
import torch

from shuffle_exchange_amd.ops import moe
from shuffle_exchange_amd.ops.fp_quantizer import quantized_weight


def test_int4_packing_and_roundtrip():
    w = torch.zeros(1, 128, 256)
    w[0, 0, 0], w[0, 0, 1] = -7.0, 3.0
    W = moe.QuantizedExperts(w, 4)
    assert W.q.shape == (1, 128, 128) and W.q.dtype == torch.uint8
    assert int(W.q[0, 0, 0]) == ((-7) & 0xF) | (3 << 4)   # low nibble first, two's complement
    torch.testing.assert_close(W.dequantize(torch.float32), w)


def test_grouped_q_cpu_matches_dequantized_loop():
    torch.manual_seed(0)
    w = torch.randn(3, 128, 256) * 0.1
    for bits in (8, 4):
        W = moe.QuantizedExperts(w, bits)
        x = torch.randn(10, 256)
        offs = torch.tensor([0, 4, 4, 10], dtype=torch.int32)
        y = moe.grouped_gemm_q(x, W, offs)
        wd = W.dequantize(torch.float32)
        ref = torch.cat([x[:4] @ wd[0].t(), x[4:] @ wd[2].t()])
        torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
        assert (wd - w).abs().max() <= W.scale.max() / 2 + 1e-6


def test_int_weight_cpu():
    torch.manual_seed(1)
    w = torch.randn(128, 256) * 0.05
    x = torch.randn(2, 5, 256)
    for kind in ("int8", "int4"):
        W = quantized_weight(w, kind)
        y = W.linear(x, bias=torch.ones(128))
        torch.testing.assert_close(y, x @ W.dequantize(torch.float32).t() + 1, rtol=1e-5, atol=1e-5)
