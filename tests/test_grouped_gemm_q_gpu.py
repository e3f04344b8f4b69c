"""Mixed-precision (int8 / int4 weight) grouped expert GEMM (csrc/kernels/grouped_gemm.hip
grouped_gemm_q_kernel) against an fp32 PyTorch reference over the dequantized weights."""
import pytest
import torch

from shuffle_exchange_amd.ops import moe

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from shuffle_exchange_amd.ops import native
    native.require_hip()


@pytest.mark.parametrize("bits,group", [(8, None), (4, None), (4, 256), (8, 128)])
@pytest.mark.parametrize("E,N,K,rows", [(4, 256, 512, [0, 37, 200, 5]), (8, 128, 256, [130, 1, 0, 64, 3, 257, 9, 12])])
def test_grouped_gemm_q(bits, group, E, N, K, rows):
    torch.manual_seed(E * N + K + bits)
    w = torch.randn(E, N, K, device="cuda") * 0.03
    W = moe.QuantizedExperts(w, bits, group)
    R = sum(rows)
    x = torch.randn(R, K, device="cuda").to(torch.bfloat16)
    offs = torch.tensor([0] + list(torch.tensor(rows).cumsum(0)), dtype=torch.int32, device="cuda")
    rs = torch.rand(R, device="cuda")
    y = moe.grouped_gemm_q(x, W, offs, rs)
    wd = W.dequantize(torch.float32)
    ref = torch.empty(R, N, device="cuda")
    o = offs.tolist()
    for e in range(E):
        ref[o[e]:o[e + 1]] = x[o[e]:o[e + 1]].float() @ wd[e].t()
    ref = ref * rs[:, None]
    # operands are bf16-rounded (q * scale) inside the kernel; fp32 accumulation
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-3, err
    # and the quantisation itself is faithful
    full = torch.cat([x[o[e]:o[e + 1]].float() @ w[e].t() for e in range(E)]) * rs[:, None]
    rel = (y.float() - full).norm() / full.norm()
    assert rel < (0.02 if bits == 8 else 0.15)


def test_int_weight_dense_linear():
    from shuffle_exchange_amd.ops.fp_quantizer import quantized_weight
    torch.manual_seed(0)
    w = torch.randn(384, 512, device="cuda") * 0.05
    x = torch.randn(3, 9, 512, device="cuda").to(torch.bfloat16)
    for kind in ("int8", "int4"):
        W = quantized_weight(w, kind)
        y = W.linear(x)
        ref = x.float() @ W.dequantize(torch.float32).t()
        assert y.shape == (3, 9, 384)
        assert (y.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item() + 1e-3
