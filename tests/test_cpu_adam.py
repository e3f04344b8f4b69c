"""Host Adam/AdamW kernel of the ZeRO-Offload tier (csrc/cpu/cpu_adam.cpp, vectorised: built with
-fno-math-errno so the sqrt / divide loop compiles to SIMD) against a plain fp32 PyTorch reference
of the same update, including the fused bit16 copy of the updated parameter (round to nearest
even, NaN kept) and bf16 gradients."""
import pytest
import torch

from shuffle_exchange_amd.ops import native


def _ref(p, g, m, v, lr, b1, b2, eps, wd, step, adamw):
    g = g.float()
    if not adamw:
        g = g + wd * p
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    if adamw:
        p = p - lr * wd * p
    p = p - (lr / bc1) * m / (v.sqrt() / bc2 ** 0.5 + eps)
    return p, m, v


@pytest.mark.parametrize("adamw", [True, False])
@pytest.mark.parametrize("gdtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("lpdtype", [None, torch.bfloat16, torch.float16])
def test_cpu_adam_matches_fp32_reference(adamw, gdtype, lpdtype):
    if not native.cpu_available():
        pytest.skip("native CPU extension not built")
    torch.manual_seed(0)
    n = 3 * 4096 + 123  # several tiles and a ragged tail
    p = torch.randn(n)
    g = torch.randn(n).to(gdtype)
    m = torch.randn(n) * 0.1
    v = torch.rand(n) * 0.01
    lp = torch.empty(n, dtype=lpdtype) if lpdtype is not None else None
    rp, rm, rv = _ref(p.clone(), g, m.clone(), v.clone(), 1e-3, 0.9, 0.999, 1e-8, 0.01, 3, adamw)
    torch.ops.sxe_cpu.adam_step_(p, g, m, v, lp, 1e-3, 0.9, 0.999, 1e-8, 0.01, 3, adamw, True, 1.0)
    torch.testing.assert_close(p, rp, rtol=1e-5, atol=1e-6)  # FMA contraction order
    torch.testing.assert_close(m, rm, rtol=1e-5, atol=1e-6)  # FMA contraction order
    torch.testing.assert_close(v, rv, rtol=1e-5, atol=1e-6)  # FMA contraction order
    if lpdtype is not None:
        assert torch.equal(lp, p.to(lpdtype))  # the fused copy rounds exactly like a cast


def test_cpu_adam_bf16_copy_keeps_nan_and_inf():
    if not native.cpu_available():
        pytest.skip("native CPU extension not built")
    p = torch.tensor([1.0, float("nan"), float("inf"), -float("inf"), 3.0e38] * 1000)
    g = torch.zeros_like(p)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    lp = torch.empty(p.numel(), dtype=torch.bfloat16)
    torch.ops.sxe_cpu.adam_step_(p, g, m, v, lp, 0.0, 0.9, 0.999, 1e-8, 0.0, 1, True, True, 1.0)
    ref = p.to(torch.bfloat16)
    assert torch.equal(lp.isnan(), ref.isnan())
    assert torch.equal(lp[~ref.isnan()], ref[~ref.isnan()])
