"""DS4Sci_EvoformerAttention vs the plain formula (fp32, CPU), values and all five gradients."""
import pytest
import torch

from shuffle_exchange_amd.ops.deepspeed4science import DS4Sci_EvoformerAttention
from shuffle_exchange_amd.ops.deepspeed4science import evoformer_attn as ea


def test_evoformer_matches_formula_with_grads(monkeypatch):
    monkeypatch.setattr(ea, "CHUNK", 8)
    torch.manual_seed(0)
    B, N, L, H, D = 1, 3, 20, 2, 16
    Q, K, V = (torch.randn(B, N, L, H, D, requires_grad=True) for _ in range(3))
    b1 = torch.randn(B, N, 1, 1, L, requires_grad=True)
    b2 = torch.randn(B, 1, H, L, L, requires_grad=True)
    out = ea.evoformer_attention(Q, K, V, b1, b2, chunk=8)
    s = torch.einsum("bnqhd,bnkhd->bnhqk", Q, K) / D ** 0.5 + b1 + b2
    ref = torch.einsum("bnhqk,bnkhd->bnqhd", torch.softmax(s, -1), V)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(out)
    got = torch.autograd.grad(out, (Q, K, V, b1, b2), g)
    exp = torch.autograd.grad(ref, (Q, K, V, b1, b2), g)
    for a, b in zip(got, exp):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-4)
    o2 = DS4Sci_EvoformerAttention(Q, K, V, [b1, b2])
    torch.testing.assert_close(o2, ref, atol=1e-5, rtol=1e-5)
    o3 = DS4Sci_EvoformerAttention(Q, K, V, [])
    s3 = torch.einsum("bnqhd,bnkhd->bnhqk", Q, K) / D ** 0.5
    torch.testing.assert_close(o3, torch.einsum("bnhqk,bnkhd->bnqhd", torch.softmax(s3, -1), V), atol=1e-5,
                               rtol=1e-5)


def _formula(Q, K, V, b1, b2):
    D = Q.shape[-1]
    q, k, v = (t.float().transpose(-2, -3) for t in (Q, K, V))  # [B, N, H, L, D]
    s = q @ k.transpose(-1, -2) / D ** 0.5 + b1.float() + b2.float()
    return (torch.softmax(s, -1) @ v).transpose(-2, -3)


@pytest.mark.gpu
@pytest.mark.parametrize("D,L", [(32, 70), (64, 133), (64, 256)])
def test_evoformer_hip_kernels_vs_fp32(D, L):
    """Fused HIP forward / backward (evoformer.hip) vs the fp32 formula: output, dQ, dK, dV, dbias1,
    dbias2, for sequence lengths that are not tile multiples."""
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    torch.manual_seed(0)
    B, N, H = 2, 3, 2
    mk = lambda *s: torch.randn(*s, device="cuda")
    Q, K, V = (mk(B, N, L, H, D).bfloat16().requires_grad_(True) for _ in range(3))
    b1 = (mk(B, N, 1, 1, L) * 2).bfloat16().requires_grad_(True)
    b2 = mk(B, 1, H, L, L).bfloat16().requires_grad_(True)
    assert ea._hip_ok(Q, K, V)
    out = DS4Sci_EvoformerAttention(Q, K, V, [b1, b2])
    g = mk(*out.shape).bfloat16()
    grads = torch.autograd.grad(out, (Q, K, V, b1, b2), g)
    ref_in = [t.detach().float().requires_grad_(True) for t in (Q, K, V, b1, b2)]
    ref = _formula(*ref_in)
    rgrads = torch.autograd.grad(ref, ref_in, g.float())
    assert (out.float() - ref).abs().max().item() < 2e-2
    for name, a, b in zip("QKV12", grads, rgrads):
        err = ((a.float() - b).norm() / b.norm()).item()
        assert err < 2e-2, (name, err)
