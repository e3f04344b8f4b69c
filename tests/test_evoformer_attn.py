"""DS4Sci_EvoformerAttention vs the plain formula (fp32, CPU), values and all five gradients."""
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
