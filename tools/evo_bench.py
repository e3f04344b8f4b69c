"""Evoformer attention: fused HIP kernels vs the chunked PyTorch path (AlphaFold-like MSA row
attention shapes), fwd and fwd+bwd times."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shuffle_exchange_amd.ops import native  # noqa: E402
from shuffle_exchange_amd.ops.deepspeed4science import evoformer_attn as ea  # noqa: E402

native.require_hip()


def t(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for (B, N, L, H, D) in [(1, 128, 256, 8, 32), (1, 256, 384, 8, 32), (1, 64, 512, 4, 64)]:
    mk = lambda *s: torch.randn(*s, device="cuda", dtype=torch.bfloat16)
    Q, K, V = (mk(B, N, L, H, D).requires_grad_(True) for _ in range(3))
    b1, b2 = mk(B, N, 1, 1, L).requires_grad_(True), mk(B, 1, H, L, L).requires_grad_(True)
    g = mk(B, N, L, H, D)
    hip = lambda: ea.EvoformerFusedAttention.apply(Q, K, V, b1, b2)
    ref = lambda: ea.evoformer_attention(Q.float(), K.float(), V.float(), b1.float(), b2.float())
    res = {}
    for name, f, gg in (("hip", hip, g), ("torch_chunked_fp32", ref, g.float())):
        res[name + "_fwd_ms"] = t(lambda: f())
        res[name + "_fwdbwd_ms"] = t(lambda: torch.autograd.grad(f(), (Q, K, V, b1, b2), gg))
    print({"B": B, "N": N, "L": L, "H": H, "D": D, **{k: round(v, 3) for k, v in res.items()}}, flush=True)
