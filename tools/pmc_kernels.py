"""Workload for rocprofv3 --pmc passes over the hand-written gfx950 kernels (a few dispatches each):
flash attention fwd/bwd (B4 S2048 H32/8 D128 causal), skinny decode GEMM (bf16 and FP8 weights,
4096x14336 at M=1), paged decode attention (B32 ctx 1024), RMSNorm fwd (8192x4096), fused AdamW on
64M params, k-major wgrad GEMM, dual-layout gated kernels (16k x 14336), grouped expert GEMM
(60 experts). Run under:  rocprofv3 --pmc <counters> --output-format csv -d DIR -o pmc -- python3 tools/pmc_kernels.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from shuffle_exchange_amd.ops import native
    from shuffle_exchange_amd.ops.attention import attention
    from shuffle_exchange_amd.ops.fp_quantizer import quantize_weight_fp8_rowwise
    from shuffle_exchange_amd.ops.norm import rms_norm
    from shuffle_exchange_amd.ops.optim import adam_flat_
    native.require_hip()
    dev = "cuda"
    bf = torch.bfloat16
    q = torch.randn(4, 2048, 32, 128, device=dev, dtype=bf, requires_grad=True)
    k = torch.randn(4, 2048, 8, 128, device=dev, dtype=bf, requires_grad=True)
    v = torch.randn(4, 2048, 8, 128, device=dev, dtype=bf, requires_grad=True)
    g = torch.randn(4, 2048, 32, 128, device=dev, dtype=bf)
    for _ in range(0 if os.environ.get("PMC_ONLY_GEMM") else 3):
        torch.autograd.grad(attention(q, k, v), (q, k, v), g)
    x1 = torch.randn(1, 14336, device=dev, dtype=bf)
    w = torch.randn(4096, 14336, device=dev, dtype=bf)
    wq, ws = quantize_weight_fp8_rowwise(w)
    for _ in range(3):
        torch.ops.sxe.skinny_gemm(x1, w, None)
        torch.ops.sxe.skinny_gemm_fp8w(x1, wq.view(torch.uint8), ws, None)
    B, ctx, nkv, bs = 32, 1024, 8, 64
    nb = ctx // bs
    cache = torch.randn(B * nb, 2, nkv, bs, 128, device=dev, dtype=bf)
    bt = torch.arange(B * nb, device=dev, dtype=torch.int32).view(B, nb)
    qd = torch.randn(B, 32, 128, device=dev, dtype=bf)
    ar = torch.arange(B, device=dev, dtype=torch.int32)
    for _ in range(3):
        torch.ops.sxe.paged_attention(qd, cache, bt, ar, torch.ones_like(ar), torch.full_like(ar, ctx), 128 ** -0.5,
                                      ctx, 2)
    xn = torch.randn(8192, 4096, device=dev, dtype=bf)
    wn = torch.ones(4096, device=dev, dtype=bf)
    for _ in range(3):
        rms_norm(xn, wn, 1e-5)
    n = 64 << 20
    p, gr, m, vv = (torch.randn(n, device=dev) for _ in range(4))
    vv.abs_()
    lp = torch.empty(n, device=dev, dtype=bf)
    for s in range(1, 4):
        adam_flat_(p, gr, m, vv, lp, lr=1e-3, step=s)
    # weight-gradient GEMM (k-major operands, fp32 accumulate) vs hipBLASLt's forward-layout GEMM
    gy = torch.randn(8192, 28672, device=dev, dtype=bf)
    xw = torch.randn(8192, 4096, device=dev, dtype=bf)
    accw = torch.zeros(28672, 4096, device=dev)
    gyt, xwt = gy.t().contiguous(), xw.t().contiguous()
    for _ in range(3):
        torch.ops.sxe.wgrad_gemm_variant_(gy, xw, accw, 1.0, True, 0)
        torch.mm(gyt, xwt.t())
    del gy, xw, accw, gyt, xwt
    # dual-layout gated kernels of the fused MLP (16k tokens x 14336) and the grouped expert GEMM
    gu = torch.randn(16384, 28672, device=dev, dtype=bf)
    dh = torch.randn(16384, 14336, device=dev, dtype=bf)
    for _ in range(3):
        torch.ops.sxe.gated_act_fwd_dual(gu, 3, 4)
        torch.ops.sxe.gated_act_bwd_dual(dh, gu, 3, 4)
    del gu, dh
    E, N, K, R = 60, 2816, 2048, 16384
    xs = torch.randn(R, K, device=dev, dtype=bf)
    we = torch.randn(E, N, K, device=dev, dtype=bf)
    flat = torch.randint(0, E, (R,), device=dev).sort().values
    from shuffle_exchange_amd.ops.moe import expert_offsets
    offs = expert_offsets(flat, E)
    for _ in range(3):
        torch.ops.sxe.grouped_gemm(xs, we, offs, None)
    torch.cuda.synchronize()
    print("pmc workload done", flush=True)


if __name__ == "__main__":
    main()
