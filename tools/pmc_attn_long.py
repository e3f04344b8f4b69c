"""Flash-attention forward / backward at the SP-32k per-GPU shape (B1 S32768 H4/1 D128 causal: the
8-wave dQ / dK/dV kernels and the per-head split), 2 dispatches each, for rocprofv3 --pmc passes
(bash tools/gpu_run.sh pmcw=pmc_attn_long.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from shuffle_exchange_amd.ops import native
    from shuffle_exchange_amd.ops.attention import attention
    native.require_hip()
    bf = torch.bfloat16
    q = torch.randn(1, 32768, 4, 128, device="cuda", dtype=bf, requires_grad=True)
    k = torch.randn(1, 32768, 1, 128, device="cuda", dtype=bf, requires_grad=True)
    v = torch.randn(1, 32768, 1, 128, device="cuda", dtype=bf, requires_grad=True)
    g = torch.randn(1, 32768, 4, 128, device="cuda", dtype=bf)
    for _ in range(2):
        torch.autograd.grad(attention(q, k, v), (q, k, v), g)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
