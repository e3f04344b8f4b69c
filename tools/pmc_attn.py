"""Flash-attention forward / backward only (B4 S2048 H32/8 D128 causal), 3 dispatches each, for
rocprofv3 --pmc passes (bash tools/gpu_run.sh pmc_attn)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from shuffle_exchange_amd.ops import native
    from shuffle_exchange_amd.ops.attention import attention
    native.require_hip()
    bf = torch.bfloat16
    q = torch.randn(4, 2048, 32, 128, device="cuda", dtype=bf, requires_grad=True)
    k = torch.randn(4, 2048, 8, 128, device="cuda", dtype=bf, requires_grad=True)
    v = torch.randn(4, 2048, 8, 128, device="cuda", dtype=bf, requires_grad=True)
    g = torch.randn(4, 2048, 32, 128, device="cuda", dtype=bf)
    for _ in range(3):
        torch.autograd.grad(attention(q, k, v), (q, k, v), g)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
