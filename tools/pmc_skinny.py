"""Workload for rocprofv3 --pmc passes over the decode (batch-1) skinny GEMMs with the fused RMSNorm
prologue (csrc/kernels/skinny_gemm.hip): the Llama-3-8B QKV shape (6144 x 4096, the one streaming
at 2.8 TB/s) next to gate_up (28672 x 4096, 5.1 TB/s) and down (4096 x 14336, SwiGLU prologue),
20 calls each.  rocprofv3 --pmc <counters> -- python3 tools/pmc_skinny.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    bf = torch.bfloat16
    x = torch.randn(1, 4096, device="cuda", dtype=bf)
    res = torch.randn(1, 4096, device="cuda", dtype=bf)
    gw = torch.ones(4096, device="cuda", dtype=bf)
    wq = torch.randn(6144, 4096, device="cuda", dtype=bf) * 0.02
    wgu = torch.randn(28672, 4096, device="cuda", dtype=bf) * 0.02
    wd = torch.randn(4096, 14336, device="cuda", dtype=bf) * 0.02
    gu = torch.randn(1, 28672, device="cuda", dtype=bf)
    for _ in range(20):
        torch.ops.sxe.skinny_gemm_pro(x, res, gw, 1e-5, wq, None, None, 1)
        torch.ops.sxe.skinny_gemm_pro(x, res, gw, 1e-5, wgu, None, None, 1)
        torch.ops.sxe.skinny_gemm_pro(gu, None, None, 0.0, wd, None, None, 2)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
