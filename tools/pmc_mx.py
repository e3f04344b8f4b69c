"""Workload for rocprofv3 --pmc passes over the MX block-scaled GEMM (csrc/kernels/mx_gemm.hip) at
the Llama-3-8B prefill shapes, with bf16 hipBLASLt on the same shapes for comparison. Tile variant
from SXE_MX_TILE. Run under: rocprofv3 --pmc <counters> -- python3 tools/pmc_mx.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from shuffle_exchange_amd.ops import mx, native
    native.require_hip()
    fmts = os.environ.get("PMC_MX_FMTS", "mxfp8").split(",")
    for M, N, K in ((2048, 28672, 4096), (8192, 4096, 4096)):
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        q, s = torch.ops.sxe.mx_quant_fp8(x)
        for fmt in fmts:
            W = mx.MXWeight(w.float(), fmt)
            for _ in range(3):
                torch.ops.sxe.mx_gemm(q, s, W.q, W.scale, mx.FORMATS[fmt][0], None, None)
        for _ in range(3):
            torch.nn.functional.linear(x, w)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
