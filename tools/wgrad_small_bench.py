"""Weight-gradient GEMMs of the attention projections (dW [M, N] += dY^T [M, T] X [T, N] into an
fp32 accumulator), the shapes ops/linear.py routes to the NT fp32-out library GEMM today: NT
hipBLASLt fp32-out vs the hand-written k-major kernel (csrc/kernels/gemm_wgrad.hip) vs transposes +
TN hipBLASLt fp32-out.  python tools/wgrad_small_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


def main():
    from shuffle_exchange_amd.ops import native
    from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms
    native.require_hip()
    load_tuned_gemms()
    for T in (8192, 16384):
        shapes = ((6144, 4096), (4096, 4096), (4096, 14336), (28672, 4096), (128256, 4096))
        if os.environ.get("WGRAD_SHAPES") == "lmhead":
            shapes = ((128256, 4096),)
        for M, N in shapes:
            gy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
            x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
            buf = torch.zeros(M, N, device="cuda")
            fl = 2 * T * M * N
            nt = t(lambda: torch.ops.aten.addmm.dtype_out(buf, gy.t(), x, torch.float32, beta=1, alpha=1, out=buf))
            own = t(lambda: torch.ops.sxe.wgrad_gemm_(gy, x, buf, 1.0, True)) if M * N < 2 ** 27 else float("nan")  # the kernel's 32-bit offsets

            def tn():
                a, b = torch.ops.sxe.transpose16(gy), torch.ops.sxe.transpose16(x).t()
                torch.ops.aten.addmm.dtype_out(buf, a, b, torch.float32, beta=1, alpha=1, out=buf)
            tt = t(tn)

            def tn16():  # bf16-out TN GEMM (TunableOp-tuned shapes) + fp32 accumulate pass
                a, b = torch.ops.sxe.transpose16(gy), torch.ops.sxe.transpose16(x).t()
                buf.add_(torch.mm(a, b))
            t16 = t(tn16, it=10)
            print(json.dumps({"T": T, "M": M, "N": N, "nt_ms": round(nt, 4), "nt_TF": round(fl / nt / 1e9),
                              "own_ms": round(own, 4), "own_TF": None if own != own else round(fl / own / 1e9),
                              "tn_ms": round(tt, 4), "tn_TF": round(fl / tt / 1e9),
                              "tn_bf16_add_ms": round(t16, 4), "tn_bf16_add_TF": round(fl / t16 / 1e9)}), flush=True)


if __name__ == "__main__":
    main()
