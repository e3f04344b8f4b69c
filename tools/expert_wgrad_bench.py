"""Expert weight gradients of the capacity-based MoE layer (moe/experts.py ``_GroupedMM``):
dW[e] = x[e]^T dy[e] with few tokens per expert (the reduction axis, C = capacity), accumulated into
the fp32 ZeRO buffer. Arms: the hand-written k-major kernel (gemm_wgrad.hip), hipBLASLt NT with an
fp32 output (beta = 1), transposes + hipBLASLt TN fp32, and TN bf16 + fp32 add.
  python tools/expert_wgrad_bench.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shuffle_exchange_amd.ops import native  # noqa: E402

native.require_hip()


def t(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms
    load_tuned_gemms()
    torch.manual_seed(0)
    for C in (1024, 2048, 4096):
        for name, K, N in (("gate_up", 4096, 28672), ("down", 14336, 4096)):
            x = torch.randn(C, K, device="cuda", dtype=torch.bfloat16)
            dy = torch.randn(C, N, device="cuda", dtype=torch.bfloat16)
            acc = torch.zeros(K, N, device="cuda")
            ref = torch.zeros(K, N, device="cuda")
            torch.ops.aten.addmm.dtype_out(ref, x.t(), dy, torch.float32, beta=0, alpha=1, out=ref)
            fl = 2.0 * C * K * N

            def tn_fp32():
                a, b = torch.ops.sxe.transpose16(x), torch.ops.sxe.transpose16(dy)
                torch.ops.aten.addmm.dtype_out(acc, a, b.t(), torch.float32, beta=1, alpha=1, out=acc)

            def tn_bf16_add():
                a, b = torch.ops.sxe.transpose16(x), torch.ops.sxe.transpose16(dy)
                acc.add_(torch.mm(a, b.t()))

            arms = {"wgrad kernel": lambda: torch.ops.sxe.wgrad_gemm_(x, dy, acc, 1.0, True),
                    "hipBLASLt NT fp32": lambda: torch.ops.aten.addmm.dtype_out(acc, x.t(), dy, torch.float32, beta=1,
                                                                                 alpha=1, out=acc),
                    "transposes+TN fp32": tn_fp32, "transposes+TN bf16+add": tn_bf16_add}
            out = []
            for k, fn in arms.items():
                if k == "wgrad kernel":
                    from shuffle_exchange_amd.ops.linear import _sxe_wgrad_ok
                    if not _sxe_wgrad_ok(x, dy, acc):
                        out.append(f"{k} n/a")
                        continue
                acc.zero_()
                fn()
                err = ((acc - ref).norm() / ref.norm()).item()
                s = min(t(fn, 5) for _ in range(2))
                out.append(f"{k} {s * 1e3:.3f} ms {fl / s / 1e12:.0f} TF (err {err:.1e})")
            print(f"[{name} C={C}] " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
