"""Where does the k-major weight-gradient GEMM lose against hipBLASLt's forward-layout GEMM?
A/B in one process (interleaved rounds, best of each arm): block-order super-row height, padded
leading dimensions (row stride), and hipBLASLt TN on pre-transposed operands as the ceiling."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shuffle_exchange_amd.ops import native  # noqa: E402
from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms  # noqa: E402

native.require_hip()
load_tuned_gemms()


def t(fn, n=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


T = 8192
for (Mo, Ni) in [(28672, 4096), (4096, 14336)]:
    gy = torch.randn(T, Mo, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, Ni, device="cuda", dtype=torch.bfloat16)
    gyp = torch.randn(T, Mo + 128, device="cuda", dtype=torch.bfloat16)[:, :Mo]
    xp = torch.randn(T, Ni + 128, device="cuda", dtype=torch.bfloat16)[:, :Ni]
    acc = torch.zeros(Mo, Ni, device="cuda")
    gyt, xt = gy.t().contiguous(), x.t().contiguous()
    fl = 2.0 * T * Mo * Ni
    arms = {f"v0 g{g}": (lambda g=g: torch.ops.sxe.wgrad_gemm_variant_(gy, x, acc, 1.0, True, 16 * g))
            for g in (1, 4, 8, 16)}
    arms["v0 g8 padded ld"] = lambda: torch.ops.sxe.wgrad_gemm_variant_(gyp, xp, acc, 1.0, True, 16 * 8)
    arms["v3 (no DMA in loop) g8"] = lambda: torch.ops.sxe.wgrad_gemm_variant_(gy, x, acc, 1.0, True, 3 + 16 * 8)
    arms["v0 g8 overwrite"] = lambda: torch.ops.sxe.wgrad_gemm_variant_(gy, x, acc, 1.0, False, 16 * 8)
    arms["hipBLASLt TN bf16 (pre-transposed)"] = lambda: torch.mm(gyt, xt.t())
    best = {k: 1e9 for k in arms}
    for _ in range(3):
        for k, fn in arms.items():
            best[k] = min(best[k], t(fn))
    print(f"[{Mo}x{Ni}] K={T}: " + " | ".join(f"{k} {v*1e3:.3f} ms {fl/v/1e12:.0f} TF" for k, v in best.items()),
          flush=True)
    del gy, x, gyp, xp, acc, gyt, xt
