"""Weight-gradient GEMM variants on MI355X (T = 8192 tokens, Llama-3-8B shapes), all accumulating
into an fp32 buffer: (a) fused NT addmm fp32-out beta=1, (b) transposes + TN bf16 GEMM + fp32 add
(current), (c) transposes + TN addmm fp32-out beta=1 (no separate add), (d) TN GEMM only (bf16)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shuffle_exchange_amd.ops import native  # noqa: E402
from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms  # noqa: E402

native.require_hip()
load_tuned_gemms()


def t(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


T = 8192
for (O, I) in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]:
    dy = torch.randn(T, O, device="cuda", dtype=torch.bfloat16)
    xx = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
    acc = torch.zeros(O, I, device="cuda")
    fl = 2 * T * O * I / 1e9
    dyt, xt = torch.ops.sxe.transpose16(dy), torch.ops.sxe.transpose16(xx)
    ref = torch.mm(dyt.float(), xt.float().t()) if O * I <= 4096 * 14336 else None
    a = t(lambda: torch.ops.aten.addmm.dtype_out(acc, dy.t(), xx, torch.float32, beta=1, alpha=1, out=acc))

    def tn_add():
        d1, x1 = torch.ops.sxe.transpose16(dy), torch.ops.sxe.transpose16(xx)
        acc.add_(torch.mm(d1, x1.t()))
    b = t(tn_add)

    def tn_fp32():
        d1, x1 = torch.ops.sxe.transpose16(dy), torch.ops.sxe.transpose16(xx)
        torch.ops.aten.addmm.dtype_out(acc, d1, x1.t(), torch.float32, beta=1, alpha=1, out=acc)
    c = t(tn_fp32)
    d = t(lambda: torch.mm(dyt, xt.t()))
    if ref is not None:
        acc.zero_()
        tn_fp32()
        err = ((acc - ref).norm() / ref.norm()).item()
    else:
        err = float("nan")
    print(f"[{O}x{I}] fusedNT {a:.3f} ms ({fl/a:.0f} TF) | tr+TN+add {b:.3f} ({fl/b:.0f} TF) | "
          f"tr+TN fp32-out beta=1 {c:.3f} ({fl/c:.0f} TF, rel err {err:.1e}) | TN bf16 GEMM alone {d:.3f} "
          f"({fl/d:.0f} TF)", flush=True)
    del dy, xx, acc, dyt, xt
