"""Llama-3-8B training GEMMs on MI355X by layout (T = 8192 tokens, bf16, tuned hipBLASLt):
forward y = x W^T, data-grad dX = dY W (as autograd issues it) vs dX = dY (W^T)^T with a
materialised W^T (forward layout), and weight-grad (transposes + forward-layout GEMM)."""
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
    x = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(O, I, device="cuda", dtype=torch.bfloat16) * 0.02
    dy = torch.randn(T, O, device="cuda", dtype=torch.bfloat16)
    fl = 2 * T * O * I / 1e9
    f = t(lambda: torch.mm(x, w.t()))
    dg = t(lambda: torch.mm(dy, w))
    wt_tr = t(lambda: torch.ops.sxe.transpose16(w))
    wt = torch.ops.sxe.transpose16(w)
    dg2 = t(lambda: torch.mm(dy, wt.t()))
    err = ((torch.mm(dy, wt.t()).float() - torch.mm(dy, w).float()).norm() / torch.mm(dy, w).float().norm()).item()
    print(f"[{O}x{I}] fwd {f:.3f} ms ({fl/f:.0f} TF) | dgrad dY@W {dg:.3f} ({fl/dg:.0f} TF) | "
          f"W^T transpose {wt_tr:.3f} + dY@(W^T)^T {dg2:.3f} ({fl/dg2:.0f} TF) -> gain {dg - dg2 - wt_tr:+.3f} ms "
          f"(rel diff {err:.1e})", flush=True)
    del x, w, dy, wt
