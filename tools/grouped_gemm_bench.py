"""Grouped expert GEMM on MI355X: one ragged launch (csrc/kernels/grouped_gemm.hip) vs the
per-expert hipBLASLt loop (counts read on the host), Mixtral-8x7B / Qwen-MoE shapes.
usage: python tools/grouped_gemm_bench.py"""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shuffle_exchange_amd.ops import moe as moe_ops, native  # noqa: E402
from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms  # noqa: E402

native.require_hip()
load_tuned_gemms()


def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for name, (E, N, K, tokens, k) in {"mixtral gate_up": (8, 28672, 4096, 4096, 2),
                                   "mixtral down": (8, 4096, 14336, 4096, 2),
                                   "mixtral gate_up decode": (8, 28672, 4096, 64, 2),
                                   "qwen-moe gate_up": (60, 2816, 2048, 4096, 4),
                                   "mixtral gate_up 16k": (8, 28672, 4096, 16384, 2),
                                   "mixtral down 16k": (8, 4096, 14336, 16384, 2)}.items():
    torch.manual_seed(0)
    flat = torch.randint(0, E, (tokens * k,), device="cuda").sort().values
    offs = moe_ops.expert_offsets(flat, E)
    R = flat.numel()
    x = torch.randn(R, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(E, N, K, device="cuda", dtype=torch.bfloat16)

    def loop():
        o = offs.tolist()
        y = x.new_empty(R, N)
        for e in range(E):
            if o[e + 1] > o[e]:
                torch.mm(x[o[e]:o[e + 1]], w[e].t(), out=y[o[e]:o[e + 1]])
        return y

    g = t(lambda: torch.ops.sxe.grouped_gemm(x, w, offs, None))
    os.environ["SXE_GG_TILE"] = "128"
    g128 = t(lambda: torch.ops.sxe.grouped_gemm(x, w, offs, None))
    os.environ["SXE_GG_TILE"] = "256"
    os.environ["SXE_GG_WN"] = "2"
    g256_4w = t(lambda: torch.ops.sxe.grouped_gemm(x, w, offs, None)) if N % 256 == 0 else float("nan")
    os.environ["SXE_GG_WN"] = "4"
    g256 = t(lambda: torch.ops.sxe.grouped_gemm(x, w, offs, None)) if N % 256 == 0 else float("nan")
    del os.environ["SXE_GG_TILE"], os.environ["SXE_GG_WN"]
    lp = t(loop)
    fl = 2 * R * N * K / 1e9
    print(f"[{name}] rows {R}: grouped kernel (auto) {g:.3f} ms ({fl / g:.0f} TF) | 128x128 {g128:.3f} ms "
          f"({fl / g128:.0f} TF) | 256x256 LDS-DMA 4 waves {g256_4w:.3f} ms ({fl / g256_4w:.0f} TF), 8 waves "
          f"{g256:.3f} ms ({fl / g256:.0f} TF) | per-expert hipBLASLt loop "
          f"{lp:.3f} ms ({fl / lp:.0f} TF)", flush=True)
