"""Tile variants of the dual-layout gated kernels (csrc/kernels/act.hip) at the Llama-3-8B MLP shape,
16,384 tokens x 14,336: time and effective HBM rate of forward (reads gu, writes h + h^T) and backward
(reads dout + gu, writes dgu + dgu^T). python tools/gated_dual_bench.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    T, I = 16384, 14336
    gu = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16)
    dout = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
    names = {0: "64x64", 1: "64x128", 2: "128x64", 3: "128x128", 4: "64x256"}
    for v, nm in names.items():
        tf = timeit(lambda: torch.ops.sxe.gated_act_fwd_dual(gu, 3, v))
        tb = timeit(lambda: torch.ops.sxe.gated_act_bwd_dual(dout, gu, 3, v))
        bf = (2 * T * I * 2 + 2 * T * I * 2) / tf
        bb = (2 * T * I * 2 + T * I * 2 + 2 * T * 2 * I * 2) / tb  # gu + dout in, dgu + dgu^T out
        print(f"variant {v} ({nm:7s}) fwd {tf * 1e3:.3f} ms {bf / 1e12:.2f} TB/s | bwd {tb * 1e3:.3f} ms {bb / 1e12:.2f} TB/s",
              flush=True)


if __name__ == "__main__":
    main()
