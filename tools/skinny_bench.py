"""Decode GEMM micro-benchmark: MFMA skinny GEMM (torch.ops.sxe.skinny_gemm) vs hipBLASLt
(F.linear) on Llama-3-8B projection shapes, M = 1..16 rows (graph of back-to-back calls).
  python tools/skinny_bench.py"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timeit(f, reps=20):
    f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * reps) * 1e3


def main():
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    for name, (N, K) in SHAPES.items():
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(4)]  # > L2/MALL reuse
        for M in (1, 4, 8, 16):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            i = [0]

            def sk():
                i[0] = (i[0] + 1) % 4
                torch.ops.sxe.skinny_gemm(x, ws[i[0]], None)

            def bl():
                i[0] = (i[0] + 1) % 4
                F.linear(x, ws[i[0]])
            from shuffle_exchange_amd.ops.fp_quantizer import quantize_weight_fp8_rowwise
            qs = [quantize_weight_fp8_rowwise(wi) for wi in ws]

            def f8():
                i[0] = (i[0] + 1) % 4
                torch.ops.sxe.skinny_gemm_fp8w(x, qs[i[0]][0].view(torch.uint8), qs[i[0]][1], None)
            from shuffle_exchange_amd.ops.fp_quantizer import FPxWeight
            f6s = [FPxWeight(wi, 6) for wi in ws]
            f4s = [FPxWeight(wi, 4) for wi in ws]

            def f6():
                i[0] = (i[0] + 1) % 4
                q = f6s[i[0]]
                torch.ops.sxe.skinny_gemm_fpxw(x, q.wa, q.wb, q.scale, None, 6)

            def f4():
                i[0] = (i[0] + 1) % 4
                q = f4s[i[0]]
                torch.ops.sxe.skinny_gemm_fpxw(x, q.wa, None, q.scale, None, 4)
            t_sk, t_bl, t_f8, t_f6, t_f4 = timeit(sk), timeit(bl), timeit(f8), timeit(f6), timeit(f4)
            gb = N * K * 2 / 1e9
            print(json.dumps({"shape": name, "N": N, "K": K, "M": M, "skinny_us": round(t_sk, 2),
                              "hipblaslt_us": round(t_bl, 2), "skinny_fp8w_us": round(t_f8, 2),
                              "skinny_TBps": round(gb / t_sk * 1e3, 2), "hipblaslt_TBps": round(gb / t_bl * 1e3, 2),
                              "fp8w_weight_TBps": round(gb / 2 / t_f8 * 1e3, 2),
                              "skinny_fp6w_us": round(t_f6, 2), "fp6w_weight_TBps": round(gb * 0.375 / t_f6 * 1e3, 2),
                              "skinny_fp4w_us": round(t_f4, 2), "fp4w_weight_TBps": round(gb * 0.25 / t_f4 * 1e3, 2)}),
                  flush=True)
            del qs, f6s, f4s
        del ws


if __name__ == "__main__":
    main()
