"""Weight-gradient GEMM variants at the Llama-3-8B headline micro-step (16,384 tokens), fp32 accumulator:
  nt32   : hipBLASLt fp32-out, beta = 1, token-major operands (the current QKV path)
  hand   : csrc/kernels/gemm_wgrad.hip k-major kernel (fp32 accumulate)
  tn+T32 : two transposes + TN fp32-out beta = 1 (the current LM-head path)
  tn32   : TN fp32-out beta = 1 with operands already token-minor (producers write them)
  tn16   : TN bf16-out + fp32 add, operands already token-minor (the MLP path)
  T      : cost of the two transposes alone
  python tools/wgrad_variants_bench.py [--tokens 16384] [--shapes qkv,o_proj,lm_head]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="qkv,o_proj,gate_up,down,lm_head")
    a = ap.parse_args()
    from shuffle_exchange_amd.ops import native
    from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms
    native.require_hip()
    load_tuned_gemms()
    T = a.tokens
    shapes = {"qkv": (6144, 4096), "o_proj": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    tr = torch.ops.sxe.transpose16
    addmm32 = torch.ops.aten.addmm.dtype_out
    print(f"| GEMM | N | K | variant | ms | TFLOP/s |\n|---|---:|---:|---|---:|---:|")
    for name in a.shapes.split(","):
        N, K = shapes[name]
        fl = 2.0 * T * N * K
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        gy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        buf = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        gyT, xT = tr(gy), tr(x)
        res = {}
        res["nt32"] = timeit(lambda: addmm32(buf, gy.t(), x, torch.float32, beta=1, alpha=1, out=buf), a.iters)
        try:
            torch.ops.sxe.wgrad_gemm_(gy, x, buf, 1.0, True)
            res["hand"] = timeit(lambda: torch.ops.sxe.wgrad_gemm_(gy, x, buf, 1.0, True), a.iters)
        except RuntimeError:
            pass
        res["tn+T32"] = timeit(lambda: addmm32(buf, tr(gy), tr(x).t(), torch.float32, beta=1, alpha=1, out=buf),
                               a.iters)
        res["tn32"] = timeit(lambda: addmm32(buf, gyT, xT.t(), torch.float32, beta=1, alpha=1, out=buf), a.iters)
        res["tn16"] = timeit(lambda: buf.add_(torch.mm(gyT, xT.t())), a.iters)
        res["T"] = timeit(lambda: (tr(gy), tr(x)), a.iters)
        for k, t in res.items():
            print(f"| {name} | {N} | {K} | {k} | {t * 1e3:.3f} | {fl / t / 1e12:.0f} |", flush=True)
        del x, gy, buf, gyT, xT
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
