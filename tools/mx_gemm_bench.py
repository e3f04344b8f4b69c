"""MX GEMM (gfx950 block-scaled MFMA, csrc/kernels/mx_gemm.hip) vs bf16 hipBLASLt and FP8
row-scaled hipBLASLt (_scaled_mm) on Llama-3-8B prefill shapes. Times include the MXFP8
activation quantisation pass (reported separately too)."""
import sys

import torch

sys.path.insert(0, ".")
from shuffle_exchange_amd.ops import mx, native  # noqa: E402
from shuffle_exchange_amd.ops.fp_quantizer import fp8_linear, quantize_weight_fp8_rowwise  # noqa: E402


def t(fn, it=50):
    for _ in range(5):
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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="two shapes, MX formats only (tile sweeps)")
    ap.add_argument("--shapes", default=None, help="M,N,K[;M,N,K...] instead of the default list")
    args = ap.parse_args()
    native.require_hip()
    shapes = [(2048, 6144, 4096), (2048, 4096, 4096), (2048, 28672, 4096), (2048, 4096, 14336), (8192, 4096, 4096),
              (512, 4096, 4096), (128, 14336, 4096)]
    if args.quick:
        shapes = [(2048, 28672, 4096), (8192, 4096, 4096), (2048, 4096, 4096)]
    if args.shapes:
        shapes = [tuple(int(v) for v in sh.split(",")) for sh in args.shapes.split(";")]
    import os
    print(f"SXE_MX_TILE={os.environ.get('SXE_MX_TILE', '0')}", flush=True)
    for M, N, K in shapes:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        fl = 2 * M * N * K
        tb = t(lambda: torch.nn.functional.linear(x, w))
        wq8, ws8 = quantize_weight_fp8_rowwise(w)
        t8 = t(lambda: fp8_linear(x, wq8, ws8)) if not args.quick else float("nan")
        q, s = torch.ops.sxe.mx_quant_fp8(x)
        tq = t(lambda: torch.ops.sxe.mx_quant_fp8(x))
        line = f"M={M} N={N} K={K}: bf16 {tb*1e3:.0f} us ({fl/tb/1e9:.0f} TF) | fp8 rowwise {t8*1e3:.0f} us ({fl/t8/1e9:.0f} TF) | act quant {tq*1e3:.0f} us"
        for fmt in ["mxfp8", "mxfp6", "mxfp4"]:
            W = mx.MXWeight(w.float(), fmt)
            code = mx.FORMATS[fmt][0]
            tg = t(lambda: torch.ops.sxe.mx_gemm(q, s, W.q, W.scale, code, None, None))
            line += f" | {fmt} {tg*1e3:.0f} us ({fl/tg/1e9:.0f} TF) +q {fl/(tg+tq)/1e9:.0f} TF"
        if not args.quick and N % 128 == 0:
            from shuffle_exchange_amd.ops.fp_quantizer import FPxWeight
            for bits in (6, 4):
                Wp = FPxWeight(w, bits)
                tp = t(lambda: Wp.linear(x))
                line += f" | FPxWeight fp{bits} planes {tp*1e3:.0f} us ({fl/tp/1e9:.0f} TF incl. quant)"
        print(line, flush=True)


if __name__ == "__main__":
    main()
