"""Per-shape table of the Llama-3-8B training GEMMs at the headline micro-batch (8 x 2048 = 16,384 tokens),
timed through the SAME code paths the step uses (ops/linear.py: forward F.linear, data_grad with the
transposed weight, write_weight_grad into an fp32 accumulator; ops/mlp.py weight_grad_tn for the MLP),
with the TunableOp solution each hipBLASLt call resolves to.
  python tools/gemm_step_table.py [--tokens 16384] [--iters 20]
Prints one markdown table: achieved TFLOP/s and % of the 2.5 PF dense bf16 peak per call."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK = 2.5e15


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
    a = ap.parse_args()
    from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms
    from shuffle_exchange_amd.ops import linear as L
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    from shuffle_exchange_amd.ops.mlp import weight_grad_tn
    load_tuned_gemms()
    T = a.tokens
    dev = "cuda"
    shapes = {"qkv": (6144, 4096), "o_proj": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    rows = []
    for name, (N, K) in shapes.items():
        w = torch.nn.Parameter(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02)
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        gy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * N * K
        buf = torch.zeros(N, K, device=dev, dtype=torch.float32)
        w._sxe_grad_target = lambda p, buf=buf: (buf, True)
        w._sxe_grad_done = lambda p: None
        t_f = timeit(lambda: torch.nn.functional.linear(x, w), a.iters)
        t_d = timeit(lambda: L.data_grad(gy, w), a.iters)
        if name in ("gate_up", "down"):  # the MLP autograd node: token-minor operands from the producers
            gyT, xT = gy.t().contiguous(), x.t().contiguous()
            t_w = timeit(lambda: weight_grad_tn(w, gyT, xT), a.iters)
            wpath = "bf16 TN + fp32 add (operands pre-transposed by the producers)"
        else:
            t_w = timeit(lambda: L.write_weight_grad(w, gy, x), a.iters)
            if L._sxe_wgrad_ok(gy, x, buf):
                wpath = "hand-written k-major wgrad kernel (fp32 accumulate)"
            elif L._tn_ok(gy, x):
                wpath = "transposes + TN " + ("fp32-out beta=1" if L.TN_FP32_OUT else "bf16 + fp32 add")
            else:
                wpath = "NT fp32-out beta=1"
        for kind, t, path in (("fwd", t_f, "F.linear"), ("dgrad", t_d, "data_grad (W^T cached)"), ("wgrad", t_w, wpath)):
            rows.append((name, kind, N, K, T, t * 1e3, fl / t / 1e12, 100 * fl / t / PEAK, path))
        del w, x, gy, buf
        torch.cuda.empty_cache()
    print(f"| GEMM | pass | N | K | tokens | ms | TFLOP/s | % of 2.5 PF | path |\n|---|---|---:|---:|---:|---:|---:|---:|---|")
    for r in rows:
        print(f"| {r[0]} | {r[1]} | {r[2]} | {r[3]} | {r[4]} | {r[5]:.3f} | {r[6]:.0f} | {r[7]:.1f} | {r[8]} |")
    tun = torch.cuda.tunable
    try:
        res = tun.get_results()
        print("\nTunableOp solutions in use (op, shape, solution, ms):")
        for r in res:
            print("  ", *r)
    except Exception as e:  # noqa: BLE001
        print("TunableOp results unavailable:", e)


if __name__ == "__main__":
    main()
