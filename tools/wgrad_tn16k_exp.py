"""Weight-gradient layout experiment at the bench's 16,384 tokens per micro-step (MI355X).

dW[out, in] (+)= dY^T X, dY [T, out], X [T, in] bf16, fp32 accumulator. Compares
(a) the hand-written k-major wgrad kernel (ops/linear.py's current path, accumulate),
(b) hipBLASLt bf16 "TN" on operands that a producer kernel already wrote transposed,
(c) (b) + fp32 accumulate pass, (d) TN with fp32 output accumulating in the epilogue (beta=1),
first with the packaged TunableOp table (lookup only), then after TunableOp tunes (b)/(d).
The transposed copies are made OUTSIDE the timed region: the question is what a producer-fused
transposed write buys.
usage: python tools/wgrad_tn16k_exp.py [tokens]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shuffle_exchange_amd.ops import native  # noqa: E402
from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms  # noqa: E402

native.require_hip()
load_tuned_gemms()
T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384


def t(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


shapes = [(28672, 4096), (4096, 14336), (4096, 4096), (6144, 4096)]
data = {}
for (O, I) in shapes:
    dy = torch.randn(T, O, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
    acc = torch.zeros(O, I, device="cuda")
    dyt, xt = torch.ops.sxe.transpose16(dy), torch.ops.sxe.transpose16(x)
    data[(O, I)] = (dy, x, acc, dyt, xt)


def run(tag):
    for (O, I), (dy, x, acc, dyt, xt) in data.items():
        fl = 2 * T * O * I / 1e9
        a = t(lambda: torch.ops.sxe.wgrad_gemm_(dy, x, acc, 1.0, True))
        b = t(lambda: torch.mm(dyt, xt.t()))
        c = t(lambda: acc.add_(torch.mm(dyt, xt.t())))
        d = t(lambda: torch.ops.aten.addmm.dtype_out(acc, dyt, xt.t(), torch.float32, beta=1, alpha=1, out=acc))
        tr = t(lambda: torch.ops.sxe.transpose16(dy))
        ref = (dy.float().t() @ x.float())
        dw = torch.mm(dyt, xt.t()).float()
        err = ((dw - ref).norm() / ref.norm()).item()
        print(f"[{tag}] [{O}x{I}] T={T} sxe-wgrad {a:.3f} ms {fl / a:.0f} TF | bf16TN {b:.3f} {fl / b:.0f} | "
              f"TN+add {c:.3f} {fl / c:.0f} | fusedTN {d:.3f} {fl / d:.0f} | dY transpose {tr:.3f} | "
              f"bf16TN rel err {err:.1e}", flush=True)


run("table")
tun = torch.cuda.tunable
tun.tuning_enable(True)
tun.set_max_tuning_duration(30)
tun.set_max_tuning_iterations(20)
tun.set_filename(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "tn16k_tuned%d.csv"))
run("tuned")
tun.write_file()
