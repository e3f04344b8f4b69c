"""Can the MLP keep its big activations token-minor (transposed) end to end? (MI355X, bf16)

If gated_fwd / gated_bwd wrote h^T [I, T] / dgu^T [2I, T] INSTEAD of the token-major tensors, the
weight-gradient GEMMs would run in hipBLASLt's fast K-contiguous layout with no extra HBM traffic --
provided the other consumers of those tensors (down-proj forward, gate_up data-grad) stay fast when
fed the transposed view. This times every operand-layout combination of those consumers at the
bench's 16,384 tokens (packaged TunableOp table, lookup only; new layouts use hipBLASLt defaults).
usage: python tools/act_layout_exp.py [tokens]
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


def bf(*s):
    return torch.randn(*s, device="cuda", dtype=torch.bfloat16)


# data grad of gate_up: dx[T, H] = dgu[T, 2I] @ Wgu[2I, H]; and of down: dh[T, I] = dout[T, H] @ Wd[H, I]
for name, (N, K) in {"gate_up dgrad": (28672, 4096), "down dgrad": (4096, 14336), "o dgrad": (4096, 4096)}.items():
    dy, w = bf(T, N), bf(N, K)
    dyt, wt = torch.ops.sxe.transpose16(dy), torch.ops.sxe.transpose16(w)
    fl = 2 * T * N * K / 1e9
    r = [t(lambda: dy @ wt.t()), t(lambda: dy @ w), t(lambda: dyt.t() @ w), t(lambda: dyt.t() @ wt.t())]
    print(f"[{name}] T={T} dY@(W^T)^T {r[0]:.3f} ms {fl / r[0]:.0f} TF | dY@W {r[1]:.3f} {fl / r[1]:.0f} | "
          f"(dY^T)^T@W {r[2]:.3f} {fl / r[2]:.0f} | (dY^T)^T@(W^T)^T {r[3]:.3f} {fl / r[3]:.0f}", flush=True)

# forward of down / o: out[T, H] = h[T, I] @ Wd[H, I]^T, with h given transposed (h^T [I, T])
for name, (O, I) in {"down fwd": (4096, 14336), "o fwd": (4096, 4096), "gate_up fwd": (28672, 4096)}.items():
    x, w = bf(T, I), bf(O, I)
    xt, wt = torch.ops.sxe.transpose16(x), torch.ops.sxe.transpose16(w)
    fl = 2 * T * O * I / 1e9
    r = [t(lambda: x @ w.t()), t(lambda: xt.t() @ w.t()), t(lambda: xt.t() @ wt)]
    print(f"[{name}] T={T} X@W^T {r[0]:.3f} ms {fl / r[0]:.0f} TF | (X^T)^T@W^T {r[1]:.3f} {fl / r[1]:.0f} | "
          f"(X^T)^T@W^T(materialised) {r[2]:.3f} {fl / r[2]:.0f}", flush=True)

# the gated kernels: current token-major bandwidth, for the cost of a transposed write
gu, d = bf(T, 28672), bf(T, 14336)
g1 = t(lambda: torch.ops.sxe.gated_act_fwd(gu, 3))
g2 = t(lambda: torch.ops.sxe.gated_act_bwd(d, gu, 3))
tr = t(lambda: torch.ops.sxe.transpose16(gu))
print(f"[gated] fwd {g1:.3f} ms ({3 * T * 14336 * 2 / g1 / 1e9:.2f} TB/s) | bwd {g2:.3f} ms "
      f"({5 * T * 14336 * 2 / g2 / 1e9:.2f} TB/s) | transpose16 of gu {tr:.3f} ms "
      f"({2 * T * 28672 * 2 / tr / 1e9:.2f} TB/s)", flush=True)

# dual-layout kernels (token-major + token-minor outputs), per tile variant
for v, name in enumerate(["64x64", "64x128", "128x64", "128x128", "64x256"]):
    f = t(lambda: torch.ops.sxe.gated_act_fwd_dual(gu, 3, v))
    b = t(lambda: torch.ops.sxe.gated_act_bwd_dual(d, gu, 3, v))
    print(f"[gated dual {name}] fwd {f:.3f} ms ({4 * T * 14336 * 2 / f / 1e9:.2f} TB/s) | bwd {b:.3f} ms "
          f"({7 * T * 14336 * 2 / b / 1e9:.2f} TB/s)", flush=True)
