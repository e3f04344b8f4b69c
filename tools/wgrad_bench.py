"""Correctness + speed of the hand-written weight-gradient GEMM vs hipBLASLt (addmm fp32-out)."""
import sys, time, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shuffle_exchange_amd.ops import native
native.require_hip()

def t(fn, n=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n

torch.manual_seed(0)
# correctness on a small case against an fp64 reference
K, M, N = 512, 512, 768
a = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
c = torch.randn(M, N, device="cuda")
ref = c.double() + 0.5 * (a.double().t() @ b.double())
torch.ops.sxe.wgrad_gemm_(a, b, c, 0.5, True)
err = ((c.double() - ref).norm() / ref.norm()).item()
print(f"correctness rel err {err:.2e}", flush=True)
assert err < 1e-3
T = 8192
for (Mo, Ni) in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]:
    gy = torch.randn(T, Mo, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, Ni, device="cuda", dtype=torch.bfloat16)
    acc = torch.zeros(Mo, Ni, device="cuda")
    acc2 = torch.zeros(Mo, Ni, device="cuda")
    torch.ops.sxe.wgrad_gemm_(gy, x, acc, 1.0, True)
    torch.ops.aten.addmm.dtype_out(acc2, gy.t(), x, torch.float32, beta=1, alpha=1, out=acc2)
    e = ((acc - acc2).norm() / acc2.norm()).item()
    fl = 2.0 * T * Mo * Ni
    t1 = t(lambda: torch.ops.sxe.wgrad_gemm_(gy, x, acc, 1.0, True))
    t2 = t(lambda: torch.ops.aten.addmm.dtype_out(acc2, gy.t(), x, torch.float32, beta=1, alpha=1, out=acc2))
    print(f"[{Mo}x{Ni}] K={T}: sxe {t1*1e3:.3f} ms {fl/t1/1e12:.0f} TF | hipBLASLt {t2*1e3:.3f} ms {fl/t2/1e12:.0f} TF | err {e:.1e}", flush=True)
    del gy, x, acc, acc2
