"""Weight-gradient GEMM layout experiment on MI355X: dW[out,in] = dY^T X with dY [T,out], X [T,in].
(a) fused fp32-out NT (current), (b) bf16 NT, (c) transposed copies + TN bf16 + fp32 add,
(d) transposed copies + TN fp32-out fused accumulate, (e) transposes alone."""
import os, sys, time, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms
load_tuned_gemms()
def t(fn, n=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e3
T = 8192
for (O, I) in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]:
    dy = torch.randn(T, O, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
    acc = torch.zeros(O, I, device="cuda")
    dyt, xt = dy.t().contiguous(), x.t().contiguous()
    fl = 2 * T * O * I / 1e9
    a = t(lambda: torch.ops.aten.addmm.dtype_out(acc, dy.t(), x, torch.float32, beta=1, alpha=1, out=acc))
    b = t(lambda: torch.mm(dy.t(), x))
    tn = t(lambda: torch.mm(dyt, xt.t()))
    tr = t(lambda: (dy.t().contiguous(), x.t().contiguous()))
    d = t(lambda: torch.ops.aten.addmm.dtype_out(acc, dyt, xt.t(), torch.float32, beta=1, alpha=1, out=acc))
    add = t(lambda: acc.add_(torch.mm(dyt, xt.t())))
    print(f"[{O}x{I}] fusedNT {a:.3f}ms {fl/a:.0f}TF | bf16NT {b:.3f} {fl/b:.0f} | bf16TN {tn:.3f} {fl/tn:.0f} | "
          f"transposes {tr:.3f} | fusedTN {d:.3f} {fl/d:.0f} | TN+add {add:.3f}", flush=True)
