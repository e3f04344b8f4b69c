"""wgrad via HIP transposes + TN GEMM + fp32 add vs fused NT addmm (MI355X)."""
import os, sys, time, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shuffle_exchange_amd.ops import native
from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms
native.require_hip(); load_tuned_gemms()
def t(fn, n=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e3
x = torch.randn(640, 1984, device="cuda", dtype=torch.bfloat16)
assert torch.equal(torch.ops.sxe.transpose16(x), x.t().contiguous()), "transpose16 wrong"
T = 8192
for (O, I) in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]:
    dy = torch.randn(T, O, device="cuda", dtype=torch.bfloat16)
    xx = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
    acc = torch.zeros(O, I, device="cuda")
    fl = 2 * T * O * I / 1e9
    a = t(lambda: torch.ops.aten.addmm.dtype_out(acc, dy.t(), xx, torch.float32, beta=1, alpha=1, out=acc))
    tr = t(lambda: (torch.ops.sxe.transpose16(dy), torch.ops.sxe.transpose16(xx)))
    def tn():
        dyt, xt = torch.ops.sxe.transpose16(dy), torch.ops.sxe.transpose16(xx)
        acc.add_(torch.mm(dyt, xt.t()))
    b = t(tn)
    gb = (dy.numel() + xx.numel()) * 2 * 2 / 1e6
    print(f"[{O}x{I}] fusedNT {a:.3f} ms ({fl/a:.0f} TF) | HIP transposes {tr:.3f} ms ({gb/tr:.0f} GB/s) | "
          f"transpose+TN+add {b:.3f} ms ({fl/b:.0f} TF) | gain {a-b:+.3f} ms", flush=True)
    del dy, xx, acc
