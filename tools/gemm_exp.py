"""GEMM experiments on MI355X: fp32-accumulating weight-grad GEMM (addmm.dtype_out) vs bf16 mm + add."""
import time, torch
def t(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n
dev = "cuda"
T = 8192
for (N, K) in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]:
    gy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    acc = torch.zeros(N, K, device=dev, dtype=torch.float32)
    def fused():
        torch.ops.aten.addmm.dtype_out(acc, gy.t(), x, torch.float32, beta=1, alpha=1, out=acc)
    def unfused():
        g = gy.t() @ x
        acc.add_(g)
    ok = True
    try:
        acc.zero_(); fused(); ref = (gy.t().float() @ x.float())
        err = ((acc - ref).norm() / ref.norm()).item()
    except Exception as e:
        ok = False; err = repr(e)[:200]
    fl = 2 * T * N * K
    tf = t(fused) if ok else float('nan'); tu = t(unfused)
    print(f"dW [{N}x{K}] K={T}: fused addmm.dtype_out {tf*1e3:.3f} ms ({fl/tf/1e12:.0f} TF) err={err} | mm+add {tu*1e3:.3f} ms ({fl/tu/1e12:.0f} TF)", flush=True)
