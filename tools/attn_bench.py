"""Time the flash attention kernels alone at the Llama-3-8B shape (fwd, fwd+bwd) vs SDPA."""
import sys, time, torch
sys.path.insert(0, '.')
from shuffle_exchange_amd.ops.attention import attention, _sdpa
B, S, H, Hk, D = int(sys.argv[1]) if len(sys.argv) > 1 else 4, 2048, 32, 8, 128
q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, S, Hk, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, S, Hk, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
flops = 4 * B * H * S * S * D / 2
def t(fn, n=10):
    for _ in range(2): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n
g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
for name, f in [("hip", lambda: attention(q, k, v)), ("sdpa", lambda: _sdpa(q, k, v, True, D ** -0.5))]:
    tf = t(f); tb = t(lambda: torch.autograd.grad(f(), (q, k, v), g))
    print(f"{name}: fwd {tf*1e3:.2f} ms {flops/tf/1e12:.0f} TF | fwd+bwd {tb*1e3:.2f} ms {3.5*flops/tb/1e12:.0f} TF | bwd only {(tb-tf)*1e3:.2f} ms", flush=True)
