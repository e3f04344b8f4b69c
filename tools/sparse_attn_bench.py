"""Block-sparse flash attention vs dense flash attention at long sequence (MI355X)."""
import os, sys, time, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shuffle_exchange_amd.ops import sparse_attention as sa
from shuffle_exchange_amd.ops.attention import attention
def t(fn, n=5):
    for _ in range(2): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e3
B, H, S, D = 1, 16, 16384, 128
q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
g = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16)
for name, conf in [("bigbird64", sa.BigBirdSparsityConfig(H, block=64, num_random_blocks=2, num_sliding_window_blocks=5,
                                                           num_global_blocks=2)),
                   ("longformer128", sa.BSLongformerSparsityConfig(H, block=128, num_sliding_window_blocks=9)),
                   ("fixed64", sa.FixedSparsityConfig(H, block=64, num_local_blocks=8))]:
    lay = conf.make_layout(S)
    dens = lay.float().mean().item()
    f = lambda: sa.block_sparse_attention(q, k, v, lay, conf.block)
    tf = t(f); tb = t(lambda: torch.autograd.grad(f(), (q, k, v), g))
    print(f"{name}: density {dens:.3f} | fwd {tf:.2f} ms | fwd+bwd {tb:.2f} ms", flush=True)
qt, kt, vt = (x.detach().transpose(1, 2).requires_grad_() for x in (q, k, v))
fd = lambda: attention(qt, kt, vt, causal=False)
print(f"dense (full): fwd {t(fd):.2f} ms | fwd+bwd {t(lambda: torch.autograd.grad(fd(), (qt, kt, vt), g.transpose(1, 2))):.2f} ms")
