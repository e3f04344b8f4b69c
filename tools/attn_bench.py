"""Time the flash attention kernels alone (fwd, fwd+bwd) vs SDPA, per head dim; for D < 128 also
the old zero-padded-to-128 path, for Sq != Sk the prefix shape.
  python tools/attn_bench.py [B]
  python tools/attn_bench.py --shapes B,Sq,Sk,H,Hk,D,causal[;...] [--no-sdpa]"""
import json
import sys
import time

import torch

sys.path.insert(0, '.')
from shuffle_exchange_amd.ops.attention import _sdpa, attention  # noqa: E402


def t(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def run(B, Sq, Sk, H, Hk, D, causal=True, sdpa=True):
    q = torch.randn(B, Sq, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Sk, Hk, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Sk, Hk, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    # causal work: the visible fraction of the Sq x Sk score matrix (bottom-right aligned)
    frac = (1.0 - Sq / (2.0 * Sk)) if causal and Sq <= Sk else 1.0
    flops = 4 * B * H * Sq * Sk * D * frac
    g = torch.randn(B, Sq, H, D, device="cuda", dtype=torch.bfloat16)
    paths = [("hip", lambda: attention(q, k, v, causal=causal))]
    if D < 128:
        qp, kp, vp = (torch.nn.functional.pad(x.detach(), (0, 128 - D)).requires_grad_() for x in (q, k, v))
        paths.append(("hip_padded128", lambda: attention(qp, kp, vp, causal=causal, softmax_scale=D ** -0.5)))
    if Sq == Sk and sdpa:
        paths.append(("sdpa", lambda: _sdpa(q, k, v, causal, D ** -0.5)))
    for name, f in paths:
        tf = t(f)
        gg = g if name != "hip_padded128" else torch.nn.functional.pad(g, (0, 128 - D))
        ins = (q, k, v) if name != "hip_padded128" else (qp, kp, vp)
        tb = t(lambda: torch.autograd.grad(f(), ins, gg))
        print(json.dumps({"path": name, "B": B, "Sq": Sq, "Sk": Sk, "H": H, "Hk": Hk, "D": D, "causal": causal,
                          "fwd_ms": round(tf * 1e3, 3), "fwd_TF": round(flops / tf / 1e12, 1),
                          "fwdbwd_ms": round(tb * 1e3, 3), "fwdbwd_TF": round(3.5 * flops / tb / 1e12, 1)}),
              flush=True)


def main():
    if "--shapes" in sys.argv:
        spec = sys.argv[sys.argv.index("--shapes") + 1]
        for sh in spec.split(";"):
            B, Sq, Sk, H, Hk, D, c = (int(x) for x in sh.split(","))
            run(B, Sq, Sk, H, Hk, D, causal=bool(c), sdpa="--no-sdpa" not in sys.argv)
        return
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    run(B, 2048, 2048, 32, 8, 128)          # Llama-3-8B training shape
    run(B, 2048, 2048, 32, 8, 64)           # head dim 64 (BERT / GPT-2 / Phi-class)
    run(B, 2048, 2048, 16, 8, 256)          # head dim 256
    run(B, 512, 4096, 32, 8, 128)           # prefix / chunked prefill: 512 new tokens over 4k context


if __name__ == "__main__":
    main()
