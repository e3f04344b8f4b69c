"""Micro-benchmark of the paged-attention decode kernel (HIP graph of N back-to-back calls, so
launch overhead is excluded): time per call vs batch, context, splits and KV-cache size.
  python tools/paged_attn_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(B, ctx, nq=32, nkv=8, D=128, bs=64, total_blocks=None, splits=None, reps=20):
    from shuffle_exchange_amd.ops.paged_attention import choose_splits
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    nb = (ctx + bs - 1) // bs
    total_blocks = total_blocks or B * nb
    cache = torch.randn(total_blocks, 2, nkv, bs, D, device="cuda", dtype=torch.bfloat16)
    perm = torch.randperm(total_blocks, device="cuda")[:B * nb].to(torch.int32)
    bt = perm.view(B, nb).contiguous()
    q = torch.randn(B, nq, D, device="cuda", dtype=torch.bfloat16)
    qs = torch.arange(B, device="cuda", dtype=torch.int32)
    ql = torch.ones(B, device="cuda", dtype=torch.int32)
    kl = torch.full((B,), ctx, device="cuda", dtype=torch.int32)
    sp = splits or choose_splits(B, nkv, ctx)
    f = lambda: torch.ops.sxe.paged_attention(q, cache, bt, qs, ql, kl, D ** -0.5, ctx, sp)  # noqa: E731
    f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / (5 * reps) * 1e3
    kv_bytes = B * ctx * nkv * D * 2 * 2
    return {"B": B, "ctx": ctx, "splits": sp, "cache_GB": round(cache.numel() * 2 / 1e9, 2), "us": round(us, 2),
            "TB_per_s": round(kv_bytes / us / 1e6, 2)}


def main():
    for B, ctx in ((1, 1024), (1, 8192), (8, 1024), (32, 1024), (64, 2048), (128, 4096)):
        print(json.dumps(bench(B, ctx)), flush=True)
    for sp in (1, 2, 4, 8, 16):
        print(json.dumps(bench(1, 4096, splits=sp)), flush=True)
    print(json.dumps(bench(1, 1024, total_blocks=131072)), flush=True)  # 34 GB cache, scattered blocks


if __name__ == "__main__":
    main()
