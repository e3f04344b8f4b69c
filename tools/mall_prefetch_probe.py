"""Does a decode GEMM read its weight faster when the weight was just read (MI355X's 256 MB
Infinity Cache / MALL warm) than after a flush? Batch-1 skinny GEMMs of Llama-3-8B (o_proj 32 MB,
QKV 48 MB, down 112 MB), each timed alone with HIP events, cold (a 1 GB sweep first) vs warm (the
weight itself swept first).  python tools/mall_prefetch_probe.py"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    bf = torch.bfloat16
    flush = torch.empty(1 << 29, device="cuda", dtype=torch.float16)  # 1 GiB
    x = torch.randn(1, 4096, device="cuda", dtype=bf)
    for name, (N, K) in {"o_proj": (4096, 4096), "qkv": (6144, 4096), "down": (4096, 14336)}.items():
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.02
        xx = torch.randn(1, K, device="cuda", dtype=bf)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        res = {}
        for mode in ("cold", "warm", "cold", "warm"):
            ts = []
            for _ in range(20):
                flush.add_(1)  # evict: stream 1 GiB through the caches
                if mode == "warm":
                    w.sum()  # bring the weight into the Infinity Cache
                a.record()
                torch.ops.sxe.skinny_gemm(xx, w, None)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            res.setdefault(mode, []).append(statistics.median(ts))
        mb = N * K * 2 / 1e6
        out = {"gemm": name, "MB": round(mb, 1)}
        for m, v in res.items():
            t = min(v)
            out[m + "_us"] = round(t, 2)
            out[m + "_TBps"] = round(mb / t, 2)  # MB per us = TB/s
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
