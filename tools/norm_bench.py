"""RMSNorm forward (+ residual) and backward HIP kernels (csrc/kernels/norm.hip) at the Llama-3-8B
training shape (16k tokens x 4096, bf16): time per call and effective HBM bandwidth.
  python tools/norm_bench.py   (SXE_NORM_EXACT=0: the bounds-checked variants)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


def main():
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    R, H = 16384, 4096
    x = torch.randn(R, H, device="cuda", dtype=torch.bfloat16)
    res = torch.randn_like(x)
    w = torch.rand(H, device="cuda", dtype=torch.bfloat16) + 0.5
    dy = torch.randn_like(x)
    y, rstd, mean, h = torch.ops.sxe.norm_fwd(x, res, w, None, 1e-5, False)
    tf = t(lambda: torch.ops.sxe.norm_fwd(x, res, w, None, 1e-5, False))
    tf0 = t(lambda: torch.ops.sxe.norm_fwd(x, None, w, None, 1e-5, False))
    tb = t(lambda: torch.ops.sxe.norm_bwd(dy, h, rstd, None, w, dy, False))
    mb = R * H * 2 / 1e6
    print(json.dumps({"exact": os.environ.get("SXE_NORM_EXACT", "1"), "fwd_res_ms": round(tf, 4),
                      "fwd_res_TBps": round(4 * mb / tf / 1e3, 2), "fwd_ms": round(tf0, 4),
                      "fwd_TBps": round(2 * mb / tf0 / 1e3, 2), "bwd_dres_ms": round(tb, 4),
                      "bwd_TBps": round(4 * mb / tb / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
