"""Can the MLP GEMMs read the token-minor copies instead of the token-major ones? hipBLASLt time of
  dgrad gate_up: dx[T, H] = dgu[T, 2I] @ Wgu[2I, H]   -- current: dgu row-major x cached Wgu^T
                  vs dguT.t() @ Wgu (A column-major, the dual kernel's token-minor copy only)
  fwd down:       y[T, H]  = h[T, I] @ Wd^T          -- current: F.linear(h, Wd)
                  vs hT.t() @ Wd.t() (A column-major)
at 16,384 tokens (Llama-3-8B). python tools/colmajor_a_bench.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms
    load_tuned_gemms()
    T, H, I = 16384, 4096, 14336
    d = dict(device="cuda", dtype=torch.bfloat16)
    dgu = torch.randn(T, 2 * I, **d)
    dguT = dgu.t().contiguous()
    wgu = torch.randn(2 * I, H, **d) * 0.02
    wguT = wgu.t().contiguous()
    h = torch.randn(T, I, **d)
    hT = h.t().contiguous()
    wd = torch.randn(H, I, **d) * 0.02
    fl_dx, fl_down = 2.0 * T * H * 2 * I, 2.0 * T * H * I
    rows = [("dgrad gate_up: dgu @ (Wgu^T)^T [current]", lambda: torch.mm(dgu, wguT.t()), fl_dx),
            ("dgrad gate_up: dgu @ Wgu (NN)", lambda: torch.mm(dgu, wgu), fl_dx),
            ("dgrad gate_up: dguT^T @ Wgu", lambda: torch.mm(dguT.t(), wgu), fl_dx),
            ("dgrad gate_up: dguT^T @ (Wgu^T)^T", lambda: torch.mm(dguT.t(), wguT.t()), fl_dx),
            ("fwd down: F.linear(h, Wd) [current]", lambda: torch.nn.functional.linear(h, wd), fl_down),
            ("fwd down: hT^T @ Wd^T", lambda: torch.mm(hT.t(), wd.t()), fl_down)]
    for name, fn, fl in rows:
        t = timeit(fn)
        print(f"{name:45s} {t * 1e3:7.3f} ms {fl / t / 1e12:7.0f} TF", flush=True)


if __name__ == "__main__":
    main()
