"""Does a memory-bound kernel overlap a compute-bound hipBLASLt GEMM on MI355X when they are issued on
two streams? Pairs from the Llama-3-8B backward at 16,384 tokens: the down-projection weight-gradient
GEMM (TN, [4096 x 14336] x K 16384) with the gated SwiGLU backward (3.3 GB of HBM traffic), and the
gate_up weight-gradient GEMM with the norm-sized transpose. Prints sequential vs two-stream time.
  python tools/stream_overlap_probe.py"""
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
    from shuffle_exchange_amd.ops import native
    from shuffle_exchange_amd.runtime.gemm_tuning import load_tuned_gemms
    native.require_hip()
    load_tuned_gemms()
    T, H, I = 16384, 4096, 14336
    d = dict(device="cuda", dtype=torch.bfloat16)
    d2T, hT = torch.randn(H, T, **d), torch.randn(I, T, **d)
    gu, dh = torch.randn(T, 2 * I, **d), torch.randn(T, I, **d)
    dguT, xT = torch.randn(2 * I, T, **d), torch.randn(H, T, **d)
    x2 = torch.randn(T, H, **d)
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()
    pairs = {
        "down wgrad GEMM + gated bwd": (lambda: torch.mm(d2T, hT.t()),
                                        lambda: torch.ops.sxe.gated_act_bwd_dual(dh, gu, 3, 4)),
        "gate_up wgrad GEMM + transpose [16k x 4096]": (lambda: torch.mm(dguT, xT.t()),
                                                        lambda: torch.ops.sxe.transpose16(x2)),
    }
    for name, (g, m) in pairs.items():
        tg, tm = timeit(g), timeit(m)

        def seq():
            g()
            m()

        def conc():
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                g()
            m()
            main_s.wait_stream(side)

        ts, tc = timeit(seq), timeit(conc)
        print(f"{name}: GEMM {tg * 1e3:.3f} ms, mem {tm * 1e3:.3f} ms, sequential {ts * 1e3:.3f} ms, "
              f"two streams {tc * 1e3:.3f} ms ({(ts - tc) * 1e3:+.3f} ms)", flush=True)


if __name__ == "__main__":
    main()
