"""Tune the distinct GEMM shapes of the Llama-3-8B training step with PyTorch TunableOp (hipBLASLt
solution search only, bounded per solution) and report tuned-vs-default TFLOP/s per shape.

Standalone (no model): every shape is issued exactly like ops/linear.py issues it -- forward
``x @ W.T``, input grad on a transposed weight ``gy @ (W^T)^T`` (data_grad), weight grad as
transposes + forward-layout GEMM (TN path) or the fp32-accumulating ``addmm.dtype_out``. Writes the TunableOp CSV that
runtime/gemm_tuning.py loads (SXE_TUNABLEOP_FILE or the packaged tuning/ file).

usage: python tools/tune_gemms.py OUT.csv [tokens] [--max-ms 8] [--iters 10]
"""
import argparse
import os
import sys
import threading
import time

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("tokens", nargs="?", type=int, default=8192)
ap.add_argument("--max-ms", type=int, default=8)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--hidden", type=int, default=4096)
ap.add_argument("--inter", type=int, default=14336)
ap.add_argument("--qkv", type=int, default=6144)
ap.add_argument("--vocab", type=int, default=128256)
a = ap.parse_args()
os.environ.setdefault("PYTORCH_TUNABLEOP_ROCBLAS_ENABLED", "0")
import torch  # noqa: E402

done = False


def beat():
    t0 = time.time()
    while not done:
        time.sleep(20)
        print(f"[tune] alive {time.time() - t0:.0f}s", flush=True)


threading.Thread(target=beat, daemon=True).start()
T, H = a.tokens, a.hidden
layers = {"qkv": (a.qkv, H), "o": (H, H), "gate_up": (2 * a.inter, H), "down": (H, a.inter), "lm_head": (a.vocab, H)}
dev = "cuda"


def timeit(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


cases = []
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shuffle_exchange_amd.ops import native  # noqa: E402
from shuffle_exchange_amd.ops.linear import DGRAD_WT_MIN_ELEMS, TN_MIN_ELEMS  # noqa: E402
native.require_hip()
tr = torch.ops.sxe.transpose16
for name, (N, K) in layers.items():
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    gy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    acc = torch.zeros(N, K, device=dev, dtype=torch.float32)
    fl = 2.0 * T * N * K
    cases.append((f"{name} fwd", fl, lambda x=x, w=w: x @ w.t()))
    if N * K >= DGRAD_WT_MIN_ELEMS:  # ops/linear.data_grad: forward-layout GEMM on a transposed weight
        wt = tr(w)
        cases.append((f"{name} dgrad-wT", fl, lambda gy=gy, wt=wt: gy @ wt.t()))
    else:
        cases.append((f"{name} dgrad", fl, lambda gy=gy, w=w: gy @ w))
    if N * K >= TN_MIN_ELEMS:  # ops/linear.write_weight_grad TN path: transposes + forward-layout GEMM
        gyt, xt = tr(gy), tr(x)
        cases.append((f"{name} wgrad-TN", fl, lambda gyt=gyt, xt=xt: gyt @ xt.t()))
    else:
        cases.append((f"{name} wgrad-fp32acc", fl,
                      lambda gy=gy, x=x, acc=acc: torch.ops.aten.addmm.dtype_out(acc, gy.t(), x, torch.float32,
                                                                                  beta=1, alpha=1, out=acc)))

base = {}
for nm, fl, fn in cases:
    base[nm] = timeit(fn)
    print(f"[default] {nm:24s} {base[nm] * 1e3:8.3f} ms {fl / base[nm] / 1e12:7.0f} TF/s", flush=True)

tun = torch.cuda.tunable
tun.enable(True)
tun.tuning_enable(True)
tun.set_filename(a.out)
tun.set_max_tuning_duration(a.max_ms)
tun.set_max_tuning_iterations(a.iters)
for nm, fl, fn in cases:
    t0 = time.time()
    fn()
    torch.cuda.synchronize()
    print(f"[tuning] {nm} took {time.time() - t0:.1f}s", flush=True)
tun.tuning_enable(False)  # results are flushed to the file at exit
tot_b = tot_t = 0.0
for nm, fl, fn in cases:
    t = timeit(fn)
    tot_b += base[nm]
    tot_t += t
    print(f"[tuned]   {nm:24s} {t * 1e3:8.3f} ms {fl / t / 1e12:7.0f} TF/s  (default {fl / base[nm] / 1e12:5.0f})",
          flush=True)
print(f"[tune] sum of shapes: default {tot_b * 1e3:.2f} ms -> tuned {tot_t * 1e3:.2f} ms", flush=True)
done = True
print("[tune] wrote", a.out, flush=True)
sys.exit(0)
