"""Probe: are the Mixtral-arch expert weight-gradient shapes (capacity 1280 tokens) eligible for the
hand-written k-major wgrad kernel (ops/linear._sxe_wgrad_ok)? usage: python tools/probe_moe_wgrad.py"""
import torch, sys
sys.path.insert(0, ".")
from shuffle_exchange_amd.ops.linear import _sxe_wgrad_ok
from shuffle_exchange_amd.ops import native
native.require_hip()
E, C, K, N = 8, 1280, 4096, 28672
x = torch.randn(E, C, K, device="cuda", dtype=torch.bfloat16)
dy = torch.randn(E, C, N, device="cuda", dtype=torch.bfloat16)
buf = torch.zeros(E, K, N, device="cuda")
print("gate_up ok", _sxe_wgrad_ok(x[0], dy[0], buf[0]), flush=True)
h = torch.randn(E, C, 14336, device="cuda", dtype=torch.bfloat16)
d2 = torch.randn(E, C, K, device="cuda", dtype=torch.bfloat16)
buf2 = torch.zeros(E, 14336, K, device="cuda")
print("down ok", _sxe_wgrad_ok(h[0], d2[0], buf2[0]), flush=True)
