"""Workload for rocprofv3 --pmc passes over the round-6 training-step kernels at the Llama-3-8B
headline shapes (a few dispatches each): xent_grad_dual (16,384 x 128,256), acc2_bf16_ (the gate_up
weight gradient, 117 M elements), the dual-layout gated kernels (16k x 14336) and transpose16
(16k x 4096). Run under: rocprofv3 --pmc <counters> --output-format csv -d DIR -o pmc -- python3
tools/pmc_step_kernels.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    bf = dict(device="cuda", dtype=torch.bfloat16)
    T, V, H, I = 16384, 128256, 4096, 14336
    logits = torch.randn(T, V, **bf)
    tgt = torch.randint(0, V, (T,), device="cuda")
    lse = torch.logsumexp(logits[:64].float(), -1).repeat(T // 64)
    one = torch.ones(1, device="cuda")
    for _ in range(2):
        torch.ops.sxe.xent_grad_dual(logits, tgt, lse, -100, one, one)
    del logits
    n = 2 * I * H
    dst = torch.zeros(n, device="cuda")
    a, b = torch.randn(n, **bf), torch.randn(n, **bf)
    for _ in range(2):
        torch.ops.sxe.acc2_bf16_(dst, a, b, True)
    del dst, a, b
    gu, d = torch.randn(T, 2 * I, **bf), torch.randn(T, I, **bf)
    for _ in range(2):
        torch.ops.sxe.gated_act_fwd_dual(gu, 3, 4)
        torch.ops.sxe.gated_act_bwd_dual(d, gu, 3, 4)
    x = torch.randn(T, H, **bf)
    for _ in range(2):
        torch.ops.sxe.transpose16(x)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
