"""Causal/non-causal multi-head attention with GQA, layout [B, S, H, D] (no transposes around the
QKV / output projections).

Backends:
* ``hip``  -- this repo's gfx950 flash-attention kernels (csrc/kernels/flash_attn.hip): MFMA bf16,
  online softmax, LSE output for backward / FPDT chunk merging;
* ``sdpa`` -- ``torch.nn.functional.scaled_dot_product_attention`` (the stopgap SURVEY §7.2 step 4
  allows until the HIP kernel covers a shape; always used on CPU).
Selection: ``SXE_ATTN_BACKEND`` env (hip|sdpa), else hip when the kernel supports the shape.
"""
import math
import os

import torch
import torch.nn.functional as F

from . import native
from ..utils.logging import warning_once


def _sdpa(q, k, v, causal, scale):
    # [B,S,H,D] -> [B,H,S,D] views; SDPA handles GQA via enable_gqa
    qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    gqa = qt.shape[1] != kt.shape[1]
    if gqa and not q.is_cuda:
        rep = qt.shape[1] // kt.shape[1]
        kt = kt.repeat_interleave(rep, dim=1)
        vt = vt.repeat_interleave(rep, dim=1)
        gqa = False
    o = F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal, scale=scale, enable_gqa=gqa)
    return o.transpose(1, 2)


def _hip_supported(q, k, v):
    D = q.shape[-1]
    return (q.is_cuda and q.dtype == torch.bfloat16 and D in (64, 128) and q.shape[2] % k.shape[2] == 0
            and hasattr(torch.ops.sxe, "flash_attn_fwd"))


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        o, lse = torch.ops.sxe.flash_attn_fwd(q, k, v, bool(causal), float(scale))
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = torch.ops.sxe.flash_attn_bwd(do.contiguous(), q, k, v, o, lse, bool(ctx.causal), float(ctx.scale))
        return dq, dk, dv, None, None


def attention(q, k, v, causal=True, softmax_scale=None, backend=None):
    """q: [B, S, Hq, D], k/v: [B, S, Hkv, D] (strided views allowed) -> [B, S, Hq, D]."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    backend = backend or os.environ.get("SXE_ATTN_BACKEND")
    if q.is_cuda and backend != "sdpa":
        native.require_hip()
        if _hip_supported(q, k, v):
            return _FlashAttn.apply(q, k, v, causal, scale)
        warning_once(f"sxe attention: HIP kernel does not cover dtype={q.dtype} D={q.shape[-1]}; using SDPA")
    return _sdpa(q, k, v, causal, scale)


def attention_with_lse(q, k, v, causal=True, softmax_scale=None):
    """Forward-only attention returning (out, lse[B, H, S]) for chunk merging (FPDT)."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if q.is_cuda and _hip_supported(q, k, v):
        return torch.ops.sxe.flash_attn_fwd(q, k, v, bool(causal), float(scale))
    qt, kt, vt = q.transpose(1, 2).float(), k.transpose(1, 2).float(), v.transpose(1, 2).float()
    if kt.shape[1] != qt.shape[1]:
        rep = qt.shape[1] // kt.shape[1]
        kt, vt = kt.repeat_interleave(rep, 1), vt.repeat_interleave(rep, 1)
    s = torch.matmul(qt, kt.transpose(-1, -2)) * scale
    if causal:
        S, T = s.shape[-2], s.shape[-1]
        mask = torch.ones(S, T, dtype=torch.bool, device=s.device).tril(T - S)
        s = s.masked_fill(~mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    o = torch.matmul(torch.softmax(s, dim=-1), vt)
    return o.transpose(1, 2).to(q.dtype), lse
