"""Causal/non-causal multi-head attention with GQA, layout [B, S, H, D] (no transposes around the
QKV / output projections).

Backends:
* ``hip``  -- this repo's gfx950 flash-attention kernels (csrc/kernels/flash_attn.hip): MFMA bf16,
  online softmax, LSE output; deterministic backward (dK/dV kernel + dQ kernel, no atomics); head
  dims 64 / 128 / 256 natively, query length != key length (cross / prefix attention, causal mask
  bottom-right aligned as in flash-attn: query i sees keys <= i + Sk - Sq);
* ``sdpa`` -- ``torch.nn.functional.scaled_dot_product_attention``: CPU (plumbing tests) and head
  dims above 256 on GPU (logged once so a silent fallback cannot hide in a benchmark).

Shapes outside the kernels' native tiles run the same kernels on padded copies: each sequence axis
is zero-padded to the next multiple of 128 (padded keys are masked with the kernels' ``kv_len``,
padded query rows are dropped, the causal offset is the one of the true lengths) and other head
dims (80, 96, 160, ...) are zero-padded to the next native one (zero q/k columns leave the scores
unchanged, zero v columns produce zero output columns that are dropped). The softmax scale is the
true head dim's. ``SXE_ATTN_BACKEND=sdpa`` forces the stopgap for A/B comparisons.

``attention_qkv_rope`` is the training entry point of the Llama family: it takes the fused QKV
projection output [B, S, Hq + 2*Hkv, D], applies RoPE in place, runs attention reading q/k/v as
strided views, and in backward writes dq/dk/dv straight into ONE dqkv buffer (then rotates the
dq/dk slices back in place) -- no per-view gradient scatter, no transposes, no clones.
"""
import math
import os

import torch
import torch.nn.functional as F

from . import native
from ..utils.logging import warning_once


def _sdpa(q, k, v, causal, scale):
    qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    gqa = qt.shape[1] != kt.shape[1]
    if gqa and not q.is_cuda:
        rep = qt.shape[1] // kt.shape[1]
        kt = kt.repeat_interleave(rep, dim=1)
        vt = vt.repeat_interleave(rep, dim=1)
        gqa = False
    o = F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal, scale=scale, enable_gqa=gqa)
    return o.transpose(1, 2)


TILE = 128
HEAD_DIMS = (64, 128, 256)


def _native_dim(D):
    for d in HEAD_DIMS:  # a plain loop: generator builtins are graph breaks under torch.compile
        if d >= D:
            return d
    return None


def _aligned(t):
    # 16-byte aligned rows: base allocations are 512-B aligned, so the element offset decides. Under
    # torch.compile the offset is not traceable (storage_offset() is a graph break): the strides
    # decide there and the kernel's own host check (flash_attn.hip) refuses a misaligned base loudly.
    ok = t.stride(-1) == 1 and t.stride(0) % 8 == 0 and t.stride(1) % 8 == 0 and t.stride(2) % 8 == 0
    if torch.compiler.is_compiling():
        return ok
    return ok and (t.storage_offset() * t.element_size()) % 16 == 0


def hip_supported(q, k, v):
    """The kernels run these tensors in place (no padding copies)."""
    if os.environ.get("SXE_ATTN_BACKEND") == "sdpa":
        return False
    return (q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] in HEAD_DIMS and q.shape[1] % TILE == 0
            and k.shape[1] % TILE == 0 and k.shape[-1] == q.shape[-1] and v.shape[-1] == q.shape[-1]
            and q.shape[2] % k.shape[2] == 0 and _aligned(q) and _aligned(k) and _aligned(v))


def hip_paddable(q, k, v):
    """The kernels run these tensors on padded copies (sequence axes and/or head dim)."""
    if os.environ.get("SXE_ATTN_BACKEND") == "sdpa":
        return False
    return (q.is_cuda and q.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and _native_dim(q.shape[-1]) is not None and q.shape[-1] % 8 == 0 and k.shape[-1] == q.shape[-1]
            and v.shape[-1] == q.shape[-1] and q.shape[2] % k.shape[2] == 0)


def _pad(t, S_pad, D_pad):
    B, S, H, D = t.shape
    if S == S_pad and D == D_pad and t.dtype == torch.bfloat16 and _aligned(t):
        return t
    out = torch.zeros(B, S_pad, H, D_pad, dtype=torch.bfloat16, device=t.device)
    out[:, :S, :, :D].copy_(t)
    return out


def _padded_fwd(q, k, v, causal, scale):
    Sq, Sk, D = q.shape[1], k.shape[1], q.shape[-1]
    Dp = _native_dim(D)
    Sqp, Skp = -(-Sq // TILE) * TILE, -(-Sk // TILE) * TILE
    qp, kp, vp = _pad(q, Sqp, Dp), _pad(k, Skp, Dp), _pad(v, Skp, Dp)
    o, lse = torch.ops.sxe.flash_attn_fwd(qp, kp, vp, bool(causal), float(scale), Sk, Sk - Sq)
    return qp, kp, vp, o, lse


class _FlashAttnPadded(torch.autograd.Function):
    """Flash attention on padded copies (see the module docstring)."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        Sq, Sk, D = q.shape[1], k.shape[1], q.shape[-1]
        qp, kp, vp, o, lse = _padded_fwd(q, k, v, causal, scale)
        ctx.save_for_backward(qp, kp, vp, o, lse)
        ctx.meta = (causal, scale, Sq, Sk, D, q.dtype)
        return o[:, :Sq, :, :D].to(q.dtype)

    @staticmethod
    def backward(ctx, do):
        qp, kp, vp, o, lse = ctx.saved_tensors
        causal, scale, Sq, Sk, D, dtype = ctx.meta
        dop = _pad(do, qp.shape[1], qp.shape[-1])
        dq, dk, dv = torch.empty_like(qp), torch.empty_like(kp), torch.empty_like(vp)
        torch.ops.sxe.flash_attn_bwd(dop, qp, kp, vp, o, lse, dq, dk, dv, bool(causal), float(scale), Sk, Sk - Sq)
        sq = (slice(None), slice(0, Sq), slice(None), slice(0, D))
        sk = (slice(None), slice(0, Sk), slice(None), slice(0, D))
        return dq[sq].to(dtype), dk[sk].to(dtype), dv[sk].to(dtype), None, None


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
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        torch.ops.sxe.flash_attn_bwd(do.contiguous(), q, k, v, o, lse, dq, dk, dv, bool(ctx.causal),
                                     float(ctx.scale))
        return dq, dk, dv, None, None


def attention(q, k, v, causal=True, softmax_scale=None):
    """q: [B, Sq, Hq, D], k/v: [B, Sk, Hkv, D] (strided views allowed) -> [B, Sq, Hq, D]. With Sq != Sk
    and ``causal`` the mask is bottom-right aligned (query i sees keys <= i + Sk - Sq)."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if q.is_cuda:
        native.require_hip()
        if hip_supported(q, k, v):
            return _FlashAttn.apply(q, k, v, causal, scale)
        if hip_paddable(q, k, v):
            return _FlashAttnPadded.apply(q, k, v, causal, scale)
        warning_once(f"sxe attention: HIP flash kernel does not cover dtype={q.dtype} D={q.shape[-1]} "
                     f"S={q.shape[1]}; using SDPA")
    return _sdpa(q, k, v, causal, scale)


class _FlashAttnQKVRope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, nq, nkv, causal, scale, pos):
        B, S = qkv.shape[0], qkv.shape[1]
        if cos is not None:
            torch.ops.sxe.rope_(qkv[:, :, :nq + nkv], cos, sin, pos, S, 0, False)
        q, k, v = qkv[:, :, :nq], qkv[:, :, nq:nq + nkv], qkv[:, :, nq + nkv:]
        o, lse = torch.ops.sxe.flash_attn_fwd(q, k, v, bool(causal), float(scale))
        # qkv (the fresh QKV-projection output, consumed only here) was rotated in place; it is
        # saved AFTER the rotation, and no other autograd node holds it, so it is not marked dirty
        # (a dirty view input would forbid returning it).
        ctx.save_for_backward(qkv, o, lse, cos, sin, pos)
        ctx.meta = (nq, nkv, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, cos, sin, pos = ctx.saved_tensors
        nq, nkv, causal, scale = ctx.meta
        dqkv = torch.empty_like(qkv)
        q, k, v = qkv[:, :, :nq], qkv[:, :, nq:nq + nkv], qkv[:, :, nq + nkv:]
        dq, dk, dv = dqkv[:, :, :nq], dqkv[:, :, nq:nq + nkv], dqkv[:, :, nq + nkv:]
        torch.ops.sxe.flash_attn_bwd(do.contiguous(), q, k, v, o, lse, dq, dk, dv, bool(causal), float(scale))
        if cos is not None:
            torch.ops.sxe.rope_(dqkv[:, :, :nq + nkv], cos, sin, pos, qkv.shape[1], 0, True)
        return dqkv, None, None, None, None, None, None, None


def attention_qkv_rope(qkv, nq, nkv, rope=None, position_ids=None, causal=True, softmax_scale=None):
    """qkv: [B, S, nq + 2*nkv, D] fused projection output. Returns o [B, S, nq, D]."""
    D = qkv.shape[-1]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    q, k, v = qkv[:, :, :nq], qkv[:, :, nq:nq + nkv], qkv[:, :, nq + nkv:]
    if qkv.is_cuda:
        native.require_hip()
        if hip_supported(q, k, v):
            pos = position_ids.reshape(-1).contiguous().long() if position_ids is not None else None
            cos = rope.cos if rope is not None else None
            sin = rope.sin if rope is not None else None
            return _FlashAttnQKVRope.apply(qkv, cos, sin, nq, nkv, causal, scale, pos)
    if rope is not None:
        from .rope import apply_rope_qkv_
        qkv = apply_rope_qkv_(qkv, rope, nq + nkv, position_ids)
    q, k, v = qkv[:, :, :nq], qkv[:, :, nq:nq + nkv], qkv[:, :, nq + nkv:]
    return attention(q, k, v, causal, scale)


QKV_TN = os.environ.get("SXE_QKV_TN", "1") == "1"


class _QKVProjAttn(torch.autograd.Function):
    """QKV projection + RoPE + attention as ONE autograd node (GPU bf16 training). It keeps x^T
    (token-minor) instead of x and transposes dqkv in the backward, so the QKV weight gradient runs
    as hipBLASLt's TN fp32-out GEMM (0.62 ms at 16k tokens x 6144 x 4096) instead of the token-major
    NT one (0.84 ms); the two transposes cost ~0.13 ms (profiles/r06/wgrad_variants_16k.log)."""

    @staticmethod
    def forward(ctx, x, w, cos, sin, nq, nkv, causal, scale, pos):
        B, S, H = x.shape
        x2 = x.reshape(-1, H)
        qkv = F.linear(x2, w).view(B, S, nq + 2 * nkv, -1)
        if cos is not None:
            torch.ops.sxe.rope_(qkv[:, :, :nq + nkv], cos, sin, pos, S, 0, False)
        q, k, v = qkv[:, :, :nq], qkv[:, :, nq:nq + nkv], qkv[:, :, nq + nkv:]
        o, lse = torch.ops.sxe.flash_attn_fwd(q, k, v, bool(causal), float(scale))
        xT = torch.ops.sxe.transpose16(x2) if ctx.needs_input_grad[1] else None
        ctx.save_for_backward(xT, qkv, o, lse, cos, sin, pos, w)
        ctx.meta = (nq, nkv, causal, scale, x.shape)
        return o

    @staticmethod
    def backward(ctx, do):
        xT, qkv, o, lse, cos, sin, pos, w = ctx.saved_tensors
        nq, nkv, causal, scale, x_shape = ctx.meta
        dqkv = torch.empty_like(qkv)
        q, k, v = qkv[:, :, :nq], qkv[:, :, nq:nq + nkv], qkv[:, :, nq + nkv:]
        dq, dk, dv = dqkv[:, :, :nq], dqkv[:, :, nq:nq + nkv], dqkv[:, :, nq + nkv:]
        torch.ops.sxe.flash_attn_bwd(do.contiguous(), q, k, v, o, lse, dq, dk, dv, bool(causal), float(scale))
        del q, k, v, o, lse, qkv
        if cos is not None:
            torch.ops.sxe.rope_(dqkv[:, :, :nq + nkv], cos, sin, pos, dqkv.shape[1], 0, True)
        d2 = dqkv.view(-1, w.shape[0])
        from .linear import data_grad
        from .mlp import weight_grad_tn
        dx = data_grad(d2, w).view(x_shape) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            dw = weight_grad_tn(w, torch.ops.sxe.transpose16(d2), xT, fp32_out=True)
        return dx, dw, None, None, None, None, None, None, None


def qkv_proj_attention(x, qkv_proj, nq, nkv, rope=None, position_ids=None, causal=True, softmax_scale=None):
    """``attention_qkv_rope(qkv_proj(x))`` for x [B, S, H]; one fused autograd node (``_QKVProjAttn``)
    when the shapes, dtypes and the plain bias-free projection allow, else the two-step path."""
    B, S, H = x.shape
    w = getattr(qkv_proj, "weight", None)
    from .mlp import _plain
    N = (nq + 2 * nkv)
    if (QKV_TN and x.is_cuda and x.dtype == torch.bfloat16 and torch.is_grad_enabled() and _plain(qkv_proj)
            and (w.requires_grad or x.requires_grad) and (B * S) % 64 == 0 and H % 64 == 0 and w.shape[1] == H
            and w.shape[0] % (64 * N) == 0 and native.use_hip(x)):
        D = w.shape[0] // N
        # hip_supported() for the q / k / v views of a fresh contiguous [B, S, N, D] projection
        if D in HEAD_DIMS and S % TILE == 0 and nq % nkv == 0 and os.environ.get("SXE_ATTN_BACKEND") != "sdpa":
            scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
            pos = position_ids.reshape(-1).contiguous().long() if position_ids is not None else None
            cos = rope.cos if rope is not None else None
            sin = rope.sin if rope is not None else None
            return _QKVProjAttn.apply(x, w, cos, sin, nq, nkv, causal, scale, pos)
    qkv = qkv_proj(x).view(B, S, N, -1)
    return attention_qkv_rope(qkv, nq, nkv, rope, position_ids, causal, softmax_scale)


def attention_with_lse(q, k, v, causal=True, softmax_scale=None):
    """Forward-only attention returning (out [B,S,H,D], lse [B,H,S]) for chunk merging (FPDT)."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if q.is_cuda and hip_supported(q, k, v):
        return torch.ops.sxe.flash_attn_fwd(q, k, v, bool(causal), float(scale))
    if q.is_cuda and hip_paddable(q, k, v):
        Sq, D = q.shape[1], q.shape[-1]
        _, _, _, o, lse = _padded_fwd(q, k, v, causal, scale)
        return o[:, :Sq, :, :D].to(q.dtype), lse[:, :, :Sq].contiguous()
    return reference_attention(q, k, v, causal, scale, return_lse=True)


def reference_attention(q, k, v, causal=True, scale=None, return_lse=False):
    """fp32 eager oracle used by the tests (and the CPU path of attention_with_lse)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
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
    o = torch.matmul(torch.softmax(s, dim=-1), vt).transpose(1, 2).to(q.dtype)
    return (o, lse) if return_lse else o
