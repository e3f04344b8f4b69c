"""MoE routing ops on the gfx950 kernels of csrc/kernels/moe.hip, with autograd.

* ``topk_softmax(logits, k)`` -> (probs, top_idx): fused softmax + top-k per token (one wave per
  token); ``probs`` is differentiable (softmax backward), ``top_idx`` int64;
* ``routing_tables(expert, location, keep, capacity, E)`` -> (slots [S, k], slot_src [E*C]): the
  forward map (assignment -> capacity slot, -1 = dropped) and its inverse (slot -> assignment,
  -1 = empty) that make dispatch / combine atomic-free gathers;
* ``dispatch(x, slots, slot_src)``: [S, H] -> [E*C, H] expert-ordered rows (empty slots zero);
* ``combine(expert_out, slots, slot_src, w)``: [E*C, H] -> [S, H], weighted by the fp32 gate
  weights ``w`` [S, k] (differentiable in both ``expert_out`` and ``w``).

Parity: reference inference/v2/kernels/ragged_ops/top_k_gating (:15), moe_scatter (:23),
moe_gather (:21); training dispatch/combine of runtime moe/sharded_moe.py:587-678. CPU tensors
(gloo plumbing tests) take the equivalent PyTorch ops.
"""
import torch
import torch.nn.functional as F

from . import native


def _hip(t):
    return t.is_cuda and native.use_hip(t)


class _TopKSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, k):
        probs, _, topi = torch.ops.sxe.moe_topk_softmax(logits.contiguous(), int(k))
        ctx.save_for_backward(probs)
        ctx.mark_non_differentiable(topi)
        return probs, topi

    @staticmethod
    def backward(ctx, gprobs, _gtopi):
        (p,) = ctx.saved_tensors
        return p * (gprobs - (gprobs * p).sum(-1, keepdim=True)), None


def topk_softmax(logits, k):
    """(softmax(logits) [S, E] fp32, indices of the k largest [S, k] int64)."""
    logits = logits.float()
    if _hip(logits) and logits.dim() == 2 and logits.shape[1] <= 512:
        return _TopKSoftmax.apply(logits, k)
    probs = F.softmax(logits, dim=1)
    return probs, torch.topk(logits, k=k, dim=1).indices


def routing_tables(expert, location, keep, capacity, num_experts):
    slots = torch.where(keep, expert * capacity + location, torch.full_like(expert, -1)).contiguous()
    flat = slots.reshape(-1)
    kept = flat >= 0
    slot_src = torch.full((num_experts * capacity,), -1, dtype=torch.int64, device=expert.device)
    slot_src.index_copy_(0, flat[kept], torch.arange(flat.numel(), device=expert.device)[kept])
    return slots, slot_src


class _Dispatch(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, slots, slot_src):
        ctx.save_for_backward(slots)
        return torch.ops.sxe.moe_dispatch(x.contiguous(), slot_src, slots.shape[1])

    @staticmethod
    def backward(ctx, g):
        (slots,) = ctx.saved_tensors
        return torch.ops.sxe.moe_gather_sum(g.contiguous(), slots, None), None, None


class _Combine(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out, slots, slot_src, w):
        out = out.contiguous()
        w = w.float().contiguous()
        ctx.save_for_backward(out, slot_src, w, slots)
        return torch.ops.sxe.moe_gather_sum(out, slots, w)

    @staticmethod
    def backward(ctx, gy):
        out, slot_src, w, slots = ctx.saved_tensors
        gout, gw = torch.ops.sxe.moe_combine_bwd(gy.contiguous(), out, slot_src, w)
        return gout, None, None, gw


def _kernel_ok(x):
    return _hip(x) and x.dim() == 2 and x.shape[1] % 8 == 0 and x.dtype in (torch.bfloat16, torch.float16,
                                                                            torch.float32)


def dispatch(x, slots, slot_src):
    if _kernel_ok(x):
        return _Dispatch.apply(x, slots, slot_src)
    k = slots.shape[1]
    src = slot_src.clamp(min=0) // k
    rows = x.index_select(0, src)
    return rows * (slot_src >= 0).unsqueeze(1).to(rows.dtype)


def combine(expert_out, slots, slot_src, w):
    if _kernel_ok(expert_out):
        return _Combine.apply(expert_out, slots, slot_src, w)
    S, k = slots.shape
    idx = slots.clamp(min=0).reshape(-1)
    rows = expert_out.index_select(0, idx).view(S, k, -1)
    ww = (w.float() * (slots >= 0)).to(rows.dtype).unsqueeze(-1)
    return (rows * ww).sum(1)


# ------------------------------------------------------------------------------ grouped expert GEMM
def expert_offsets(flat_expert, num_experts):
    """int32 [E + 1] cumulative row offsets of expert-sorted rows, computed on the device without a
    host synchronisation (torch.bincount on the GPU reads the max back to the host)."""
    counts = torch.zeros(num_experts, dtype=torch.int32, device=flat_expert.device)
    counts.index_add_(0, flat_expert, torch.ones_like(flat_expert, dtype=torch.int32))
    offs = torch.zeros(num_experts + 1, dtype=torch.int32, device=flat_expert.device)
    torch.cumsum(counts, 0, out=offs[1:])
    return offs


def grouped_gemm_ok(x, w):
    return (_hip(x) and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 2 and w.dim() == 3
            and w.is_cuda and w.shape[2] == x.shape[1] and x.shape[1] % 128 == 0 and w.shape[1] % 128 == 0)


def grouped_gemm(x, w, offsets, row_scale=None):
    """y[r] = row_scale[r] * x[r] @ w[e]^T for expert-sorted rows x [R, K], per-expert weights
    w [E, N, K] (nn.Linear layout) and device offsets [E + 1] (``expert_offsets``): ONE launch of
    the ragged MFMA kernel (csrc/kernels/grouped_gemm.hip; reference cutlass_ops/moe_gemm), no host
    sync. CPU / unsupported shapes: a per-expert loop (reads the offsets on the host)."""
    if grouped_gemm_ok(x, w):
        rs = None if row_scale is None else row_scale.reshape(-1).contiguous()
        if rs is not None and rs.dtype not in (torch.float32, torch.bfloat16):
            rs = rs.float()
        return torch.ops.sxe.grouped_gemm(x.contiguous(), w.contiguous(), offsets.to(torch.int32).contiguous(), rs)
    y = x.new_empty(x.shape[0], w.shape[1])
    off = offsets.tolist()
    for e in range(w.shape[0]):
        a, b = off[e], off[e + 1]
        if b > a:
            y[a:b] = F.linear(x[a:b], w[e])
    if row_scale is not None:
        y = (y.float() * row_scale.reshape(-1, 1).float()).to(x.dtype)
    return y
