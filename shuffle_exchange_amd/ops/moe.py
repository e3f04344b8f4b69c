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


GG_LOOP_MIN_ROWS = 1024  # mean rows per expert from which the per-expert hipBLASLt loop is used


def _use_expert_loop(x, w):
    """Dispatch on the measured table (profiles/grouped_gemm_bench.log): with few large experts and
    many rows each (Mixtral prefill: 2048-4096 rows per expert) the per-expert hipBLASLt GEMMs run
    1.3-1.6x the ragged kernel (1,081 vs 793 TF at 8k rows, 1,410 vs 899 TF at 32k), at the price of
    one host read of the offsets; with many small experts (Qwen-MoE: 1/3 the loop's time) or
    decode-sized inputs the single ragged launch wins, and it is the only choice inside a HIP-graph
    capture (no host sync allowed). SXE_GG_DISPATCH=kernel|loop forces one."""
    import os
    mode = os.environ.get("SXE_GG_DISPATCH", "auto")
    if mode == "kernel":
        return False
    if x.is_cuda and torch.cuda.is_current_stream_capturing():
        return False
    if mode == "loop":
        return True
    return x.shape[0] >= GG_LOOP_MIN_ROWS * w.shape[0]


def grouped_gemm(x, w, offsets, row_scale=None):
    """y[r] = row_scale[r] * x[r] @ w[e]^T for expert-sorted rows x [R, K], per-expert weights
    w [E, N, K] (nn.Linear layout) and device offsets [E + 1] (``expert_offsets``): ONE launch of
    the ragged MFMA kernel (csrc/kernels/grouped_gemm.hip; reference cutlass_ops/moe_gemm), no host
    sync -- or, for few experts with many rows each, the per-expert hipBLASLt loop
    (``_use_expert_loop``). CPU / unsupported shapes: the per-expert loop."""
    if grouped_gemm_ok(x, w) and not _use_expert_loop(x, w):
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


# ------------------------------------------------------------- mixed-precision (int8 / int4) experts
class QuantizedExperts:
    """Expert weights [E, N, K] (nn.Linear layout per expert) stored as symmetric int8 or int4 codes
    with one fp32 scale per (expert, output row, ``group`` K elements); ``group`` defaults to the
    whole row for int8 (per-channel) and 128 for int4. int4 codes are two's complement, two per
    byte, low nibble first. Used by ``grouped_gemm`` (csrc/kernels/grouped_gemm.hip
    grouped_gemm_q_kernel; reference cutlass_ops/mixed_gemm mixed_moe_gemm)."""

    def __init__(self, w, bits=8, group=None):
        assert bits in (8, 4), "QuantizedExperts: int8 or int4"
        if w.dim() == 2:
            w = w.unsqueeze(0)
        E, N, K = w.shape
        group = int(group or (K if bits == 8 else min(128, K)))
        assert K % group == 0, "QuantizedExperts: group must divide K"
        self.bits, self.group, self.shape, self.dtype = bits, group, (E, N, K), w.dtype
        g = w.detach().float().reshape(E, N, K // group, group)
        qmax = 127 if bits == 8 else 7
        scale = (g.abs().amax(-1) / qmax).clamp_min(1e-12)
        q = torch.clamp(torch.round(g / scale[..., None]), -qmax, qmax).to(torch.int32).reshape(E, N, K)
        if bits == 4:
            q = q & 0xF
            q = (q[..., 0::2] | (q[..., 1::2] << 4))
        self.q = q.to(torch.uint8).contiguous()
        self.scale = scale.contiguous()

    def dequantize(self, dtype=torch.bfloat16):
        E, N, K = self.shape
        q = self.q.to(torch.int32)
        if self.bits == 8:
            q = torch.where(q >= 128, q - 256, q)
        else:
            q = torch.stack([q & 0xF, q >> 4], -1).reshape(E, N, K)
            q = torch.where(q >= 8, q - 16, q)
        v = q.float().reshape(E, N, K // self.group, self.group) * self.scale[..., None]
        return v.reshape(E, N, K).to(dtype)

    def to(self, device):
        self.q, self.scale = self.q.to(device), self.scale.to(device)
        return self

    @property
    def nbytes(self):
        return self.q.numel() + 4 * self.scale.numel()


def grouped_gemm_q(x, w: QuantizedExperts, offsets, row_scale=None):
    """``grouped_gemm`` with int8 / int4 expert weights: one launch, codes widened to bf16 per
    staged K block inside the kernel (HBM streams 1 or 0.5 bytes per weight). CPU: per-expert loop
    over the dequantized weights."""
    E, N, K = w.shape
    if (_hip(x) and x.dtype == torch.bfloat16 and x.dim() == 2 and w.q.is_cuda and K % 128 == 0 and N % 128 == 0
            and w.group % 128 == 0 and x.shape[1] == K):
        rs = None if row_scale is None else row_scale.reshape(-1).float().contiguous()
        return torch.ops.sxe.grouped_gemm_q(x.contiguous(), w.q, w.scale, w.bits, offsets.to(torch.int32).contiguous(),
                                            rs)
    return grouped_gemm(x, w.dequantize(x.dtype), offsets, row_scale)


class IntWeight:
    """Dense int8 / int4 weight-only linear (W8A16 / W4A16) on the mixed-precision grouped kernel
    with a single group covering all rows (reference inference/v2 mixed_gemm)."""

    def __init__(self, w, bits=8, group=None):
        self.e = QuantizedExperts(w, bits, group)
        self.shape, self.dtype, self.bits = tuple(w.shape), w.dtype, bits

    def dequantize(self, dtype=torch.bfloat16):
        return self.e.dequantize(dtype)[0]

    def linear(self, x, bias=None):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if (x2.is_cuda and 0 < x2.shape[0] <= 16 and x2.dtype == torch.bfloat16 and K % 128 == 0
                and self.e.group % 32 == 0 and x2.stride(-1) == 1 and x2.stride(0) % 8 == 0
                and x2.data_ptr() % 16 == 0):
            # decode: the skinny kernel streams the codes once (csrc/kernels/skinny_dq.hip)
            native.require_hip()
            b = bias.to(torch.bfloat16).contiguous() if bias is not None else None
            y = torch.ops.sxe.skinny_gemm_dq(x2, self.e.q, self.e.scale, 8 if self.bits == 8 else 9, self.e.group, b)
            return y.view(*x.shape[:-1], self.shape[0]).to(x.dtype)
        offs = torch.zeros(2, dtype=torch.int32, device=x2.device)  # no host copy: HIP-graph capturable
        offs[1:].fill_(x2.shape[0])
        y = grouped_gemm_q(x2.to(torch.bfloat16) if x2.is_cuda else x2, self.e, offs)
        if bias is not None:
            y = y + bias.to(y.dtype)
        return y.view(*x.shape[:-1], self.shape[0]).to(x.dtype)
