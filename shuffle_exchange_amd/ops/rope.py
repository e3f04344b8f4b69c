"""Rotary position embeddings applied in place on the fused QKV buffer.

Layout: ``qkv`` is ``[B, S, Hq + 2*Hkv, D]`` (the QKV projection output viewed per head). The
first ``Hq + Hkv`` heads (q then k) are rotated in one HIP launch; v is untouched. The autograd
function marks ``qkv`` dirty and rotates the incoming gradient back (the rotation is orthogonal,
so backward = forward with sin negated).
"""
import torch

from . import native


class RopeCache:
    """fp32 cos/sin tables [max_pos, D/2] (Llama-3 uses theta = 500000)."""

    def __init__(self, head_dim, max_pos, theta=10000.0, device=None, scaling=None):
        inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
        if scaling is not None:
            inv = scaling(inv)
        t = torch.arange(max_pos, dtype=torch.float64)
        f = torch.outer(t, inv)
        self.cos = f.cos().float().to(device)
        self.sin = f.sin().float().to(device)
        self.head_dim = head_dim
        self.max_pos = max_pos

    def to(self, device):
        self.cos = self.cos.to(device)
        self.sin = self.sin.to(device)
        return self


def _ref_rope(x, cos, sin, pos):
    # x: [T, H, D] float
    half = x.shape[-1] // 2
    c = cos[pos][:, None, :]
    s = sin[pos][:, None, :]
    a, b = x[..., :half], x[..., half:]
    return torch.cat([a * c - b * s, b * c + a * s], dim=-1)


def _positions(B, S, pos_offset, device):
    return (torch.arange(S, device=device) + pos_offset).repeat(B)


class _RopeQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, n_rot, pos, pos_offset):
        B, S = qkv.shape[0], qkv.shape[1]
        x = qkv[:, :, :n_rot, :]
        torch.ops.sxe.rope_(x, cos, sin, pos, S, int(pos_offset), False)
        ctx.mark_dirty(qkv)
        ctx.save_for_backward(cos, sin, pos)
        ctx.n_rot, ctx.pos_offset = n_rot, pos_offset
        return qkv

    @staticmethod
    def backward(ctx, g):
        cos, sin, pos = ctx.saved_tensors
        g = g.contiguous().clone() if not g.is_contiguous() else g.clone()
        S = g.shape[1]
        torch.ops.sxe.rope_(g[:, :, :ctx.n_rot, :], cos, sin, pos, S, int(ctx.pos_offset), True)
        return g, None, None, None, None, None


def apply_rope_qkv_(qkv, cache, n_rot, position_ids=None, pos_offset=0):
    """Rotate the first ``n_rot`` heads of ``qkv`` [B, S, H_total, D] in place; returns qkv."""
    pos = position_ids.reshape(-1).contiguous().long() if position_ids is not None else None
    if native.use_hip(qkv):
        return _RopeQKV.apply(qkv, cache.cos, cache.sin, n_rot, pos, pos_offset)
    B, S, Ht, D = qkv.shape
    if pos is None:
        pos = _positions(B, S, pos_offset, qkv.device)
    x = qkv[:, :, :n_rot, :].reshape(B * S, n_rot, D).float()
    r = _ref_rope(x, cache.cos.to(qkv.device), cache.sin.to(qkv.device), pos).to(qkv.dtype).view(B, S, n_rot, D)
    return torch.cat([r, qkv[:, :, n_rot:, :]], dim=2)


def apply_rope(x, cache, position_ids=None, pos_offset=0):
    """Out-of-place RoPE on a [B, S, H, D] tensor (used by the Ulysses/inference paths)."""
    x = x.contiguous()
    H = x.shape[2]
    if native.use_hip(x):
        return _RopeQKV.apply(x.clone(), cache.cos, cache.sin, H,
                              position_ids.reshape(-1).contiguous().long() if position_ids is not None else None,
                              pos_offset)
    return apply_rope_qkv_(x, cache, H, position_ids, pos_offset)


def apply_rope_tokens_(qkv, cache, n_rot, positions, rot_dim=None):
    """In-place RoPE on the first ``n_rot`` heads of a ragged token batch ``qkv`` [T, H, D] with
    absolute ``positions`` [T] (inference engine; no autograd). ``rot_dim`` < D rotates only the
    first ``rot_dim`` dims of each head (partial rotary: Phi, GPT-NeoX); ``cache`` is built for it."""
    T = qkv.shape[0]
    if T == 0:
        return qkv
    rd = rot_dim or qkv.shape[-1]
    pos = positions.reshape(-1).contiguous().long()
    if native.use_hip(qkv) and rd % 16 == 0:
        torch.ops.sxe.rope_(qkv.unsqueeze(0)[:, :, :n_rot, :rd], cache.cos, cache.sin, pos, T, 0, False)
        return qkv
    x = qkv[:, :n_rot, :rd].float()
    qkv[:, :n_rot, :rd] = _ref_rope(x, cache.cos.to(qkv.device), cache.sin.to(qkv.device), pos).to(qkv.dtype)
    return qkv
