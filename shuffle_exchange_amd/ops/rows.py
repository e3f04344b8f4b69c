"""Row gather / scatter on the gfx950 kernels of csrc/kernels/rows.hip (16-byte chunks, one wave
per row), with autograd and CPU fallbacks.

* ``gather_rows(src, idx, offset=0, add=None)``: out[i] = src[idx[i] - offset] (+ add[...]); an
  index outside the table gives a zero row (vocab-shard embedding semantics);
* ``scatter_rows_(dst, idx, src)``: dst[idx[i]] = src[i] for unique indices;
* ``embed(weight, ids, offset=0)``: ragged embedding lookup (reference ragged_ops/embed);
* ``gather_last(x, last, res=None)``: last-token rows (+ the fused residual) for the LM head
  (reference ragged_ops/logits_gather);
* ``gather_tokens`` / ``scatter_tokens``: random-LTD token selection on [B, S, H] with per-batch
  sorted indices (reference ops/random_ltd gather_scatter), differentiable.
"""
import torch

from . import native


def _hip_rows(t):
    return (t.is_cuda and native.use_hip(t) and t.dim() == 2 and t.is_contiguous()
            and (t.shape[1] * t.element_size()) % 16 == 0 and t.data_ptr() % 16 == 0)


def gather_rows(src, idx, offset=0, add=None):
    idx = idx.reshape(-1)
    if _hip_rows(src) and (add is None or _hip_rows(add)) and idx.dtype in (torch.int32, torch.int64):
        return torch.ops.sxe.gather_rows(src, idx.contiguous(), int(offset), add)
    s = idx.long() - offset
    ok = (s >= 0) & (s < src.shape[0])
    rows = src.index_select(0, s.clamp(0, max(src.shape[0] - 1, 0)))
    if add is not None:
        rows = rows + add.index_select(0, s.clamp(0, max(src.shape[0] - 1, 0)))
    return rows * ok.unsqueeze(1).to(rows.dtype) if not bool(ok.all()) else rows


def scatter_rows_(dst, idx, src):
    idx = idx.reshape(-1)
    if _hip_rows(dst) and _hip_rows(src) and idx.dtype in (torch.int32, torch.int64):
        torch.ops.sxe.scatter_rows_(dst, idx.contiguous(), src)
        return dst
    dst.index_copy_(0, idx.long(), src)
    return dst


def embed(weight, ids, offset=0):
    """Inference embedding lookup (no autograd): [T] ids -> [T, H]."""
    return gather_rows(weight, ids, offset)


def gather_last(x, last, res=None):
    """x[last] (+ res[last]) for the final norm + LM head of a ragged batch."""
    return gather_rows(x, last, 0, res)


def _flat_index(idx, S):
    B = idx.shape[0]
    return (idx + torch.arange(B, device=idx.device, dtype=idx.dtype).unsqueeze(1) * S).reshape(-1)


class _GatherTokens(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, idx):
        B, S, H = x.shape
        flat = _flat_index(idx, S)
        ctx.save_for_backward(flat)
        ctx.shape = x.shape
        return gather_rows(x.reshape(B * S, H), flat).view(B, idx.shape[1], H)

    @staticmethod
    def backward(ctx, g):
        (flat,) = ctx.saved_tensors
        B, S, H = ctx.shape
        gx = g.new_zeros(B * S, H)
        scatter_rows_(gx, flat, g.reshape(-1, H).contiguous())
        return gx.view(B, S, H), None


class _ScatterTokens(torch.autograd.Function):
    @staticmethod
    def forward(ctx, full, part, idx):
        B, S, H = full.shape
        flat = _flat_index(idx, S)
        ctx.save_for_backward(flat)
        out = full.contiguous().clone().view(B * S, H)
        scatter_rows_(out, flat, part.reshape(-1, H).contiguous())
        return out.view(B, S, H)

    @staticmethod
    def backward(ctx, g):
        (flat,) = ctx.saved_tensors
        B, S, H = g.shape
        g2 = g.contiguous().view(B * S, H)
        gpart = gather_rows(g2, flat).view(B, -1, H)
        gfull = g2.clone()
        scatter_rows_(gfull, flat, torch.zeros_like(gpart).view(-1, H))
        return gfull.view(B, S, H), gpart, None


def gather_tokens(x, idx):
    """x [B, S, H], idx [B, k] (unique per row) -> [B, k, H]."""
    return _GatherTokens.apply(x.contiguous(), idx)


def scatter_tokens(full, part, idx):
    """Out of place: full [B, S, H] with rows idx [B, k] replaced by part [B, k, H]."""
    return _ScatterTokens.apply(full, part, idx)
