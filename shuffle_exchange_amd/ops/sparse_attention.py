"""Block-sparse self-attention with the reference's sparsity-layout zoo.

Parity: reference ops/sparse_attention -- ``SparsityConfig`` and ``Dense`` / ``Fixed`` / ``Variable``
/ ``BigBird`` / ``BSLongformer`` / ``LocalSlidingWindow`` configs (sparsity_config.py:10-727, layout
``[num_heads, S/block, S/block]``), ``SparseSelfAttention`` (sparse_self_attention.py:12: q/k/v
``[B, H, S, D]``, softmax scale ``D**-0.5``, key-padding / attention masks, rpe),
``BertSparseSelfAttention`` and ``SparseAttentionUtils`` (pad to a block multiple).

MI355X path: the reference runs three Triton block-sparse kernels (SDD matmul -> block softmax ->
DSD matmul) that materialise the sparse score blocks in HBM. Here the layout drives this repo's
flash-attention kernels directly (``flash_attn_fwd_sparse`` / ``flash_attn_bwd_sparse`` in
csrc/kernels/flash_attn.hip): every workgroup compacts the list of 64-key (forward, dQ) or 32-query
(dK/dV) tiles that touch a non-zero block, skips the rest, and masks inside the tiles it visits --
scores never leave registers and work scales with the layout density. Inputs ``[B, H, S, D]`` are
consumed through strided views (no transposes). Head dims 64 / 128 / 256 run natively, other
dims up to 256 zero-padded to the next of those; fp16 inputs run in bf16; additive masks and rpe
use the fp32 reference path (logged once).
"""
import math
import random

import torch
import torch.nn as nn

from . import native
from ..utils.logging import warning_once


# ------------------------------------------------------------------------------------- layouts
class SparsityConfig:
    def __init__(self, num_heads, block=16, different_layout_per_head=False):
        self.num_heads, self.block, self.different_layout_per_head = num_heads, block, different_layout_per_head
        self.num_layout_heads = num_heads if different_layout_per_head else 1

    def setup_layout(self, seq_len):
        if seq_len % self.block:
            raise ValueError(f"sequence length {seq_len} must be divisible by block size {self.block}")
        nb = seq_len // self.block
        return torch.zeros(self.num_heads, nb, nb, dtype=torch.int64)

    def check_and_propagate_first_head_layout(self, layout):
        if not self.different_layout_per_head:
            layout[1:] = layout[0]
        return layout

    def make_layout(self, seq_len):
        raise NotImplementedError

    @staticmethod
    def _causal(layout, attention):
        return torch.tril(layout) if attention == "unidirectional" else layout


class DenseSparsityConfig(SparsityConfig):
    def make_layout(self, seq_len):
        return torch.ones_like(self.setup_layout(seq_len))


def _local_windows(nb, sizes):
    """(start, end) of consecutive local windows: sizes[0], sizes[1], ..., then sizes[-1] repeated."""
    out, start = [], 0
    for i in range(10 ** 9):
        w = sizes[min(i, len(sizes) - 1)]
        if start >= nb:
            break
        out.append((start, min(start + w, nb)))
        start += w
    return out


def _fill_windows(layout, h, windows, attention):
    for s, e in windows:
        blk = torch.ones(e - s, e - s, dtype=layout.dtype)
        layout[h, s:e, s:e] = torch.tril(blk) if attention == "unidirectional" else blk


class FixedSparsityConfig(SparsityConfig):
    """Sparse Transformer "fixed" pattern: local windows + per-window global representatives."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_local_blocks=4, num_global_blocks=1,
                 attention="bidirectional", horizontal_global_attention=False, num_different_global_patterns=1):
        super().__init__(num_heads, block, different_layout_per_head)
        if num_local_blocks % num_global_blocks:
            raise ValueError("num_local_blocks must be divisible by num_global_blocks")
        if attention not in ("unidirectional", "bidirectional"):
            raise NotImplementedError("only uni/bi-directional attention")
        if horizontal_global_attention and attention != "bidirectional":
            raise ValueError("horizontal global attention needs bidirectional attention")
        if num_different_global_patterns > 1 and not different_layout_per_head:
            raise ValueError("several global patterns need different_layout_per_head")
        if num_different_global_patterns > num_local_blocks // num_global_blocks:
            raise ValueError("too many global patterns for the local window")
        self.num_local_blocks, self.num_global_blocks = num_local_blocks, num_global_blocks
        self.attention, self.horizontal_global_attention = attention, horizontal_global_attention
        self.num_different_global_patterns = num_different_global_patterns

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        nb, L, G = layout.shape[1], self.num_local_blocks, self.num_global_blocks
        for h in range(self.num_layout_heads):
            _fill_windows(layout, h, _local_windows(nb, [L]), self.attention)
            first = L - (1 + h % self.num_different_global_patterns) * G
            full_end = nb - nb % L
            starts = list(range(first, full_end, L))
            if full_end < nb:  # short last window: its global block(s) sit at the same offset, clamped
                starts.append(min(full_end + first, nb - G))
            for st in starts:
                row0 = 0 if self.attention == "bidirectional" else st
                layout[h, row0:, st:st + G] = 1
                if self.horizontal_global_attention:
                    layout[h, st:st + G, :] = 1
        return self.check_and_propagate_first_head_layout(layout)


class VariableSparsityConfig(SparsityConfig):
    """Fixed-like pattern with variable local windows, explicit global blocks and random blocks."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_random_blocks=0,
                 local_window_blocks=(4,), global_block_indices=(0,), global_block_end_indices=None,
                 attention="bidirectional", horizontal_global_attention=False):
        super().__init__(num_heads, block, different_layout_per_head)
        if global_block_end_indices is not None:
            if len(global_block_indices) != len(global_block_end_indices):
                raise ValueError("global start/end index lists differ in length")
            if any(s >= e for s, e in zip(global_block_indices, global_block_end_indices)):
                raise ValueError("global block start must be < end")
        if attention not in ("unidirectional", "bidirectional"):
            raise NotImplementedError("only uni/bi-directional attention")
        if horizontal_global_attention and attention != "bidirectional":
            raise ValueError("horizontal global attention needs bidirectional attention")
        self.num_random_blocks, self.local_window_blocks = num_random_blocks, list(local_window_blocks)
        self.global_block_indices = list(global_block_indices)
        self.global_block_end_indices = None if global_block_end_indices is None else list(global_block_end_indices)
        self.attention, self.horizontal_global_attention = attention, horizontal_global_attention

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        nb = layout.shape[1]
        if nb < self.num_random_blocks:
            raise ValueError("more random blocks than blocks in a row")
        ends = self.global_block_end_indices or [i + 1 for i in self.global_block_indices]
        for h in range(self.num_layout_heads):
            for row in range(nb):
                layout[h, row, random.sample(range(nb), self.num_random_blocks)] = 1
            _fill_windows(layout, h, _local_windows(nb, self.local_window_blocks), self.attention)
            for s, e in zip(self.global_block_indices, ends):
                if s >= nb:
                    continue
                e = min(e, nb)
                if self.horizontal_global_attention:
                    layout[h, s:e, :] = 1
                layout[h, (0 if self.attention == "bidirectional" else s):, s:e] = 1
        return self.check_and_propagate_first_head_layout(layout)


class BigBirdSparsityConfig(SparsityConfig):
    """BigBird: random blocks + sliding window + leading global blocks (rows and columns)."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_random_blocks=1,
                 num_sliding_window_blocks=3, num_global_blocks=1, attention="bidirectional"):
        super().__init__(num_heads, block, different_layout_per_head)
        if attention not in ("unidirectional", "bidirectional"):
            raise NotImplementedError("only uni/bi-directional attention")
        self.num_random_blocks, self.num_sliding_window_blocks = num_random_blocks, num_sliding_window_blocks
        self.num_global_blocks, self.attention = num_global_blocks, attention

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        nb = layout.shape[1]
        for name, n in (("random", self.num_random_blocks), ("sliding window", self.num_sliding_window_blocks),
                        ("global", self.num_global_blocks)):
            if nb < n:
                raise ValueError(f"number of {name} blocks {n} exceeds blocks per row {nb}")
        w = self.num_sliding_window_blocks // 2
        for h in range(self.num_layout_heads):
            for row in range(nb):
                pool = range(nb) if self.attention == "bidirectional" else range(row + 1)
                layout[h, row, random.sample(pool, self.num_random_blocks)] = 1
                layout[h, row, max(0, row - w):min(nb, row + w + 1)] = 1
            layout[h, :self.num_global_blocks, :] = 1
            layout[h, :, :self.num_global_blocks] = 1
            layout[h] = self._causal(layout[h], self.attention)
        return self.check_and_propagate_first_head_layout(layout)


class BSLongformerSparsityConfig(SparsityConfig):
    """Block-sparse Longformer: sliding window + global blocks (rows and columns)."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_sliding_window_blocks=3,
                 global_block_indices=(0,), global_block_end_indices=None, attention="bidirectional"):
        super().__init__(num_heads, block, different_layout_per_head)
        if global_block_end_indices is not None:
            if len(global_block_indices) != len(global_block_end_indices):
                raise ValueError("global start/end index lists differ in length")
            if any(s >= e for s, e in zip(global_block_indices, global_block_end_indices)):
                raise ValueError("global block start must be < end")
        self.num_sliding_window_blocks = num_sliding_window_blocks
        self.global_block_indices = list(global_block_indices)
        self.global_block_end_indices = None if global_block_end_indices is None else list(global_block_end_indices)
        self.attention = attention

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        nb = layout.shape[1]
        if nb < self.num_sliding_window_blocks:
            raise ValueError("sliding window larger than the number of blocks")
        w = self.num_sliding_window_blocks // 2
        ends = self.global_block_end_indices or [i + 1 for i in self.global_block_indices]
        for h in range(self.num_layout_heads):
            for row in range(nb):
                layout[h, row, max(0, row - w):min(nb, row + w + 1)] = 1
            for s, e in zip(self.global_block_indices, ends):
                if s < nb:
                    layout[h, s:min(e, nb), :] = 1
                    layout[h, :, s:min(e, nb)] = 1
            layout[h] = self._causal(layout[h], self.attention)
        return self.check_and_propagate_first_head_layout(layout)


class LocalSlidingWindowSparsityConfig(SparsityConfig):
    def __init__(self, num_heads, block=16, num_sliding_window_blocks=3, attention="unidirectional"):
        super().__init__(num_heads, block)
        self.num_sliding_window_blocks, self.attention = num_sliding_window_blocks, attention

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        nb = layout.shape[1]
        if nb < self.num_sliding_window_blocks:
            raise ValueError("sliding window larger than the number of blocks")
        w = self.num_sliding_window_blocks // 2
        for h in range(self.num_layout_heads):
            for row in range(nb):
                end = min(row + w + 1, nb) if self.attention == "bidirectional" else row + 1
                layout[h, row, max(0, row - w):end] = 1
        return self.check_and_propagate_first_head_layout(layout)


# ----------------------------------------------------------------------------------- attention
def sparse_attention_reference(q, k, v, layout, block, scale, causal=False, key_padding_mask=None, attn_mask=None,
                               rpe=None, kp_mask_mode="add", attn_mask_mode="mul"):
    """fp32 eager oracle on [B, H, S, D] inputs (GQA allowed)."""
    B, H, S, D = q.shape
    qf, kf, vf = q.float(), k.float(), v.float()
    if kf.shape[1] != H:
        kf, vf = kf.repeat_interleave(H // kf.shape[1], 1), vf.repeat_interleave(H // vf.shape[1], 1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if rpe is not None:
        s = s + rpe.float()
    if attn_mask is not None:
        s = s * attn_mask.float() if attn_mask_mode == "mul" else s + attn_mask.float()
    if key_padding_mask is not None:
        kp = key_padding_mask.float().view(B, 1, 1, S)
        s = s * kp if kp_mask_mode == "mul" else s + kp
    allowed = layout.bool().repeat_interleave(block, 1).repeat_interleave(block, 2).to(s.device)  # [H, S, S]
    if causal:
        allowed = allowed & torch.ones(S, S, dtype=torch.bool, device=s.device).tril()
    s = s.masked_fill(~allowed.unsqueeze(0), float("-inf"))
    p = torch.softmax(s, dim=-1).nan_to_num(0.0)
    return torch.matmul(p, vf).to(q.dtype)


_NATIVE_D = (64, 128, 256)


def _hip_ok(q, k, block):
    """Shapes the flash kernels run: any head dim <= 256 (64 / 128 / 256 natively, others zero-padded
    to the next of those), bf16 or fp16 (fp16 runs in bf16), S a multiple of 128, GQA."""
    return (q.is_cuda and q.dtype in (torch.bfloat16, torch.float16) and q.shape[-1] <= 256 and q.shape[2] % 128 == 0
            and block % 16 == 0 and q.shape[1] % k.shape[1] == 0)


class _SparseFlash(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, layout, block, causal, scale):
        # [B, H, S, D] -> [B, S, H, D] views (strides only)
        qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
        o, lse = torch.ops.sxe.flash_attn_fwd_sparse(qt, kt, vt, layout, int(block), bool(causal), float(scale))
        ctx.save_for_backward(q, k, v, o, lse, layout)
        ctx.meta = (block, causal, scale)
        return o.transpose(1, 2)

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, layout = ctx.saved_tensors
        block, causal, scale = ctx.meta
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        dot = do.transpose(1, 2).contiguous()
        torch.ops.sxe.flash_attn_bwd_sparse(dot, q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), o, lse,
                                            dq.transpose(1, 2), dk.transpose(1, 2), dv.transpose(1, 2), layout,
                                            int(block), bool(causal), float(scale))
        return dq, dk, dv, None, None, None, None


def block_sparse_attention(q, k, v, layout, block, causal=False, softmax_scale=None):
    """q/k/v [B, H, S, D] (k/v may have fewer heads: GQA); layout [H, S/block, S/block]."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if q.is_cuda:
        native.require_hip()
        if _hip_ok(q, k, block):
            lay = layout.to(device=q.device, dtype=torch.uint8).contiguous()
            D, dt = q.shape[-1], q.dtype
            Dn = next(d for d in _NATIVE_D if d >= D)
            if dt != torch.bfloat16:
                q, k, v = q.to(torch.bfloat16), k.to(torch.bfloat16), v.to(torch.bfloat16)
            if Dn != D:  # zero columns change neither q.k nor p.v; the scale stays the caller's
                pad = torch.nn.functional.pad
                q, k, v = pad(q, (0, Dn - D)), pad(k, (0, Dn - D)), pad(v, (0, Dn - D))
            o = _SparseFlash.apply(q, k, v, lay, block, causal, scale)
            return (o[..., :D] if Dn != D else o).to(dt)
        warning_once(f"block_sparse_attention: D={q.shape[-1]} dtype={q.dtype} not covered by the HIP kernel; "
                     f"using the reference path")
    return sparse_attention_reference(q, k, v, layout, block, scale, causal)


class SparseSelfAttention(nn.Module):
    """Reference-compatible module (sparse_self_attention.py:12)."""

    def __init__(self, sparsity_config=None, key_padding_mask_mode="add", attn_mask_mode="mul",
                 max_seq_length=2048):
        super().__init__()
        self.sparsity_config = sparsity_config or SparsityConfig(num_heads=4)
        self.key_padding_mask_mode, self.attn_mask_mode = key_padding_mask_mode, attn_mask_mode
        self.max_seq_length = max_seq_length
        self._layouts = {}

    def get_layout(self, L):
        if L not in self._layouts:
            self._layouts[L] = self.sparsity_config.make_layout(L)
        return self._layouts[L]

    def forward(self, query, key, value, rpe=None, key_padding_mask=None, attn_mask=None):
        assert query.dtype in (torch.float16, torch.bfloat16, torch.float32)
        B, H, L, D = query.shape
        layout = self.get_layout(L)
        blk = self.sparsity_config.block
        if rpe is None and key_padding_mask is None and attn_mask is None:
            return block_sparse_attention(query, key, value, layout, blk)
        return sparse_attention_reference(query, key, value, layout, blk, D ** -0.5, False, key_padding_mask,
                                          attn_mask, rpe, self.key_padding_mask_mode, self.attn_mask_mode)


class BertSparseSelfAttention(nn.Module):
    """Sparse self-attention layer of a BERT model (reference bert_sparse_self_attention.py:10):
    query / key / value projections, ``SparseSelfAttention`` with the config's layout, the
    attention mask applied as a key-padding mask."""

    def __init__(self, config, sparsity_config=None):
        super().__init__()
        if config.hidden_size % config.num_attention_heads != 0:
            raise ValueError(f"The hidden size ({config.hidden_size}) is not a multiple of the number of attention "
                             f"heads ({config.num_attention_heads})")
        self.num_attention_heads = config.num_attention_heads
        self.attention_head_size = config.hidden_size // config.num_attention_heads
        self.all_head_size = self.num_attention_heads * self.attention_head_size
        self.query = nn.Linear(config.hidden_size, self.all_head_size)
        self.key = nn.Linear(config.hidden_size, self.all_head_size)
        self.value = nn.Linear(config.hidden_size, self.all_head_size)
        self.sparse_self_attention = SparseSelfAttention(sparsity_config or FixedSparsityConfig(num_heads=4))

    def transpose_for_scores(self, x):
        return x.view(*x.shape[:-1], self.num_attention_heads, self.attention_head_size).permute(0, 2, 1, 3)

    def forward(self, hidden_states, attention_mask):
        q, k, v = (self.transpose_for_scores(f(hidden_states)) for f in (self.query, self.key, self.value))
        ctx = self.sparse_self_attention(q, k, v, key_padding_mask=attention_mask)
        ctx = ctx.permute(0, 2, 1, 3).contiguous()
        return ctx.view(*ctx.shape[:-2], self.all_head_size)


class SparseAttentionUtils:
    @staticmethod
    def pad_to_block_size(block_size, input_ids, attention_mask=None, pad_token_id=0):
        S = input_ids.shape[1]
        pad = (block_size - S % block_size) % block_size
        if pad:
            input_ids = torch.nn.functional.pad(input_ids, (0, pad), value=pad_token_id)
            if attention_mask is not None:
                attention_mask = torch.nn.functional.pad(attention_mask, (0, pad), value=0)
        return pad, input_ids, attention_mask

    @staticmethod
    def unpad_sequence_output(pad_len, sequence_output):
        return sequence_output[:, :-pad_len] if pad_len > 0 else sequence_output


from .sparse_ops import MatMul, Softmax  # noqa: E402,F401  (standalone block-sparse ops)
