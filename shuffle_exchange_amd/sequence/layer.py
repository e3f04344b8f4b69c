"""Ulysses sequence parallelism: head <-> sequence all-to-all around a local attention.

Parity: reference deepspeed/sequence/layer.py -- ``DistributedAttention`` :331-440,
``_SeqAllToAll`` :277, ``single_all_to_all`` :221-254 -- and the ALST HF path
(runtime/sequence_parallel/ulysses_sp.py:47 ``UlyssesSPAttentionHF``, GQA kv replication :117-138).

Layout here is batch-first [B, S, H, D] (what the QKV projection produces), so the exchange is:
  [B, S/p, H, D] --a2a--> [B, S, H/p, D]   (scatter heads, gather sequence)
and back for the output. MI355X-first differences:
* the fused QKV path (``ulysses_qkv_attention``) moves q, k and v in ONE all_to_all_single (the
  reference issues three, a TODO at sequence/layer.py:388): per destination rank the send buffer
  holds that rank's q heads, then k heads, then v heads, so the receiver gets a packed
  [B, S, Hq/p + 2*Hkv/p, D] tensor that the flash kernel reads in place;
* RoPE is applied before the exchange with global positions (sp_rank * S/p offset), inside the
  same HIP kernel call that rotates q and k;
* on one 8-GPU node an all-to-all is a full-mesh exchange: every GPU drives all 7 xGMI links.
"""
import torch
import torch.nn as nn

from .. import comm as dist


def _a2a(x, group):
    out = torch.empty_like(x)
    dist.all_to_all_single(out, x.contiguous(), group=group)
    return out


def seq_to_head(x, group):
    """[B, S_l, H, D] -> [B, S, H/p, D]."""
    p = dist.get_world_size(group)
    if p == 1:
        return x
    B, Sl, H, D = x.shape
    send = x.reshape(B, Sl, p, H // p, D).permute(2, 0, 1, 3, 4).contiguous()  # [p, B, Sl, H/p, D]
    recv = _a2a(send, group)  # [p(src seq chunk), B, Sl, H/p, D]
    return recv.permute(1, 0, 2, 3, 4).reshape(B, p * Sl, H // p, D)


def head_to_seq(x, group):
    """[B, S, H/p, D] -> [B, S_l, H, D]."""
    p = dist.get_world_size(group)
    if p == 1:
        return x
    B, S, Hp, D = x.shape
    Sl = S // p
    send = x.reshape(B, p, Sl, Hp, D).permute(1, 0, 2, 3, 4).contiguous()  # [p(dst seq chunk), B, Sl, H/p, D]
    recv = _a2a(send, group)  # [p(src head group), B, Sl, H/p, D]
    return recv.permute(1, 2, 0, 3, 4).reshape(B, Sl, p * Hp, D)


class _SeqAllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, group, x, to_heads):
        ctx.group, ctx.to_heads = group, to_heads
        return seq_to_head(x, group) if to_heads else head_to_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return None, (head_to_seq(g, ctx.group) if ctx.to_heads else seq_to_head(g, ctx.group)), None


class DistributedAttention(nn.Module):
    """Wrap any local attention ``fn(q, k, v, *args, **kw) -> [B, S, H/p, D]`` (batch-first)."""

    def __init__(self, local_attention, sequence_process_group, scatter_idx=2, gather_idx=1, sp_stream=None):
        super().__init__()
        self.local_attn = local_attention
        self.spg = sequence_process_group
        self.scatter_idx, self.gather_idx = scatter_idx, gather_idx

    def forward(self, query, key, value, *args, **kwargs):
        q = _SeqAllToAll.apply(self.spg, query, True)
        k = _SeqAllToAll.apply(self.spg, key, True)
        v = _SeqAllToAll.apply(self.spg, value, True)
        o = self.local_attn(q, k, v, *args, **kwargs)
        return _SeqAllToAll.apply(self.spg, o, False)


# ------------------------------------------------------------------------------------------------
def _pack_heads(qkv, nq, nkv, p):
    """[B, Sl, nq+2nkv, D] -> [p, B, Sl, (nq+2nkv)/p, D] with (q_j, k_j, v_j) heads for dest j."""
    B, Sl, _, D = qkv.shape
    q = qkv[:, :, :nq].reshape(B, Sl, p, nq // p, D)
    k = qkv[:, :, nq:nq + nkv].reshape(B, Sl, p, nkv // p, D)
    v = qkv[:, :, nq + nkv:].reshape(B, Sl, p, nkv // p, D)
    return torch.cat([q, k, v], dim=3).permute(2, 0, 1, 3, 4).contiguous()


def _unpack_heads(send, nq, nkv, p):
    """inverse of _pack_heads: [p, B, Sl, (nq+2nkv)/p, D] -> [B, Sl, nq+2nkv, D]."""
    P, B, Sl, Hp, D = send.shape
    x = send.permute(1, 2, 0, 3, 4)  # [B, Sl, p, Hp, D]
    q = x[:, :, :, :nq // p].reshape(B, Sl, nq, D)
    k = x[:, :, :, nq // p:nq // p + nkv // p].reshape(B, Sl, nkv, D)
    v = x[:, :, :, nq // p + nkv // p:].reshape(B, Sl, nkv, D)
    return torch.cat([q, k, v], dim=2)


class _QKVSeqToHead(torch.autograd.Function):
    """Packed qkv [B, S/p, nq+2nkv, D] -> [B, S, (nq+2nkv)/p, D] with ONE all-to-all."""

    @staticmethod
    def forward(ctx, group, qkv, nq, nkv):
        p = dist.get_world_size(group)
        ctx.group, ctx.nq, ctx.nkv = group, nq, nkv
        recv = _a2a(_pack_heads(qkv, nq, nkv, p), group)  # [p(src chunk), B, Sl, Hp, D]
        P, B, Sl, Hp, D = recv.shape
        return recv.permute(1, 0, 2, 3, 4).reshape(B, P * Sl, Hp, D)

    @staticmethod
    def backward(ctx, g):
        p = dist.get_world_size(ctx.group)
        B, S, Hp, D = g.shape
        send = g.reshape(B, p, S // p, Hp, D).permute(1, 0, 2, 3, 4).contiguous()
        back = _a2a(send, ctx.group)  # [p(head group j), B, Sl, Hp, D]
        return None, _unpack_heads(back, ctx.nq, ctx.nkv, p), None, None


def _replicate_kv(qkv, nq, nkv, p):
    """GQA with fewer kv heads than SP ranks: replicate kv heads so each rank gets one
    (ALST rule, reference ulysses_sp.py:117-138)."""
    rep = p // nkv
    q = qkv[:, :, :nq]
    k = qkv[:, :, nq:nq + nkv].repeat_interleave(rep, dim=2)
    v = qkv[:, :, nq + nkv:].repeat_interleave(rep, dim=2)
    return torch.cat([q, k, v], dim=2), nkv * rep


def ulysses_qkv_attention(qkv, nq, nkv, rope, group, position_ids=None, causal=True, softmax_scale=None):
    """Sequence-parallel attention on a packed QKV chunk [B, S/p, nq+2nkv, D] -> [B, S/p, nq, D]."""
    from ..ops.attention import attention_qkv_rope
    from ..ops.rope import apply_rope_qkv_
    p = dist.get_world_size(group)
    r = dist.get_rank(group)
    B, Sl, _, D = qkv.shape
    if rope is not None:
        pos = position_ids
        if pos is None:
            pos = (torch.arange(Sl, device=qkv.device) + r * Sl).unsqueeze(0).expand(B, Sl)
        qkv = apply_rope_qkv_(qkv, rope, nq + nkv, pos)
    if nkv % p != 0:
        qkv, nkv = _replicate_kv(qkv, nq, nkv, p)
    assert nq % p == 0 and nkv % p == 0, f"heads ({nq}, {nkv}) must be divisible by sp={p}"
    full = _QKVSeqToHead.apply(group, qkv, nq, nkv)  # [B, S, (nq+2nkv)/p, D]
    o = attention_qkv_rope(full, nq // p, nkv // p, None, None, causal=causal, softmax_scale=softmax_scale)
    return _SeqAllToAll.apply(group, o, False)  # [B, S/p, nq, D]
