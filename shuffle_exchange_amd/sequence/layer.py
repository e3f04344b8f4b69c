"""Ulysses sequence parallelism: head <-> sequence all-to-all around a local attention.

Parity: reference deepspeed/sequence/layer.py -- ``DistributedAttention`` :331-440,
``_SeqAllToAll`` :277, ``single_all_to_all`` :221-254 -- and the ALST HF path
(runtime/sequence_parallel/ulysses_sp.py:47 ``UlyssesSPAttentionHF``, GQA kv replication :117-138).

``DistributedAttention`` takes any layout (reference default: sequence-first [s/p, b, h, d],
scatter_idx=2 / gather_idx=0) and uneven head counts through one general flat-range all-to-all
(``all_to_all_dims``). The model-internal fused path is batch-first [B, S, H, D] (what the QKV
projection produces):
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
import math

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


def shard_sizes(total, p):
    """Near-even split of ``total`` items over ``p`` ranks (the first ``total % p`` get one more):
    the head partition of the uneven-heads all-to-all (reference module_inject/tp_shard.py:42-74
    without the kv-head grain, which callers express by passing kv heads as ``total``)."""
    return [total // p + (1 if r < total % p else 0) for r in range(p)]


def all_to_all_dims(x, scatter_dim, gather_dim, send_sizes, recv_sizes, group, stream=None):
    """General all-to-all over ``group``: slice ``send_sizes[j]`` of ``x`` along ``scatter_dim``
    goes to rank j; the pieces received from ranks 0..p-1 (``recv_sizes[i]`` long along
    ``gather_dim``) are concatenated along ``gather_dim``. Any layout (batch- or sequence-first),
    any scatter/gather axes, uneven sizes on either side. One ``all_to_all_single`` on flat
    element ranges (so pieces of different shapes travel in one collective).

    Parity: reference sequence/layer.py:221-254 ``single_all_to_all`` and :111-218
    ``uneven_heads_all2all`` -- one routine here instead of per-layout permute tables."""
    p = dist.get_world_size(group)
    me = dist.get_rank(group)
    nd = x.dim()
    sd, gd = scatter_dim % nd, gather_dim % nd
    assert sd != gd and sum(send_sizes) == x.shape[sd] and len(send_sizes) == p == len(recv_sizes)
    send = x.movedim(sd, 0).contiguous()  # [T, rest...]: piece j is a contiguous row range
    rest = list(send.shape[1:])
    row = math.prod(rest)
    g_in_rest = gd if gd < sd else gd - 1  # gather axis within `rest`
    per_row_wo_g = row // rest[g_in_rest] if rest[g_in_rest] else 0
    # every rank cuts the scatter axis with the same partition, so each sends us send_sizes[me]
    # rows, each holding recv_sizes[i] elements along the gather axis
    recv_t = send_sizes[me]
    in_splits = [n * row for n in send_sizes]
    out_splits = [recv_t * per_row_wo_g * n for n in recv_sizes]
    out = torch.empty(sum(out_splits), dtype=x.dtype, device=x.device)
    ctx = torch.cuda.stream(stream) if stream is not None else _nullctx()
    with ctx:
        dist.all_to_all_single(out, send.reshape(-1), output_split_sizes=out_splits, input_split_sizes=in_splits,
                               group=group)
        pieces = []
        for i, flat in enumerate(out.split(out_splits)):
            shp = [recv_t] + rest
            shp[1 + g_in_rest] = recv_sizes[i]
            pieces.append(flat.view(shp))
        y = torch.cat(pieces, dim=1 + g_in_rest) if p > 1 else pieces[0]
        y = y.movedim(0, sd).contiguous()
    return y


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class _AllToAllDims(torch.autograd.Function):
    @staticmethod
    def forward(ctx, group, x, sd, gd, send_sizes, recv_sizes, stream):
        ctx.args = (group, sd, gd, send_sizes, recv_sizes, stream)
        return all_to_all_dims(x, sd, gd, send_sizes, recv_sizes, group, stream)

    @staticmethod
    def backward(ctx, g):
        group, sd, gd, send_sizes, recv_sizes, stream = ctx.args
        # the adjoint exchange: scatter back along the gathered axis, gather along the scattered one
        if stream is not None:
            stream.wait_stream(torch.cuda.current_stream(g.device))
        dx = all_to_all_dims(g, gd, sd, recv_sizes, send_sizes, group, stream)
        if stream is not None:
            torch.cuda.current_stream(g.device).wait_stream(stream)
            dx.record_stream(torch.cuda.current_stream(g.device))
        return None, dx, None, None, None, None, None


def _rotate_half(x):
    x1, x2 = x.chunk(2, dim=-1)
    return torch.cat((-x2, x1), dim=-1)


def _apply_rotary(t, cos, sin):
    rd = cos.shape[-1]
    head, tail = t[..., :rd], t[..., rd:]
    head = head * cos + _rotate_half(head) * sin
    return head if tail.shape[-1] == 0 else torch.cat((head, tail), dim=-1)


class DistributedAttention(nn.Module):
    """Ulysses attention around any local attention callable.

    ``forward(query, key, value, batch_dim_idx, rotary_pos_emb=None, *args, **kwargs)`` with inputs
    holding the local sequence chunk: sequence-first ``[s/p, b, h, d]`` for the defaults
    ``scatter_idx=2, gather_idx=0`` (``batch_dim_idx=1``), or batch-first ``[b, s/p, h, d]`` with
    ``gather_idx=1`` (``batch_dim_idx=0``). The local attention sees the full sequence and ``h/p``
    heads in the same layout; the output is returned in the input layout. Head counts that do not
    divide by the SP degree use the near-even uneven-heads exchange (:func:`shard_sizes`) with the kv
    head as the grain, so every rank keeps whole GQA groups.

    ``sp_stream``: q, k and v travel on that HIP stream, each exchange issued as soon as its input
    is ready, and the compute stream waits on an event only right before the local attention (and,
    in backward, the three gradient exchanges run there back to back) -- the permute/copy work of
    one tensor overlaps the transfer of the next.

    Parity: reference sequence/layer.py:331-440 (``DistributedAttention``; defaults :341-347,
    rotary after the exchange :425-428, overlap :392-426)."""

    def __init__(self, local_attention, sequence_process_group, scatter_idx=2, gather_idx=0, sp_stream=None):
        super().__init__()
        self.local_attn = local_attention
        self.spg = sequence_process_group
        self.scatter_idx, self.gather_idx = scatter_idx, gather_idx
        self.sp_stream = sp_stream
        self.sp_overlap_comm = sp_stream is not None

    def _exchange(self, t, fwd, head_sizes):
        p = dist.get_world_size(self.spg)
        if p == 1:
            return t
        stream = self.sp_stream if (self.sp_stream is not None and t.is_cuda) else None
        if stream is not None:
            stream.wait_stream(torch.cuda.current_stream(t.device))
        if fwd:  # scatter heads, gather sequence
            seq = [t.shape[self.gather_idx]] * p
            return _AllToAllDims.apply(self.spg, t, self.scatter_idx, self.gather_idx, head_sizes, seq, stream)
        seq = [t.shape[self.gather_idx] // p] * p  # scatter sequence, gather heads
        return _AllToAllDims.apply(self.spg, t, self.gather_idx, self.scatter_idx, seq, head_sizes, stream)

    def forward(self, query, key, value, batch_dim_idx=None, rotary_pos_emb=None, *args, **kwargs):
        if batch_dim_idx is None:
            batch_dim_idx = 0 if self.gather_idx == 1 else 1
        assert batch_dim_idx in (0, 1)
        p = dist.get_world_size(self.spg)
        hq, hkv = query.shape[self.scatter_idx], key.shape[self.scatter_idx]
        assert hq % hkv == 0, f"query heads ({hq}) must be a multiple of kv heads ({hkv})"
        # kv heads are the partition grain: rank r gets kv_sizes[r] kv heads and the q heads of
        # exactly those kv groups, so GQA stays intact on every rank even when p does not divide
        kv_sizes = shard_sizes(hkv, p)
        q_sizes = [n * (hq // hkv) for n in kv_sizes]
        q = self._exchange(query, True, q_sizes)
        k = self._exchange(key, True, kv_sizes)
        v = self._exchange(value, True, kv_sizes)
        if self.sp_stream is not None and q.is_cuda:
            torch.cuda.current_stream(q.device).wait_stream(self.sp_stream)
            for t in (q, k, v):
                t.record_stream(torch.cuda.current_stream(q.device))
        if rotary_pos_emb is not None:
            cos, sin = rotary_pos_emb[0], rotary_pos_emb[1]
            if batch_dim_idx == 1:  # reference layout: freqs arrive [b, s, 1, d] -> [s, b, 1, d]
                cos, sin = cos.permute(1, 0, 2, 3), sin.permute(1, 0, 2, 3)
            q, k = _apply_rotary(q, cos, sin), _apply_rotary(k, cos, sin)
        ctx = self.local_attn(q, k, v, *args, **kwargs)
        out = self._exchange(ctx, False, q_sizes)
        if self.sp_stream is not None and out.is_cuda:
            torch.cuda.current_stream(out.device).wait_stream(self.sp_stream)
            out.record_stream(torch.cuda.current_stream(out.device))
        return out


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
