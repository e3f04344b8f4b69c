"""Ring attention (context parallelism) over the sequence-parallel group.

SURVEY §2.6 lists ring attention / context parallelism as absent from the reference (its long
context goes through Ulysses all-to-all, FPDT chunking and tiling) and as an optional new feature
for the xGMI full mesh. This is that feature: every rank keeps its [B, S/p, H, D] chunk of the
queries and passes the packed [k | v] chunk around the ring with point-to-point sends to the next
rank (one xGMI link per hop, ``batch_isend_irecv`` issued BEFORE the local attention so the
transfer overlaps it). Each (query chunk, key chunk) pair runs the gfx950 flash kernel, which also
returns the log-sum-exp; partial outputs are merged with the LSE rule
``o = o_a e^(l_a - l) + o_b e^(l_b - l)``, ``l = logaddexp(l_a, l_b)``. Under a causal mask the pair
(i, j) is full for j < i, causal for j = i and skipped for j > i.

Backward runs the ring again: each pair's dQ/dK/dV come from the flash backward kernel fed the
GLOBAL output and LSE (so P and delta are the merged softmax's), dQ accumulates locally and the
dK/dV partials travel with their k/v chunk, arriving home after the p-th hop. Unlike Ulysses the
head count need not be divisible by p and no all-to-all of the activations is needed; compared
with FPDT nothing is offloaded.

Load balance: with contiguous chunks (``layout="contiguous"``) a causal mask gives rank i only i+1
non-empty pairs, so the last rank's work sets the step time. ``layout="zigzag"`` cuts the sequence
into 2p chunks and gives rank r chunks r and 2p-1-r (``zigzag_shard`` lays out the batch and the
position ids): every rank then computes the same number of (half-chunk) pairs at every step.

Shapes the flash kernel does not take (CPU / gloo tests, head dims other than 128, chunks not a
multiple of 128) run the same algorithm through an fp32 math path.
"""
import torch

from .. import comm as dist


def _hip_ok(q, k, v):
    from ..ops.attention import hip_supported
    return q.is_cuda and hip_supported(q, k, v)


def _math_pair_fwd(q, k, v, causal, scale):
    B, S, H, D = q.shape
    G = H // k.shape[2]
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(G, 1)
    vf = v.float().transpose(1, 2).repeat_interleave(G, 1)
    s = (qf @ kf.transpose(-1, -2)) * scale
    if causal:
        s = s.masked_fill(torch.ones(S, k.shape[1], dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    lse = torch.logsumexp(s, -1)
    o = torch.exp(s - lse.unsqueeze(-1)) @ vf
    return o.transpose(1, 2), lse


def _math_pair_bwd(do, q, k, v, o, lse, causal, scale):
    B, S, H, D = q.shape
    Hk = k.shape[2]
    G = H // Hk
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(G, 1)
    vf = v.float().transpose(1, 2).repeat_interleave(G, 1)
    dof, of = do.float().transpose(1, 2), o.float().transpose(1, 2)
    s = (qf @ kf.transpose(-1, -2)) * scale
    if causal:
        s = s.masked_fill(torch.ones(S, k.shape[1], dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    p = torch.exp(s - lse.unsqueeze(-1))
    dv = p.transpose(-1, -2) @ dof
    dp = dof @ vf.transpose(-1, -2)
    ds = p * (dp - (dof * of).sum(-1, keepdim=True))
    dq = (ds @ kf) * scale
    dk = (ds.transpose(-1, -2) @ qf) * scale

    def fold(t):  # [B, H, S, D] -> [B, S, Hk, D], summing the query heads of each kv head
        return t.view(B, Hk, G, -1, D).sum(2).transpose(1, 2)
    return dq.transpose(1, 2), fold(dk), fold(dv)


def _pair_fwd(q, k, v, causal, scale):
    """-> (o [B, S, H, D] fp32, lse [B, H, S] fp32) of one (query chunk, key chunk) pair."""
    if _hip_ok(q, k, v):
        o, lse = torch.ops.sxe.flash_attn_fwd(q, k, v, bool(causal), float(scale))
        return o.float(), lse
    return _math_pair_fwd(q, k, v, causal, scale)


def _pair_bwd(do, q, k, v, o, lse, causal, scale):
    if _hip_ok(q, k, v) and do.dtype == q.dtype and o.dtype == q.dtype:
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        torch.ops.sxe.flash_attn_bwd(do.contiguous(), q, k, v, o, lse.contiguous(), dq, dk, dv, bool(causal),
                                     float(scale))
        return dq.float(), dk.float(), dv.float()
    return _math_pair_bwd(do, q, k, v, o, lse, causal, scale)


class _Ring:
    def __init__(self, group):
        self.group = group
        self.p = dist.get_world_size(group)
        self.r = dist.get_rank(group)
        self.nxt = dist.get_global_rank(group, (self.r + 1) % self.p)
        self.prv = dist.get_global_rank(group, (self.r - 1) % self.p)

    def start(self, send):
        """Send ``send`` to the next rank, receive the previous rank's into a new buffer."""
        recv = torch.empty_like(send)
        reqs = dist.batch_isend_irecv([dist.P2POp(torch.distributed.isend, send, self.nxt, self.group),
                                       dist.P2POp(torch.distributed.irecv, recv, self.prv, self.group)])
        return recv, reqs

    @staticmethod
    def finish(reqs):
        for w in reqs:
            w.wait()


def _merge(o_acc, lse_acc, o, lse):
    if o_acc is None:
        return o, lse
    new = torch.logaddexp(lse_acc, lse)
    a = torch.exp(lse_acc - new).transpose(1, 2).unsqueeze(-1)
    b = torch.exp(lse - new).transpose(1, 2).unsqueeze(-1)
    return o_acc * a + o * b, new


def _halves(layout, r, p):
    """Global chunk ids of a rank's local sequence pieces (in local order)."""
    return (r,) if layout == "contiguous" else (r, 2 * p - 1 - r)


def _split(t, n):
    return t.chunk(n, dim=1) if n > 1 else (t,)


def _mode(iq, ik, causal):
    """(run, causal flag) of the pair (query piece iq, key piece ik) under the global causal mask."""
    if not causal:
        return True, False
    return ik <= iq, ik == iq


class _RingAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, group, causal, scale, layout):
        ring = _Ring(group)
        Hk = k.shape[2]
        mine = _halves(layout, ring.r, ring.p)
        n = len(mine)
        qs = _split(q, n)
        kv = torch.cat([k, v], dim=2).contiguous()
        acc = [(None, None)] * n
        for step in range(ring.p):
            j = (ring.r - step) % ring.p
            pending = ring.start(kv) if step + 1 < ring.p else None
            for a, (iq, qa) in enumerate(zip(mine, qs)):
                for ik, kva in zip(_halves(layout, j, ring.p), _split(kv, n)):
                    run, cflag = _mode(iq, ik, causal)
                    if run:
                        o, lse = _pair_fwd(qa, kva[:, :, :Hk], kva[:, :, Hk:], cflag, scale)
                        acc[a] = _merge(acc[a][0], acc[a][1], o, lse)
            if pending is not None:
                ring.finish(pending[1])
                kv = pending[0]
        out = torch.cat([o for o, _ in acc], 1).to(q.dtype)
        lse = torch.cat([l for _, l in acc], 2)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.group, ctx.causal, ctx.scale, ctx.layout = group, causal, scale, layout
        return out

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        ring = _Ring(ctx.group)
        Hk = k.shape[2]
        mine = _halves(ctx.layout, ring.r, ring.p)
        n = len(mine)
        qs, os_, dos = _split(q, n), _split(o, n), _split(do.contiguous(), n)
        lses = lse.chunk(n, dim=2) if n > 1 else (lse,)
        kv = torch.cat([k, v], dim=2).contiguous()
        dkv = torch.zeros(kv.shape, dtype=torch.float32, device=kv.device)
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        dqs = _split(dq, n)
        for step in range(ring.p):
            j = (ring.r - step) % ring.p
            pending = ring.start(kv) if step + 1 < ring.p else None
            for a, iq in enumerate(mine):
                for b, (ik, kvb) in enumerate(zip(_halves(ctx.layout, j, ring.p), _split(kv, n))):
                    run, cflag = _mode(iq, ik, ctx.causal)
                    if not run:
                        continue
                    dqp, dkp, dvp = _pair_bwd(dos[a], qs[a], kvb[:, :, :Hk], kvb[:, :, Hk:], os_[a],
                                              lses[a].contiguous(), cflag, ctx.scale)
                    dqs[a].add_(dqp)
                    dkb = _split(dkv, n)[b]
                    dkb[:, :, :Hk] += dkp
                    dkb[:, :, Hk:] += dvp
            # the partial dK/dV of chunk j travel with it; after the p-th hop they are home
            dkv, reqs = ring.start(dkv)
            ring.finish(reqs)
            if pending is not None:
                ring.finish(pending[1])
                kv = pending[0]
        return dq.to(q.dtype), dkv[:, :, :Hk].to(k.dtype), dkv[:, :, Hk:].to(v.dtype), None, None, None, None


def zigzag_indices(seq_len, rank, p, device=None):
    """Token positions of ``rank``'s zig-zag shard: chunks rank and 2p-1-rank of 2p equal chunks."""
    assert seq_len % (2 * p) == 0, f"sequence length {seq_len} must be divisible by 2 * {p}"
    c = seq_len // (2 * p)
    idx = torch.arange(seq_len, device=device).view(2 * p, c)
    return torch.cat([idx[rank], idx[2 * p - 1 - rank]])


def zigzag_shard(input_ids, rank, p, labels=None, ignore_index=-100):
    """``shard_batch_for_sp`` for the zig-zag layout: input ids, next-token labels and position ids
    of this rank's two chunks."""
    B, S = input_ids.shape
    labels = input_ids if labels is None else labels
    shifted = torch.cat([labels[:, 1:], torch.full_like(labels[:, :1], ignore_index)], dim=1)
    idx = zigzag_indices(S, rank, p, input_ids.device)
    return {"input_ids": input_ids[:, idx].contiguous(), "labels": shifted[:, idx].contiguous(),
            "position_ids": idx.unsqueeze(0).expand(B, -1).contiguous(), "shift_labels": False}


def ring_attention(q, k, v, group, causal=True, softmax_scale=None, layout="contiguous"):
    """q [B, S/p, H, D], k/v [B, S/p, Hk, D]: this rank's share of the sequence -- its contiguous
    chunk (rank order = sequence order) or, with ``layout="zigzag"``, chunks r and 2p-1-r
    concatenated -- -> [B, S/p, H, D] attention over the whole sequence."""
    assert layout in ("contiguous", "zigzag"), layout
    scale = softmax_scale if softmax_scale is not None else q.shape[-1] ** -0.5
    if group is None or dist.get_world_size(group) == 1:
        from ..ops.attention import attention
        return attention(q, k, v, causal=causal, softmax_scale=scale)
    return _RingAttention.apply(q, k, v, group, causal, scale, layout)


def ring_qkv_attention(qkv, nq, nkv, rope, group, position_ids=None, causal=True, softmax_scale=None,
                       layout="contiguous"):
    """Ring attention on a packed QKV chunk [B, S/p, nq + 2nkv, D] (the Llama layout) -> [B, S/p, nq, D]:
    RoPE at the chunk's global positions, then ``ring_attention`` on strided q/k/v views."""
    from ..ops.rope import apply_rope_qkv_
    B, Sl, _, D = qkv.shape
    if rope is not None:
        pos = position_ids
        if pos is None:
            r = dist.get_rank(group) if group is not None else 0
            if layout == "zigzag" and group is not None:
                p = dist.get_world_size(group)
                pos = zigzag_indices(Sl * p, r, p, qkv.device).unsqueeze(0).expand(B, Sl)
            else:
                pos = (torch.arange(Sl, device=qkv.device) + r * Sl).unsqueeze(0).expand(B, Sl)
        qkv = apply_rope_qkv_(qkv, rope, nq + nkv, pos)
    q, k, v = qkv[:, :, :nq], qkv[:, :, nq:nq + nkv], qkv[:, :, nq + nkv:]
    return ring_attention(q, k, v, group, causal=causal, softmax_scale=softmax_scale, layout=layout)
