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
with FPDT nothing is offloaded. Without load balancing, causal ring attention idles the first ranks
for the later steps (ranks hold contiguous chunks; a zig-zag chunk order would balance it).

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


class _RingAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, group, causal, scale):
        ring = _Ring(group)
        Hk = k.shape[2]
        kv = torch.cat([k, v], dim=2).contiguous()
        o_acc = lse_acc = None
        for step in range(ring.p):
            j = (ring.r - step) % ring.p
            pending = ring.start(kv) if step + 1 < ring.p else None
            if not causal or j <= ring.r:
                o, lse = _pair_fwd(q, kv[:, :, :Hk], kv[:, :, Hk:], causal and j == ring.r, scale)
                o_acc, lse_acc = _merge(o_acc, lse_acc, o, lse)
            if pending is not None:
                ring.finish(pending[1])
                kv = pending[0]
        out = o_acc.to(q.dtype)
        ctx.save_for_backward(q, k, v, out, lse_acc)
        ctx.group, ctx.causal, ctx.scale = group, causal, scale
        return out

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        ring = _Ring(ctx.group)
        Hk = k.shape[2]
        kv = torch.cat([k, v], dim=2).contiguous()
        dkv = torch.zeros(kv.shape, dtype=torch.float32, device=kv.device)
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        for step in range(ring.p):
            j = (ring.r - step) % ring.p
            pending = ring.start(kv) if step + 1 < ring.p else None
            if not ctx.causal or j <= ring.r:
                dqp, dkp, dvp = _pair_bwd(do, q, kv[:, :, :Hk], kv[:, :, Hk:], o, lse, ctx.causal and j == ring.r,
                                          ctx.scale)
                dq += dqp
                dkv[:, :, :Hk] += dkp
                dkv[:, :, Hk:] += dvp
            # the partial dK/dV of chunk j travel with it; after the p-th hop they are home
            dkv, reqs = ring.start(dkv)
            ring.finish(reqs)
            if pending is not None:
                ring.finish(pending[1])
                kv = pending[0]
        return dq.to(q.dtype), dkv[:, :, :Hk].to(k.dtype), dkv[:, :, Hk:].to(v.dtype), None, None, None


def ring_attention(q, k, v, group, causal=True, softmax_scale=None):
    """q [B, S/p, H, D], k/v [B, S/p, Hk, D]: this rank's contiguous sequence chunk (rank order =
    sequence order) -> [B, S/p, H, D] attention over the whole sequence."""
    scale = softmax_scale if softmax_scale is not None else q.shape[-1] ** -0.5
    if group is None or dist.get_world_size(group) == 1:
        from ..ops.attention import attention
        return attention(q, k, v, causal=causal, softmax_scale=scale)
    return _RingAttention.apply(q, k, v, group, causal, scale)


def ring_qkv_attention(qkv, nq, nkv, rope, group, position_ids=None, causal=True, softmax_scale=None):
    """Ring attention on a packed QKV chunk [B, S/p, nq + 2nkv, D] (the Llama layout) -> [B, S/p, nq, D]:
    RoPE at the chunk's global positions, then ``ring_attention`` on strided q/k/v views."""
    from ..ops.rope import apply_rope_qkv_
    B, Sl, _, D = qkv.shape
    if rope is not None:
        pos = position_ids
        if pos is None:
            r = dist.get_rank(group) if group is not None else 0
            pos = (torch.arange(Sl, device=qkv.device) + r * Sl).unsqueeze(0).expand(B, Sl)
        qkv = apply_rope_qkv_(qkv, rope, nq + nkv, pos)
    q, k, v = qkv[:, :, :nq], qkv[:, :, nq:nq + nkv], qkv[:, :, nq + nkv:]
    return ring_attention(q, k, v, group, causal=causal, softmax_scale=softmax_scale)
