"""FPDT -- Fully Pipelined Distributed Transformer: chunked Ulysses attention for very long sequences.

Parity: reference deepspeed/sequence/fpdt_layer.py -- ``update_out_and_lse`` :40-76 (online-softmax
merge of per-KV-chunk partial outputs through their log-sum-exp), ``FPDT_InputConstruct`` :79-131
(load-balanced chunk -> rank assignment), ``_FPDTGPUAttentionImpl_`` :134-460 (per-chunk QKV
all-to-all, attention of query chunk i against KV chunks j <= i, chunk-pair backward re-using the
merged output + LSE), ``SequenceChunk`` :462-508 and ``_FPDTGPUOffloadingAttentionImpl_`` :510-970
(host offload of the saved chunks), ``FPDT_Attention`` :971, ``FPDT_FFN`` :1056, ``FPDT_LogitsLoss``
:1137.

MI355X-first design:
* layout is batch-first [B, S, H, D] (the QKV projection output), the per-chunk exchange moves the
  packed q|k|v heads of a chunk in ONE all_to_all_single (the reference issues three per chunk),
  and RoPE is applied before the exchange with the chunk's global positions (one HIP launch);
* every (query chunk, KV chunk) pair runs this repo's gfx950 flash-attention kernels
  (csrc/kernels/flash_attn.hip): the forward returns (o, lse), the backward of a pair is the flash
  backward fed with the MERGED output and LSE of the query chunk, which makes the per-pair
  gradients exact (delta = rowsum(dO * O_final), P = exp(S - LSE_final));
* offloaded chunks live in pinned host buffers, copied on a dedicated HIP stream with events, so the
  D2H of chunk c overlaps the attention of chunk c+1 and the H2D of KV chunk j+1 overlaps the
  backward of chunk j (288 GB HBM makes offload optional up to ~1M tokens per GPU for 8B).
"""
import math

import torch

from .. import comm as dist
from ..accelerator import get_accelerator
from ..ops.attention import hip_supported, reference_attention


# ------------------------------------------------------------------------------------ LSE merging
def _update_out_and_lse(out, lse, block_out, block_lse):
    """out [B, S, H, D] fp32, lse [B, H, S] fp32; returns the merged pair (numerically stable)."""
    new_lse = torch.logaddexp(lse, block_lse)
    a = torch.exp(lse - new_lse).transpose(1, 2).unsqueeze(-1)
    b = torch.exp(block_lse - new_lse).transpose(1, 2).unsqueeze(-1)
    return a * out + b * block_out.float(), new_lse


def update_out_and_lse(out, lse, block_out, block_lse, slice_=None):
    """Reference-compatible signature (fpdt_layer.py:58): ``out=None`` starts the accumulation."""
    if out is None:
        if slice_ is not None:
            raise RuntimeError("first update_out_and_lse should not pass slice_ args")
        return block_out.float(), block_lse.float()
    if slice_ is not None:
        o, l_ = _update_out_and_lse(out[slice_], lse[slice_], block_out, block_lse)
        out[slice_], lse[slice_] = o, l_
        return out, lse
    return _update_out_and_lse(out, lse, block_out, block_lse)


# -------------------------------------------------------------------------- chunk-pair attention
def _use_flash(q, k):
    return q.is_cuda and hip_supported(q, k, k) and q.shape[1] == k.shape[1]


def _pair_fwd(q, k, v, causal, scale):
    if _use_flash(q, k):
        return torch.ops.sxe.flash_attn_fwd(q, k, v, bool(causal), float(scale))
    return reference_attention(q, k, v, causal, scale, return_lse=True)


def _pair_bwd_reference(do, q, k, v, o, lse, causal, scale):
    """fp32 eager backward of one chunk pair given the merged (o, lse) of the query chunk."""
    G = q.shape[2] // k.shape[2]
    qt, kt, vt = (t.transpose(1, 2).float() for t in (q, k, v))
    kt, vt = kt.repeat_interleave(G, 1), vt.repeat_interleave(G, 1)
    dot, ot = do.transpose(1, 2).float(), o.transpose(1, 2).float()
    s = torch.matmul(qt, kt.transpose(-1, -2)) * scale
    p = torch.exp(s - lse.unsqueeze(-1))
    if causal:
        S, T = s.shape[-2], s.shape[-1]
        p = p * torch.ones(S, T, dtype=torch.bool, device=s.device).tril(T - S)
    dv = torch.matmul(p.transpose(-1, -2), dot)
    dp = torch.matmul(dot, vt.transpose(-1, -2))
    delta = (dot * ot).sum(-1, keepdim=True)
    ds = p * (dp - delta)
    dq = torch.matmul(ds, kt) * scale
    dk = torch.matmul(ds.transpose(-1, -2), qt) * scale
    B, Hk = k.shape[0], k.shape[2]
    dk = dk.view(B, Hk, G, *dk.shape[2:]).sum(2)
    dv = dv.view(B, Hk, G, *dv.shape[2:]).sum(2)
    return dq.transpose(1, 2), dk.transpose(1, 2), dv.transpose(1, 2)


def _pair_bwd(do, q, k, v, o, lse, causal, scale):
    if _use_flash(q, k):
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        torch.ops.sxe.flash_attn_bwd(do.contiguous(), q, k, v, o, lse, dq, dk, dv, bool(causal), float(scale))
        return dq, dk, dv
    return _pair_bwd_reference(do, q, k, v, o, lse, causal, scale)


# ------------------------------------------------------------------------------ host offloading
class SequenceChunk:
    """A saved activation chunk that can live in pinned host memory between forward and backward
    (reference fpdt_layer.py:462). Copies run on one side stream; ``get()`` waits for them."""

    _stream = None

    def __init__(self, t, offload=False):
        self.shape, self.dtype, self.device = t.shape, t.dtype, t.device
        self.gpu, self.cpu, self.event = t, None, None
        if offload and t.is_cuda:
            st = SequenceChunk.stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                self.cpu = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                self.cpu.copy_(t, non_blocking=True)
                self.event = torch.cuda.Event()
                self.event.record(st)
            t.record_stream(st)
            self.gpu = None

    @classmethod
    def stream(cls):
        if cls._stream is None:
            cls._stream = get_accelerator().named_stream("fpdt_offload")
        return cls._stream

    def prefetch(self):
        if self.gpu is None and self.cpu is not None:
            st = SequenceChunk.stream()
            with torch.cuda.stream(st):
                st.wait_event(self.event)
                self.gpu = torch.empty(self.shape, dtype=self.dtype, device=self.device)
                self.gpu.copy_(self.cpu, non_blocking=True)
                self.event = torch.cuda.Event()
                self.event.record(st)
        return self

    def get(self):
        self.prefetch()
        if self.event is not None and self.gpu is not None and self.gpu.is_cuda:
            torch.cuda.current_stream().wait_event(self.event)
            self.gpu.record_stream(torch.cuda.current_stream())
        return self.gpu

    def offload(self):
        if self.cpu is not None:
            self.gpu = None


# ------------------------------------------------------------------------- packed chunk exchange
def _pack(qkv, nq, nkv, p):
    from .layer import _pack_heads
    return _pack_heads(qkv, nq, nkv, p)


def _qkv_to_heads(qkv, nq, nkv, group):
    """local chunk [B, L, nq+2nkv, D] -> group chunk [B, p*L, (nq+2nkv)/p, D] (one a2a)."""
    p = dist.get_world_size(group) if group is not None else 1
    if p == 1:
        return qkv
    send = _pack(qkv, nq, nkv, p)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    P, B, L, Hp, D = recv.shape
    return recv.permute(1, 0, 2, 3, 4).reshape(B, P * L, Hp, D)


def _heads_to_qkv(g, nq, nkv, group):
    """inverse of _qkv_to_heads for gradients: [B, p*L, Hp, D] -> [B, L, nq+2nkv, D]."""
    p = dist.get_world_size(group) if group is not None else 1
    if p == 1:
        return g
    from .layer import _unpack_heads
    B, S, Hp, D = g.shape
    send = g.reshape(B, p, S // p, Hp, D).permute(1, 0, 2, 3, 4).contiguous()
    back = torch.empty_like(send)
    dist.all_to_all_single(back, send, group=group)
    return _unpack_heads(back, nq, nkv, p)


def _seq_to_head(x, group):
    from .layer import seq_to_head
    return seq_to_head(x, group) if group is not None else x


def _head_to_seq(x, group):
    from .layer import head_to_seq
    return head_to_seq(x, group) if group is not None else x


def _rope_(x, rope, n_rot, positions, inverse=False):
    """In-place RoPE on the first n_rot heads of x [B, L, H, D] at absolute positions [B*L]."""
    if rope is None:
        return x
    if x.is_cuda:
        torch.ops.sxe.rope_(x[:, :, :n_rot], rope.cos, rope.sin, positions, x.shape[1], 0, bool(inverse))
        return x
    from ..ops.rope import _ref_rope
    B, L, _, D = x.shape
    sin = -rope.sin if inverse else rope.sin
    r = _ref_rope(x[:, :, :n_rot].reshape(B * L, n_rot, D).float(), rope.cos, sin, positions)
    x[:, :, :n_rot] = r.view(B, L, n_rot, D).to(x.dtype)
    return x


# ------------------------------------------------------------------------------ the attention fn
class _FPDTAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, nq, nkv, rope, group, num_chunks, causal, scale, offload):
        B, S_loc, Ht, D = qkv.shape
        p = dist.get_world_size(group) if group is not None else 1
        r = dist.get_rank(group) if group is not None else 0
        assert S_loc % num_chunks == 0, "FPDT: local sequence must split into equal chunks"
        L = S_loc // num_chunks
        nqp, nkvp = nq // p, nkv // p
        qs, ks, vs, os_, lses = [], [], [], [], []
        outs = []
        for c in range(num_chunks):
            x = qkv[:, c * L:(c + 1) * L].clone(memory_format=torch.contiguous_format)
            # local chunk c of rank r is global chunk c*p + r (FPDT_InputConstruct layout)
            pos = (torch.arange(L, device=x.device) + (c * p + r) * L).repeat(B)
            _rope_(x, rope, nq + nkv, pos)
            g = _qkv_to_heads(x, nq, nkv, group)  # [B, p*L, nqp + 2 nkvp, D]
            q, k, v = g[:, :, :nqp], g[:, :, nqp:nqp + nkvp], g[:, :, nqp + nkvp:]
            out, lse = None, None
            for j in range(c + 1):
                kj = ks[j].get() if j < c else k
                vj = vs[j].get() if j < c else v
                bo, bl = _pair_fwd(q, kj, vj, causal and j == c, scale)
                out, lse = update_out_and_lse(out, lse, bo, bl)
                if j < c:
                    ks[j].offload()
                    vs[j].offload()
            o = out.to(qkv.dtype)
            ks.append(SequenceChunk(k, offload))
            vs.append(SequenceChunk(v, offload))
            qs.append(SequenceChunk(q, offload))
            os_.append(SequenceChunk(o, offload))
            lses.append(lse)
            outs.append(_head_to_seq(o, group))
        ctx.saved = (qs, ks, vs, os_, lses)
        ctx.meta = (nq, nkv, rope, group, num_chunks, causal, scale, B, S_loc, Ht, D, L, p, r)
        return torch.cat(outs, dim=1)

    @staticmethod
    def backward(ctx, dout):
        qs, ks, vs, os_, lses = ctx.saved
        nq, nkv, rope, group, C, causal, scale, B, S_loc, Ht, D, L, p, r = ctx.meta
        nqp, nkvp = nq // p, nkv // p
        dos = [_seq_to_head(dout[:, c * L:(c + 1) * L].contiguous(), group) for c in range(C)]
        dq = [None] * C
        dqkv = torch.empty(B, S_loc, Ht, D, dtype=dout.dtype, device=dout.device)
        for j in range(C):
            kj, vj = ks[j].get(), vs[j].get()
            if j + 1 < C:
                ks[j + 1].prefetch()
                vs[j + 1].prefetch()
            dk = torch.zeros(kj.shape, dtype=torch.float32, device=kj.device)
            dv = torch.zeros(vj.shape, dtype=torch.float32, device=vj.device)
            for i in range(j, C):
                qi, oi = qs[i].get(), os_[i].get()
                gq, gk, gv = _pair_bwd(dos[i], qi, kj, vj, oi, lses[i], causal and i == j, scale)
                dq[i] = gq.float() if dq[i] is None else dq[i].add_(gq.float())
                dk.add_(gk.float())
                dv.add_(gv.float())
            # dq_j is complete once every KV chunk <= j has been visited
            g = torch.cat([dq[j], dk, dv], dim=2).to(dout.dtype)
            dq[j] = None
            x = _heads_to_qkv(g, nq, nkv, group)
            pos = (torch.arange(L, device=x.device) + (j * p + r) * L).repeat(B)
            _rope_(x, rope, nq + nkv, pos, inverse=True)
            dqkv[:, j * L:(j + 1) * L] = x
            ks[j].offload()
            vs[j].offload()
        ctx.saved = None
        return dqkv, None, None, None, None, None, None, None, None


def fpdt_attention(qkv, nq, nkv, rope=None, group=None, num_chunks=2, causal=True, softmax_scale=None,
                   offload=False):
    """Chunked (FPDT) sequence-parallel attention on this rank's packed QKV [B, S/p, nq+2nkv, D]
    (its tokens laid out by ``FPDT_InputConstruct``) -> [B, S/p, nq, D]. ``group=None`` runs the
    chunked single-GPU variant (long-context memory saving without SP)."""
    D = qkv.shape[-1]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    p = dist.get_world_size(group) if group is not None else 1
    if p > 1 and nkv < p:
        from .layer import _replicate_kv
        qkv, nkv = _replicate_kv(qkv, nq, nkv, p)
    assert nq % p == 0 and nkv % p == 0, "FPDT: heads must divide the SP degree"
    assert causal, "FPDT is causal (reference asserts attention_mask is None and uses causal chunks)"
    return _FPDTAttention.apply(qkv, nq, nkv, rope, group, int(num_chunks), causal, float(scale), bool(offload))


class FPDT_InputConstruct:
    """Load-balanced token layout (reference fpdt_layer.py:79-131): the global sequence is cut into
    ``sp * num_chunk_per_gpu`` chunks and rank r holds chunks r, r+sp, r+2sp, ... so that the causal
    work of every rank is the same. ``generate()`` returns this rank's (tokens, labels, loss_mask,
    attention_mask, position_ids)."""

    def __init__(self, tokens, labels, loss_mask, attention_mask, position_ids, chunk_size, sp_size, sp_rank):
        B, S = tokens.shape
        assert S % sp_size == 0 and S % chunk_size == 0
        self.num_chunk_per_gpu = S // chunk_size
        self.local_seq_len = S // sp_size
        assert self.local_seq_len % self.num_chunk_per_gpu == 0
        self.chunk_size = self.local_seq_len // self.num_chunk_per_gpu
        self.tokens, self.labels, self.loss_mask = tokens, labels, loss_mask
        self.attention_mask, self.position_ids = attention_mask, position_ids
        self.sp_size, self.sp_rank, self.global_seq_len = sp_size, sp_rank, S

    def indices(self):
        n, L, p, r = self.num_chunk_per_gpu, self.chunk_size, self.sp_size, self.sp_rank
        chunks = [c * p + r for c in range(n)]
        return torch.cat([torch.arange(g * L, (g + 1) * L) for g in chunks])

    def generate(self):
        idx = self.indices().to(self.tokens.device)
        sel = (lambda t: t[:, idx] if t is not None else None)
        return sel(self.tokens), sel(self.labels), sel(self.loss_mask), self.attention_mask, sel(self.position_ids)


class FPDT_Attention(torch.nn.Module):
    """Module form (reference fpdt_layer.py:971): QKV projection -> chunked SP attention -> output
    projection, for a Llama-style GQA block. ``chunk_size`` is the GLOBAL chunk length."""

    def __init__(self, qkv_proj, o_proj, nq, nkv, head_dim, sequence_process_group=None, chunk_size=65536,
                 enable_offloading=False, rope=None):
        super().__init__()
        self.qkv_proj, self.o_proj = qkv_proj, o_proj
        self.nq, self.nkv, self.d = nq, nkv, head_dim
        self.spg, self.chunk_size, self.offload, self.rope = sequence_process_group, chunk_size, enable_offloading, rope

    def forward(self, x):
        B, S_loc, _ = x.shape
        p = dist.get_world_size(self.spg) if self.spg is not None else 1
        n = max(1, S_loc * p // self.chunk_size)
        qkv = self.qkv_proj(x).view(B, S_loc, self.nq + 2 * self.nkv, self.d)
        o = fpdt_attention(qkv, self.nq, self.nkv, self.rope, self.spg, n, offload=self.offload)
        return self.o_proj(o.reshape(B, S_loc, self.nq * self.d))


# ------------------------------------------------------------------------------ chunked FFN / loss
def _gelu(x):
    return x * 0.5 * (1.0 + torch.tanh(0.79788456 * x * (1 + 0.044715 * x * x)))


class FPDT_FFN(torch.autograd.Function):
    """Chunked bias-GELU MLP that recomputes each chunk's intermediate in backward
    (reference fpdt_layer.py:1056-1134): peak activation memory is one chunk of [*, ffn]."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, add_bias, chunk_size):
        n = x.shape[0] // chunk_size
        assert n * chunk_size == x.shape[0]
        out = torch.empty(x.shape[:-1] + (w2.shape[0],), dtype=x.dtype, device=x.device)
        with torch.no_grad():
            for i in range(n):
                s = slice(i * chunk_size, (i + 1) * chunk_size)
                h = _gelu(torch.matmul(x[s], w1.t()) + b1)
                out[s] = torch.matmul(h, w2.t()) + (b2 if add_bias else 0)
        ctx.save_for_backward(x, w1, b1, w2, b2)
        ctx.n, ctx.cs, ctx.add_bias = n, chunk_size, add_bias
        return out, (None if add_bias else b2)

    @staticmethod
    def backward(ctx, g, gb):
        x, w1, b1, w2, b2 = ctx.saved_tensors
        gw1, gb1 = torch.zeros_like(w1, dtype=torch.float32), torch.zeros_like(b1, dtype=torch.float32)
        gw2, gb2 = torch.zeros_like(w2, dtype=torch.float32), torch.zeros_like(b2, dtype=torch.float32)
        dx = torch.empty_like(x)
        for i in range(ctx.n):
            s = slice(i * ctx.cs, (i + 1) * ctx.cs)
            xi = x[s]
            with torch.enable_grad():
                a = (torch.matmul(xi, w1.t()) + b1).detach().requires_grad_(True)
                h = _gelu(a)
            gi = g[s]
            gw2.add_(torch.matmul(gi.reshape(-1, gi.shape[-1]).t().float(), h.detach().reshape(-1, h.shape[-1]).float()))
            gh = torch.matmul(gi, w2)
            (ga,) = torch.autograd.grad(h, a, gh)
            gw1.add_(torch.matmul(ga.reshape(-1, ga.shape[-1]).t().float(), xi.reshape(-1, xi.shape[-1]).float()))
            gb1.add_(ga.reshape(-1, ga.shape[-1]).float().sum(0))
            if ctx.add_bias:
                gb2.add_(gi.reshape(-1, gi.shape[-1]).float().sum(0))
            dx[s] = torch.matmul(ga, w1)
        if gb is not None and not ctx.add_bias:
            gb2.add_(gb.float())
        return dx, gw1.to(w1.dtype), gb1.to(b1.dtype), gw2.to(w2.dtype), gb2.to(b2.dtype), None, None


class FPDT_LogitsLoss(torch.autograd.Function):
    """Chunked LM head + per-token cross entropy on this rank's tokens, then the per-token losses of
    the SP group are all-gathered (reference fpdt_layer.py:1137-1225). h: [B, S_loc, H] batch-first;
    returns [B, S_loc * sp] fp32 losses in the group's concatenated rank order."""

    @staticmethod
    def forward(ctx, h, labels, weight, spg, num_chunk):
        B, S, H = h.shape
        cs = S // num_chunk
        assert cs * num_chunk == S
        loss = torch.empty(B, S, dtype=torch.float32, device=h.device)
        with torch.no_grad():
            for i in range(num_chunk):
                s = slice(i * cs, (i + 1) * cs)
                logits = torch.matmul(h[:, s], weight.t()).float()
                loss[:, s] = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]),
                                                               labels[:, s].reshape(-1), reduction="none").view(B, cs)
        ctx.save_for_backward(h, labels, weight)
        ctx.spg, ctx.n = spg, num_chunk
        p = dist.get_world_size(spg) if spg is not None else 1
        if p == 1:
            return loss
        parts = torch.empty(p, B, S, dtype=loss.dtype, device=loss.device)
        dist.all_gather_into_tensor(parts, loss.contiguous(), group=spg)
        return parts.permute(1, 0, 2).reshape(B, p * S)

    @staticmethod
    def backward(ctx, g):
        h, labels, weight = ctx.saved_tensors
        B, S, H = h.shape
        p = dist.get_world_size(ctx.spg) if ctx.spg is not None else 1
        r = dist.get_rank(ctx.spg) if ctx.spg is not None else 0
        g = g.reshape(B, p, S)[:, r] if p > 1 else g
        cs = S // ctx.n
        dh = torch.empty_like(h)
        dw = torch.zeros_like(weight, dtype=torch.float32)
        for i in range(ctx.n):
            s = slice(i * cs, (i + 1) * cs)
            logits = torch.matmul(h[:, s], weight.t()).float()
            prob = torch.softmax(logits, dim=-1)
            prob.scatter_add_(-1, labels[:, s].unsqueeze(-1), -torch.ones_like(prob[..., :1]))
            prob.mul_(g[:, s].unsqueeze(-1))
            gl = prob.to(h.dtype)
            dh[:, s] = torch.matmul(gl, weight)
            dw.add_(torch.matmul(gl.reshape(-1, gl.shape[-1]).t().float(), h[:, s].reshape(-1, H).float()))
        return dh, None, dw.to(weight.dtype), None, None
