"""Paged-KV attention ops for the ragged inference engine (HIP kernels in csrc/kernels/paged_attn.hip).

Cache layout per layer: ``[num_blocks, 2, n_kv_heads, block_size, head_dim]`` (bf16 on GPU).
``kv_cache_append`` scatters the k/v rows of the new tokens into their slots
(``slot = block_id * block_size + offset``); ``paged_attention`` runs causal attention of the new
tokens of each sequence over all of its cached keys. Both have PyTorch reference implementations
(CPU processes / numerics oracles).
"""
import math
import os

import torch

from . import native


def rope_kv_cache_append(qkv, rope, positions, cache, slots, nq, nkv):
    """RoPE on the q and k heads of ``qkv`` [T, nq + 2 nkv, D] (in place, absolute ``positions``)
    and the rotated k + v appended to the paged ``cache`` -- one HIP launch
    (paged_attn.hip ``rope_kv_append_kernel``) instead of rope_ + kv_cache_append."""
    from .rope import apply_rope_tokens_
    if (native.use_hip(qkv) and qkv.dtype == torch.bfloat16 and qkv.shape[-1] in (64, 128, 256)
            and qkv.is_contiguous() and rope.cos.shape[-1] * 2 == qkv.shape[-1]):
        torch.ops.sxe.rope_kv_cache_append(qkv, rope.cos, rope.sin, positions.reshape(-1).contiguous().long(), cache,
                                           slots, int(nq), int(nkv))
        return qkv
    apply_rope_tokens_(qkv, rope, nq + nkv, positions)
    kv_cache_append(qkv, cache, slots, nq, nkv)
    return qkv


def kv_cache_append(qkv, cache, slots, nq, nkv):
    """qkv: [T, nq + 2 nkv, D]; cache: [blocks, 2, nkv, bs, D]; slots: int64 [T] (-1 = skip)."""
    if native.use_hip(qkv) and qkv.shape[-1] in (64, 128) and qkv.is_contiguous():
        torch.ops.sxe.kv_cache_append(qkv, cache, slots, int(nq), int(nkv))
        return
    bs = cache.shape[3]
    ok = slots >= 0
    if not bool(ok.any()):
        return
    s = slots[ok]
    blk, off = s // bs, s % bs
    k = qkv[ok, nq:nq + nkv]
    v = qkv[ok, nq + nkv:nq + 2 * nkv]
    cache[blk, 0, :, off] = k.to(cache.dtype)
    cache[blk, 1, :, off] = v.to(cache.dtype)


def _gather_kv(cache, block_row, kv_len):
    bs = cache.shape[3]
    nb = (kv_len + bs - 1) // bs
    blocks = block_row[:nb].long()
    kv = cache[blocks]  # [nb, 2, nkv, bs, D]
    k = kv[:, 0].permute(1, 0, 2, 3).reshape(kv.shape[2], nb * bs, -1)[:, :kv_len]
    v = kv[:, 1].permute(1, 0, 2, 3).reshape(kv.shape[2], nb * bs, -1)[:, :kv_len]
    return k, v  # [nkv, kv_len, D]


def paged_attention_reference(q, cache, block_table, q_start, q_len, kv_len, scale, window=None):
    T, nq, D = q.shape
    nkv = cache.shape[2]
    G = nq // nkv
    out = torch.zeros(T, nq, D, dtype=q.dtype, device=q.device)
    for s in range(block_table.shape[0]):
        qs, ql, kl = int(q_start[s]), int(q_len[s]), int(kv_len[s])
        if ql == 0:
            continue
        k, v = _gather_kv(cache, block_table[s], kl)
        k = k.float().repeat_interleave(G, dim=0)
        v = v.float().repeat_interleave(G, dim=0)
        qq = q[qs:qs + ql].float().transpose(0, 1)  # [nq, ql, D]
        sc = torch.matmul(qq, k.transpose(1, 2)) * scale  # [nq, ql, kl]
        pos = torch.arange(kl - ql, kl, device=q.device)[:, None]
        keys = torch.arange(kl, device=q.device)[None, :]
        mask = keys > pos
        if window:  # sliding-window attention (Mistral / Qwen2): only the last `window` keys
            mask = mask | (keys <= pos - window)
        sc = sc.masked_fill(mask, float("-inf"))
        o = torch.matmul(torch.softmax(sc, dim=-1), v)  # [nq, ql, D]
        out[qs:qs + ql] = o.transpose(0, 1).to(q.dtype)
    return out


# keys per split floor (see choose_splits): 256 = four 64-key wave chunks per split. Llama-3-8B decode,
# HIP graphs, fused merge: batch 1 ctx 1024 3.571 / 3.604 / 3.700 ms per token at 256 / 128 / 64,
# ctx 4096 3.745 / 3.927 / 3.926; batch 8 and 32 within 1 % (profiles/r06/decode_split_floor_ab.log)
PA_MIN_KEYS = int(os.environ.get("SXE_PA_MIN_KEYS", 256))


PA_TARGET_WGS = int(os.environ.get("SXE_PA_TARGET_WGS", 512))


def choose_splits(num_seqs, nkv, max_kv_len, target_wgs=None):
    """KV splits so (seqs x kv heads x splits) fills the 256 CUs, never below PA_MIN_KEYS keys per
    split: at batch 1 the kernel is a latency chain (block table -> K/V loads -> MFMA -> merge), so
    more, shorter splits shorten it; at large batch one split per (seq, kv head) streams best."""
    target_wgs = PA_TARGET_WGS if target_wgs is None else target_wgs
    base = max(1, num_seqs * nkv)
    want = max(1, math.ceil(target_wgs / base))
    return max(1, min(want, math.ceil(max(max_kv_len, 1) / PA_MIN_KEYS)))


def paged_attention_parts(q, cache, block_table, q_start, q_len, kv_len, scale, max_kv_len, splits=None):
    """``paged_attention`` without the split-merge launch (HIP only): returns ``(out, None)`` when the
    kernel ran one split per (sequence, kv head), else ``(None, (part_o, part_ml))`` -- fp32
    partials [splits, T, nq, D] / [splits, T, nq, 2] for a consumer that merges them in its own
    prologue (``ops.linear.fused_merge_linear``: the o_proj skinny GEMM)."""
    if splits is None:
        splits = choose_splits(block_table.shape[0], cache.shape[2], max_kv_len)
    out, po, pml = torch.ops.sxe.paged_attention_parts(q, cache, block_table, q_start, q_len, kv_len, float(scale),
                                                       int(max_kv_len), int(splits), 0)
    return (out, None) if po.numel() == 0 else (None, (po, pml))


def merge_attention_parts(part_o, part_ml, dtype):
    """Flash-decoding merge of ``paged_attention_parts``' KV-split partials (the math of
    paged_attn.hip's merge kernel / skinny_gemm.hip PRO_MERGE): sum_s 2^(M_s - M) o_s /
    sum_s 2^(M_s - M) L_s over the splits, M the max of the split maxima (log2 domain).
    part_o [splits, T, nq, D], part_ml [splits, T, nq, 2] fp32 -> [T, nq, D] in ``dtype``."""
    m, l = part_ml[..., 0], part_ml[..., 1]
    mx = m.amax(0)
    f = torch.where(torch.isinf(m), torch.zeros_like(m), torch.exp2(m - torch.where(torch.isinf(mx), 0, mx)))
    den = (f * l).sum(0)
    num = (f.unsqueeze(-1) * part_o).sum(0)
    return torch.where(den.unsqueeze(-1) > 0, num / den.clamp_min(1e-30).unsqueeze(-1), 0.).to(dtype)


# SXE_PA_LAST_MERGE=1: with several KV splits the last split workgroup of each (sequence, kv head)
# merges the partials inside the attention launch (paged_attn.hip, arrival counters) instead of a
# second merge launch. Off: its device-scope fences write back / invalidate the L2 the K/V stream
# lives in -- Llama-3-8B ctx 1024 decode 4.50 vs 3.73 ms/token at batch 1, 6.60 vs 4.91 at batch 8
# (profiles/r06/decode_split_merge_ab.log)
PA_LAST_MERGE = os.environ.get("SXE_PA_LAST_MERGE", "0") == "1"
_COUNTERS = {}


def _split_counters(device, n):
    """Zeroed int32 split-arrival counters (self-resetting in the kernel), one buffer per device,
    grown outside any graph capture in the normal flow (the decode engine runs eagerly first)."""
    c = _COUNTERS.get(device)
    if c is None or c.numel() < n:
        c = _COUNTERS[device] = torch.zeros(max(n, 4096), dtype=torch.int32, device=device)
    return c


def paged_attention(q, cache, block_table, q_start, q_len, kv_len, scale, max_kv_len, splits=None, window=None):
    """q: [T, nq, D] (head stride D); metadata int32 [S]; returns [T, nq, D]. ``window``: sliding
    window length (keys older than ``window`` positions are masked, Mistral / Qwen2). The HIP kernel
    covers head dims 64 / 128 / 256, with or without a window (the window also skips the key chunks
    it masks entirely)."""
    if window is not None and max_kv_len <= window:
        window = None
    if native.use_hip(q) and q.shape[-1] in (64, 128, 256):
        if splits is None:
            splits = choose_splits(block_table.shape[0], cache.shape[2], max_kv_len)
        S = block_table.shape[0]
        cnt = (_split_counters(q.device, S * cache.shape[2])
               if PA_LAST_MERGE and splits > 1 and q.shape[0] <= 4 * S else None)
        return torch.ops.sxe.paged_attention(q, cache, block_table, q_start, q_len, kv_len, float(scale),
                                             int(max_kv_len), int(splits), int(window or 0), cnt)
    if q.is_cuda:
        from ..utils.logging import warning_once
        warning_once(f"paged_attention: head_dim={q.shape[-1]} window={window} not covered by the HIP kernel; "
                     f"using the PyTorch reference")
    return paged_attention_reference(q, cache, block_table, q_start, q_len, kv_len, scale, window)
