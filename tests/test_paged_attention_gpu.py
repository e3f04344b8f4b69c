"""Paged-KV attention HIP kernels vs the fp32 PyTorch reference: decode, multi-token (speculative /
chunked prefill) rows, GQA groups, block sizes, KV splits, and the KV append scatter."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _native():
    from shuffle_exchange_amd.ops import native
    native.require_hip()


def _setup(seqs, nq, nkv, D, bs, seed=0):
    """seqs: list of (cached_tokens_before, new_tokens). Builds cache with random history."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    total_blocks = sum((c + n + bs - 1) // bs for c, n in seqs) + 3
    cache = torch.randn(total_blocks, 2, nkv, bs, D, device="cuda", generator=g).to(torch.bfloat16)
    perm = torch.randperm(total_blocks, device="cpu").tolist()
    maxb = max((c + n + bs - 1) // bs for c, n in seqs)
    bt = torch.zeros(len(seqs), maxb, dtype=torch.int32)
    q_start, q_len, kv_len, slots = [], [], [], []
    t = 0
    for i, (c, n) in enumerate(seqs):
        nb = (c + n + bs - 1) // bs
        blocks = [perm.pop() for _ in range(nb)]
        bt[i, :nb] = torch.tensor(blocks, dtype=torch.int32)
        q_start.append(t)
        q_len.append(n)
        kv_len.append(c + n)
        for p in range(c, c + n):
            slots.append(blocks[p // bs] * bs + p % bs)
        t += n
    T = t
    qkv = torch.randn(T, nq + 2 * nkv, D, device="cuda", generator=g).to(torch.bfloat16)
    i32 = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")
    return (qkv, cache, bt.cuda(), i32(q_start), i32(q_len), i32(kv_len),
            torch.tensor(slots, dtype=torch.int64, device="cuda"), max(kv_len))


@pytest.mark.parametrize("seqs", [[(0, 1)], [(37, 1), (500, 1), (0, 5)], [(130, 3), (1, 20), (2000, 1)],
                                  [(0, 70)], [(4100, 1)] * 2])
@pytest.mark.parametrize("nq,nkv,D,bs", [(8, 2, 128, 64), (4, 4, 64, 16), (32, 8, 128, 32)])
@pytest.mark.parametrize("splits", [None, 1, 3])
def test_paged_attention(seqs, nq, nkv, D, bs, splits):
    from shuffle_exchange_amd.ops.paged_attention import (kv_cache_append, paged_attention,
                                                          paged_attention_reference)
    qkv, cache, bt, qs, ql, kl, slots, maxkv = _setup(seqs, nq, nkv, D, bs)
    ref_cache = cache.clone()
    kv_cache_append(qkv, cache, slots, nq, nkv)
    kv_cache_append(qkv.cpu().float(), ref_cache_cpu := ref_cache.cpu().float(), slots.cpu(), nq, nkv)
    assert torch.equal(cache.cpu().float(), ref_cache_cpu)
    q = qkv[:, :nq]
    scale = D ** -0.5
    out = paged_attention(q, cache, bt, qs, ql, kl, scale, maxkv, splits)
    ref = paged_attention_reference(q.float(), cache.float(), bt, qs, ql, kl, scale)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("seqs", [[(37, 1), (500, 1), (0, 5)], [(130, 3), (1, 20), (2000, 1)], [(4100, 1)] * 2])
@pytest.mark.parametrize("nq,nkv,D,bs,window", [(8, 2, 128, 64, 256), (4, 1, 64, 16, 100), (8, 4, 256, 32, 0),
                                                (16, 2, 256, 64, 300)])
@pytest.mark.parametrize("splits", [None, 2])
def test_paged_attention_window_and_d256(seqs, nq, nkv, D, bs, window, splits):
    """Sliding-window decode / chunked rows (Mistral, Qwen2) and head dim 256 on the HIP kernel ==
    the fp32 reference with the same window."""
    from shuffle_exchange_amd.ops.paged_attention import (kv_cache_append, paged_attention,
                                                          paged_attention_reference)
    qkv, cache, bt, qs, ql, kl, slots, maxkv = _setup(seqs, nq, nkv, D, bs, seed=3)
    kv_cache_append(qkv, cache, slots, nq, nkv)
    q = qkv[:, :nq]
    scale = D ** -0.5
    w = window or None
    out = paged_attention(q, cache, bt, qs, ql, kl, scale, maxkv, splits, window=w)
    ref = paged_attention_reference(q.float(), cache.float(), bt, qs, ql, kl, scale, w)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


def test_fused_rope_kv_cache_append_matches_separate_ops():
    """rope_kv_cache_append (one launch) == apply_rope_tokens_ + kv_cache_append (same math; bf16
    rounding may differ by FMA contraction), including skipped (-1) slots that stay untouched."""
    import torch
    from shuffle_exchange_amd.ops import native
    from shuffle_exchange_amd.ops.paged_attention import kv_cache_append, rope_kv_cache_append
    from shuffle_exchange_amd.ops.rope import RopeCache, apply_rope_tokens_
    native.require_hip()
    torch.manual_seed(0)
    for D in (64, 128):
        T, nq, nkv, bs, nblk = 37, 8, 2, 16, 8
        rope = RopeCache(D, 512, 10000.0, device="cuda")
        qkv = torch.randn(T, nq + 2 * nkv, D, device="cuda", dtype=torch.bfloat16)
        pos = torch.randint(0, 512, (T,), device="cuda")
        slots = torch.randperm(nblk * bs, device="cuda")[:T].long()
        slots[::7] = -1
        c1 = torch.zeros(nblk, 2, nkv, bs, D, device="cuda", dtype=torch.bfloat16)
        c2 = torch.zeros_like(c1)
        a, b = qkv.clone(), qkv.clone()
        apply_rope_tokens_(a, rope, nq + nkv, pos)
        kv_cache_append(a, c1, slots, nq, nkv)
        rope_kv_cache_append(b, rope, pos, c2, slots, nq, nkv)
        torch.testing.assert_close(b, a, rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(c2, c1, rtol=1e-2, atol=1e-2)
        assert torch.equal(c2 == 0, c1 == 0)


@pytest.mark.parametrize("splits", [2, 4])
def test_merge_attention_parts_matches_fused_kernel(splits):
    """The PyTorch merge of the KV-split partials (v2 llama decode's fallback when the o_proj
    weight is not covered by the fused merge GEMM) equals the kernel's merged output and the fp32
    reference."""
    from shuffle_exchange_amd.ops.paged_attention import (merge_attention_parts, paged_attention,
                                                          paged_attention_parts, paged_attention_reference)
    qkv, cache, bt, qs, ql, kl, slots, maxkv = _setup([(700, 1), (1500, 1), (37, 1)], 8, 2, 128, 64)
    q = qkv[:, :8]
    scale = 128 ** -0.5
    out, parts = paged_attention_parts(q, cache, bt, qs, ql, kl, scale, maxkv, splits)
    assert out is None and parts is not None
    merged = merge_attention_parts(parts[0], parts[1], q.dtype)
    fused = paged_attention(q, cache, bt, qs, ql, kl, scale, maxkv, splits)
    ref = paged_attention_reference(q.float(), cache.float(), bt, qs, ql, kl, scale)
    torch.testing.assert_close(merged.float(), fused.float(), atol=2e-2, rtol=2e-2)
    assert ((merged.float() - ref).norm() / ref.norm()).item() < 1e-2


@pytest.mark.parametrize("splits", [2, 5, 16])
def test_in_kernel_split_merge_matches_merge_launch(splits, monkeypatch):
    """Decode with the last split workgroup merging in-kernel (arrival counters) == the separate
    merge launch, over repeated launches and HIP-graph replays (the counters must self-reset)."""
    from shuffle_exchange_amd.ops import paged_attention as PA
    qkv, cache, bt, qs, ql, kl, slots, maxkv = _setup([(700, 1), (1500, 1), (37, 1), (3000, 1)], 32, 8, 128, 16)
    q = qkv[:, :32]
    scale = 128 ** -0.5
    monkeypatch.setattr(PA, "PA_LAST_MERGE", False)
    sep = PA.paged_attention(q, cache, bt, qs, ql, kl, scale, maxkv, splits)
    monkeypatch.setattr(PA, "PA_LAST_MERGE", True)
    ref = PA.paged_attention_reference(q.float(), cache.float(), bt, qs, ql, kl, scale)
    for _ in range(3):
        last = PA.paged_attention(q, cache, bt, qs, ql, kl, scale, maxkv, splits)
        torch.testing.assert_close(last.float(), sep.float(), atol=1e-2, rtol=1e-2)
    assert ((last.float() - ref).norm() / ref.norm()).item() < 1e-2
    assert int(PA._COUNTERS[q.device].abs().sum()) == 0
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        PA.paged_attention(q, cache, bt, qs, ql, kl, scale, maxkv, splits)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = PA.paged_attention(q, cache, bt, qs, ql, kl, scale, maxkv, splits)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(out.float(), sep.float(), atol=1e-2, rtol=1e-2)
    assert int(PA._COUNTERS[q.device].abs().sum()) == 0
