"""Decode skinny GEMM (csrc/kernels/skinny_gemm.hip) vs an fp32 PyTorch reference: M <= 16 rows,
ragged N / K tails, strided activation rows, bias; and the ops.linear dispatch under no_grad."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _native():
    from shuffle_exchange_amd.ops import native
    native.require_hip()


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("N,K", [(16, 8), (100, 264), (4104, 4096), (1000, 14336), (33, 1032)])
@pytest.mark.parametrize("with_bias", [False, True])
def test_skinny_gemm_matches_fp32(M, N, K, with_bias):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    xs = torch.randn(M, K + 16, device="cuda", dtype=torch.bfloat16, generator=g)
    x = xs[:, :K]  # row stride K + 16
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16, generator=g) if with_bias else None
    y = torch.ops.sxe.skinny_gemm(x, w, b)
    ref = x.float() @ w.float().t() + (b.float() if b is not None else 0)
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("M", [1, 4])
@pytest.mark.parametrize("N,K", [(100, 264), (4104, 4096)])
def test_skinny_gemm_nontemporal_loads_match(M, N, K, monkeypatch):
    """SXE_SKINNY_NT=1 (non-temporal weight loads: separate kernel instantiations) gives the same
    bits as the default loads, for the plain GEMM and the fused RMSNorm / SwiGLU prologues."""
    g = torch.Generator(device="cuda").manual_seed(N + K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g)
    gw = torch.rand(K, device="cuda", generator=g).bfloat16()
    x2 = torch.randn(M, 2 * K, device="cuda", dtype=torch.bfloat16, generator=g)
    outs = []
    for nt in ("0", "1"):
        monkeypatch.setenv("SXE_SKINNY_NT", nt)
        y = torch.ops.sxe.skinny_gemm(x, w, None)
        yr = torch.ops.sxe.skinny_gemm_pro(x, None, gw, 1e-5, w, None, None, 1)[0]
        ys = torch.ops.sxe.skinny_gemm_pro(x2, None, None, 0.0, w, None, None, 2)[0]
        outs.append((y, yr, ys))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_linear_dispatches_skinny_under_no_grad():
    from shuffle_exchange_amd.ops.linear import linear
    w = torch.randn(256, 512, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(2, 3, 512, device="cuda", dtype=torch.bfloat16)
    with torch.no_grad():
        y = linear(x, w)
    assert y.shape == (2, 3, 256)
    torch.testing.assert_close(y.float(), (x.float() @ w.float().t()), atol=0.25, rtol=2e-2)
    xg = x.clone().requires_grad_()
    linear(xg, w).sum().backward()  # autograd path still works (F.linear)
    assert xg.grad is not None


@pytest.mark.parametrize("M", [1, 4, 16])
@pytest.mark.parametrize("N,K", [(16, 64), (100, 576), (4104, 4096), (1000, 14336)])
def test_skinny_gemm_fp8_weights_matches_fp32(M, N, K):
    from shuffle_exchange_amd.ops.fp_quantizer import quantize_weight_fp8_rowwise
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16, generator=g)
    q, s = quantize_weight_fp8_rowwise(w)
    y = torch.ops.sxe.skinny_gemm_fp8w(x, q.view(torch.uint8), s, b)
    ref = x.float() @ (q.float() * s[:, None]).t() + b.float()  # exact dequantized weights
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("kind,min_cos", [("fp8", 0.99), ("fp6", 0.98), ("fp4", 0.8)])
def test_hf_engine_quantized_weights_close_to_bf16(kind, min_cos):
    transformers = pytest.importorskip("transformers")
    from shuffle_exchange_amd.inference.v2.engine_factory import build_hf_engine
    from shuffle_exchange_amd.inference.v2.engine_v2 import RaggedInferenceEngineConfig
    torch.manual_seed(0)
    T = transformers
    model = T.LlamaForCausalLM(T.LlamaConfig(hidden_size=512, intermediate_size=1024, num_attention_heads=4,
                                             num_key_value_heads=2, vocab_size=512, num_hidden_layers=2)).eval()
    cfg = RaggedInferenceEngineConfig(kv_block_size=64, num_kv_blocks=32)
    e16 = build_hf_engine(model, cfg, device="cuda")
    e8 = build_hf_engine(model, RaggedInferenceEngineConfig(kv_block_size=64, num_kv_blocks=32), device="cuda",
                         weight_quant=kind)
    p = torch.randint(0, 512, (40,)).tolist()
    a, b = e16.put([0], [p]), e8.put([0], [p])
    for t in (5, 9, 11):
        a, b = e16.put([0], [[t]]), e8.put([0], [[t]])  # decode steps: skinny FP8 / FP6 / FP4-weight kernels
        cos = torch.nn.functional.cosine_similarity(a.float(), b.float()).item()
        assert cos > min_cos, (kind, cos)


@pytest.mark.parametrize("M", [1, 3, 4])
@pytest.mark.parametrize("K,N", [(4096, 6144), (4096, 28672), (512, 200)])
@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("with_res", [True, False])
def test_fused_rms_prologue_vs_fp32(M, K, N, fp8, with_res):
    """skinny_gemm_pro mode 1: residual add + RMSNorm + GEMM in one launch == the fp32 reference of
    the separate ops (h rounded to bf16 like the norm kernel), and h = x + res written out."""
    from shuffle_exchange_amd.ops.fp_quantizer import FP8Weight
    from shuffle_exchange_amd.ops.linear import fused_rms_linear
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    res = torch.randn(M, K, device="cuda", dtype=torch.bfloat16) if with_res else None
    g = (1.0 + 0.1 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    w = (0.02 * torch.randn(N, K, device="cuda")).to(torch.bfloat16)
    wobj = FP8Weight(w) if fp8 else w
    y, h = fused_rms_linear(x, res, g, 1e-5, wobj)
    hr = (x.float() + res.float()).bfloat16().float() if with_res else x.float()
    a = hr * torch.rsqrt(hr.square().mean(-1, keepdim=True) + 1e-5) * g.float()
    wr = wobj.dequantize().float() if fp8 else w.float()
    ref = a @ wr.t()
    assert torch.equal(h.float(), hr)
    err = ((y.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("I,N", [(14336, 4096), (512, 256)])
@pytest.mark.parametrize("fp8", [False, True])
def test_fused_swiglu_prologue_vs_fp32(M, I, N, fp8):
    from shuffle_exchange_amd.ops.fp_quantizer import FP8Weight
    from shuffle_exchange_amd.ops.linear import fused_swiglu_linear
    torch.manual_seed(1)
    gu = torch.randn(M, 2 * I, device="cuda", dtype=torch.bfloat16)
    w = (0.02 * torch.randn(N, I, device="cuda")).to(torch.bfloat16)
    wobj = FP8Weight(w) if fp8 else w
    y = fused_swiglu_linear(gu, wobj)
    g, u = gu.float().chunk(2, dim=-1)
    a = torch.nn.functional.silu(g) * u
    wr = wobj.dequantize().float() if fp8 else w.float()
    ref = a @ wr.t()
    err = ((y.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


def test_decode_fused_layer_matches_unfused(monkeypatch):
    """Ragged engine decode with the fused prologues == with them disabled (same greedy tokens,
    logits within bf16 rounding)."""
    import os
    from shuffle_exchange_amd.inference.v2 import RaggedInferenceEngineConfig, build_engine
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=512, intermediate_size=1024, num_attention_heads=8,
                       num_key_value_heads=2, vocab_size=1000, num_hidden_layers=2)
    model = LlamaForCausalLM(cfg).cuda().bfloat16().eval()
    prompt = torch.randint(0, cfg.vocab_size, (12,)).tolist()
    outs = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("SXE_DECODE_FUSE", fuse)
        eng = build_engine(model, RaggedInferenceEngineConfig(kv_block_size=16, num_kv_blocks=64))
        logits = eng.put([1], [torch.tensor(prompt)])
        toks, lg = [], []
        for _ in range(6):
            t = int(logits[0].argmax())
            toks.append(t)
            logits = eng.put([1], [torch.tensor([t])])
            lg.append(logits.float())
        eng.flush(1)
        outs.append((toks, torch.cat(lg)))
    assert outs[0][0] == outs[1][0]
    err = ((outs[0][1] - outs[1][1]).norm() / outs[1][1].norm()).item()
    assert err < 2e-2, err


@pytest.mark.parametrize("M", [1, 3])
@pytest.mark.parametrize("splits", [2, 16, 37])
@pytest.mark.parametrize("nq,D,N", [(32, 128, 4096), (8, 64, 200)])
@pytest.mark.parametrize("fp8", [False, True])
def test_fused_merge_prologue_vs_fp32(M, splits, nq, D, N, fp8):
    """skinny_gemm_merge: the flash-decoding merge of KV-split partials (some splits empty: max -inf)
    as the o_proj GEMM's prologue == the fp32 merge followed by the GEMM."""
    from shuffle_exchange_amd.ops.fp_quantizer import FP8Weight
    from shuffle_exchange_amd.ops.linear import fused_merge_linear
    torch.manual_seed(2)
    po = torch.randn(splits, M, nq, D, device="cuda")
    mx = 4 * torch.randn(splits, M, nq, device="cuda")
    mx[-1, :, ::3] = float("-inf")  # a split past the sequence's keys
    ls = torch.rand(splits, M, nq, device="cuda") * 8 + 0.5
    pml = torch.stack([mx, ls], -1).contiguous()
    w = (0.02 * torch.randn(N, nq * D, device="cuda")).to(torch.bfloat16)
    wobj = FP8Weight(w) if fp8 else w
    y = fused_merge_linear(po, pml, wobj)
    f = torch.where(mx == float("-inf"), torch.zeros_like(mx), torch.exp2(mx - mx.amax(0, keepdim=True)))
    o = (f[..., None] * po).sum(0) / (f * ls).sum(0)[..., None]  # [M, nq, D]
    a = o.reshape(M, nq * D).bfloat16().float()
    wr = wobj.dequantize().float() if fp8 else w.float()
    ref = a @ wr.t()
    err = ((y.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


def test_decode_merge_fused_o_proj_matches_unfused(monkeypatch):
    """Ragged engine decode over a context long enough for several KV splits: the merge fused into
    the o_proj launch == the separate merge kernel + GEMM (same greedy tokens, logits within bf16)."""
    from shuffle_exchange_amd.inference.v2 import RaggedInferenceEngineConfig, build_engine
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    from shuffle_exchange_amd.ops import paged_attention as pa
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=512, intermediate_size=1024, num_attention_heads=8,
                       num_key_value_heads=2, vocab_size=1000, num_hidden_layers=2)
    model = LlamaForCausalLM(cfg).cuda().bfloat16().eval()
    prompt = torch.randint(0, cfg.vocab_size, (200,)).tolist()  # < max_position_embeddings (256)
    monkeypatch.setattr(pa, "PA_MIN_KEYS", 64)  # several KV splits at this short context
    assert pa.choose_splits(1, 2, 206) > 1
    import shuffle_exchange_amd.ops.linear as lin
    calls = {"n": 0}
    real = lin.fused_merge_linear

    def counting(*a, **k):
        y = real(*a, **k)
        calls["n"] += y is not None
        return y
    monkeypatch.setattr(lin, "fused_merge_linear", counting)
    outs = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("SXE_DECODE_FUSE", fuse)
        eng = build_engine(model, RaggedInferenceEngineConfig(kv_block_size=16, num_kv_blocks=64))
        logits = eng.put([1], [torch.tensor(prompt)])
        toks, lg = [], []
        for _ in range(5):
            t = int(logits[0].argmax())
            toks.append(t)
            logits = eng.put([1], [torch.tensor([t])])
            lg.append(logits.float())
        eng.flush(1)
        outs.append((toks, torch.cat(lg)))
        if fuse == "1":
            assert calls["n"] > 0  # the fused launch really ran
    assert outs[0][0] == outs[1][0]
    err = ((outs[0][1] - outs[1][1]).norm() / outs[1][1].norm()).item()
    assert err < 2e-2, err


@pytest.mark.parametrize("M", [1, 3])
@pytest.mark.parametrize("nq,nkv", [(32, 8), (4, 2)])
@pytest.mark.parametrize("fp8", [False, True])
def test_fused_rms_rope_epilogue_vs_separate_ops(M, nq, nkv, fp8):
    """skinny_gemm_pro_rope (RMSNorm prologue + QKV GEMM + RoPE / KV-append epilogue) == the fused
    RMS GEMM followed by rope_kv_cache_append (rotation from the fp32 accumulator instead of the
    bf16-rounded output: within bf16 rounding); slots of -1 leave the cache untouched."""
    from shuffle_exchange_amd.ops.fp_quantizer import FP8Weight
    from shuffle_exchange_amd.ops.linear import fused_rms_linear, fused_rms_rope_linear
    from shuffle_exchange_amd.ops.paged_attention import rope_kv_cache_append
    from shuffle_exchange_amd.ops.rope import RopeCache
    torch.manual_seed(3)
    K, D, bs, nblk = 1024, 128, 16, 8
    N = (nq + 2 * nkv) * D
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    res = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    g = (1.0 + 0.1 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    w = (0.05 * torch.randn(N, K, device="cuda")).to(torch.bfloat16)
    wobj = FP8Weight(w) if fp8 else w
    rope = RopeCache(D, 4096, 500000.0, device="cuda")
    pos = torch.randint(0, 4096, (M,), device="cuda")
    slots = torch.randperm(nblk * bs, device="cuda")[:M].long()
    if M > 1:
        slots[1] = -1
    c_ref = torch.randn(nblk, 2, nkv, bs, D, device="cuda").to(torch.bfloat16)
    c_f = c_ref.clone()
    y_ref, h_ref = fused_rms_linear(x, res, g, 1e-5, wobj)
    q_ref = y_ref.view(M, nq + 2 * nkv, D).clone()
    rope_kv_cache_append(q_ref, rope, pos, c_ref, slots, nq, nkv)
    y, h = fused_rms_rope_linear(x, res, g, 1e-5, wobj, rope, pos, c_f, slots, nq, nkv)
    assert torch.equal(h, h_ref)
    torch.testing.assert_close(y.view(M, nq + 2 * nkv, D).float(), q_ref.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(c_f.float(), c_ref.float(), rtol=2e-2, atol=2e-2)
    written = torch.zeros(nblk, bs, dtype=torch.bool, device="cuda")
    ok = slots[slots >= 0]
    written[ok // bs, ok % bs] = True
    diff = (c_f != c_ref).any(dim=-1).any(dim=2).any(dim=1)  # [blocks, bs]
    assert not (diff & ~written).any()  # no stray writes outside the appended slots
