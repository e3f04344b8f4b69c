"""v1 kernel injection (module_inject/replace_module.py): Hugging Face BERT / RoBERTa / GPT-2 layers
replaced by the fused layers give the same outputs as the original modules (random-init tiny
configs: no hub access), with padding masks, and GPT-2 greedy generation through the HF KV cache
matches token for token."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from shuffle_exchange_amd.module_inject import replace_module as rm  # noqa: E402


def replace_transformer_layer(model):
    """Inject, then drop the originals: a fused layer that silently delegated would fail."""
    n = rm.replace_transformer_layer(model)
    for m in model.modules():
        if isinstance(m, rm._Fused):
            m.__dict__["orig"] = None
    return n


def _bert(cls_name="Bert"):
    cfg = getattr(transformers, f"{cls_name}Config")(vocab_size=200, hidden_size=64, num_hidden_layers=2,
                                                     num_attention_heads=4, intermediate_size=128,
                                                     max_position_embeddings=64)
    torch.manual_seed(0)
    return getattr(transformers, f"{cls_name}Model")(cfg).eval()


@pytest.mark.parametrize("arch", ["Bert", "Roberta"])
def test_encoder_injection_matches_hf(arch):
    model = _bert(arch)
    ids = torch.randint(3, 200, (2, 12))
    mask = torch.ones(2, 12, dtype=torch.long)
    mask[1, 8:] = 0
    with torch.no_grad():
        ref = model(ids, attention_mask=mask).last_hidden_state
        n = replace_transformer_layer(model)
        got = model(ids, attention_mask=mask).last_hidden_state
    assert n == 2
    torch.testing.assert_close(got[0], ref[0], atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(got[1, :8], ref[1, :8], atol=2e-5, rtol=1e-4)


def _gpt2():
    cfg = transformers.GPT2Config(vocab_size=300, n_positions=64, n_embd=64, n_layer=2, n_head=4)
    torch.manual_seed(0)
    return transformers.GPT2LMHeadModel(cfg).eval()


def test_gpt2_injection_logits_and_generate():
    model = _gpt2()
    ids = torch.randint(0, 300, (2, 10))
    with torch.no_grad():
        ref = model(ids, use_cache=False).logits
        ref_gen = model.generate(ids, max_new_tokens=6, do_sample=False, pad_token_id=0)
        n = replace_transformer_layer(model)
        got = model(ids, use_cache=False).logits
        got_gen = model.generate(ids, max_new_tokens=6, do_sample=False, pad_token_id=0)
    assert n == 2
    torch.testing.assert_close(got, ref, atol=5e-5, rtol=1e-4)
    assert torch.equal(got_gen, ref_gen)


def test_init_inference_injects_hf_layers():
    import shuffle_exchange_amd as sxe
    model = _gpt2()
    ids = torch.randint(0, 300, (1, 8))
    with torch.no_grad():
        ref = model(ids, use_cache=False).logits.float()
    eng = sxe.init_inference(model, dtype=torch.float32, replace_with_kernel_inject=True)
    assert eng.injected_layers == 2
    with torch.no_grad():
        got = eng(ids.to(eng.device), use_cache=False).logits.float().cpu()
    torch.testing.assert_close(got, ref, atol=5e-5, rtol=1e-4)


@pytest.mark.gpu
def test_gpt2_injection_gpu_bf16_flash_path():
    """On the MI355X: bf16 GPT-2 with head dim 128 runs the HIP flash kernel inside the injected
    block; logits track the original HF block in bf16."""
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    cfg = transformers.GPT2Config(vocab_size=512, n_positions=256, n_embd=512, n_layer=2, n_head=4)
    torch.manual_seed(0)
    model = transformers.GPT2LMHeadModel(cfg).eval().to("cuda", torch.bfloat16)
    ids = torch.randint(0, 512, (2, 128), device="cuda")
    with torch.no_grad():
        ref = model(ids, use_cache=False).logits.float()
        replace_transformer_layer(model)
        got = model(ids, use_cache=False).logits.float()
        gen = model.generate(ids[:, :16], max_new_tokens=4, do_sample=False, pad_token_id=0)
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 2e-2, rel
    assert gen.shape == (2, 20)


@pytest.mark.parametrize("parallel", [True, False])
def test_gpt_neox_injection_logits_and_generate(parallel):
    cfg = transformers.GPTNeoXConfig(vocab_size=300, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                                     intermediate_size=128, max_position_embeddings=64, rotary_pct=0.5,
                                     use_parallel_residual=parallel)
    torch.manual_seed(0)
    model = transformers.GPTNeoXForCausalLM(cfg).eval()
    ids = torch.randint(0, 300, (2, 10))
    with torch.no_grad():
        ref = model(ids, use_cache=False).logits
        ref_gen = model.generate(ids, max_new_tokens=6, do_sample=False, pad_token_id=0)
        n = replace_transformer_layer(model)
        got = model(ids, use_cache=False).logits
        got_gen = model.generate(ids, max_new_tokens=6, do_sample=False, pad_token_id=0)
    assert n == 2
    torch.testing.assert_close(got, ref, atol=5e-5, rtol=1e-4)
    assert torch.equal(got_gen, ref_gen)


def test_decoder_bert_is_not_injected():
    """BERT/RoBERTa configured as decoders (causal self-attention + KV cache) keep their HF layers."""
    cfg = transformers.BertConfig(vocab_size=200, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                                  intermediate_size=128, max_position_embeddings=64, is_decoder=True)
    torch.manual_seed(0)
    model = transformers.BertLMHeadModel(cfg).eval()
    ids = torch.randint(3, 200, (2, 10))
    with torch.no_grad():
        ref = model(ids).logits
        n = rm.replace_transformer_layer(model)
        got = model(ids).logits
    assert n == 0
    torch.testing.assert_close(got, ref)


def test_fused_layers_share_weight_memory_and_delegate_after_to():
    """The original module's parameters are views of the fused tensors (no second copy of the
    weights), delegation still matches HF, also after a dtype move of the model."""
    model = _bert("Bert")
    ids = torch.randint(3, 200, (2, 12))
    with torch.no_grad():
        ref = model(ids, output_attentions=True)
        n = rm.replace_transformer_layer(model)
    assert n == 2
    layer = model.encoder.layer[0]
    orig = layer.orig
    assert orig.attention.self.query.weight.data_ptr() == layer.w_qkv.data_ptr()
    assert orig.output.dense.weight.data_ptr() == layer.w_out.data_ptr()
    with torch.no_grad():
        got = model(ids, output_attentions=True)  # delegated path
    torch.testing.assert_close(got.last_hidden_state, ref.last_hidden_state, atol=2e-5, rtol=1e-4)
    model.double()
    assert orig.attention.self.key.weight.dtype == torch.float64
    assert orig.attention.self.key.weight.data_ptr() == layer.w_qkv.data_ptr() + 64 * 64 * 8
    with torch.no_grad():
        got64 = model(ids, output_attentions=True).last_hidden_state
    torch.testing.assert_close(got64.float(), ref.last_hidden_state, atol=1e-4, rtol=1e-4)


def test_gpt2_left_padded_batched_generate():
    model = _gpt2()
    ids = torch.randint(1, 300, (2, 9))
    mask = torch.ones_like(ids)
    ids[1, :3] = 0
    mask[1, :3] = 0  # left padding
    with torch.no_grad():
        ref = model.generate(ids, attention_mask=mask, max_new_tokens=5, do_sample=False, pad_token_id=0)
        rm.replace_transformer_layer(model)
        got = model.generate(ids, attention_mask=mask, max_new_tokens=5, do_sample=False, pad_token_id=0)
    assert torch.equal(got, ref)


def test_init_inference_injects_and_quantizes():
    """Kernel injection with post-init weight quantization: the injected layers' GEMM weights are
    stored int8 (a key matching one of the layer's HF submodules selects it), logits stay close."""
    import shuffle_exchange_amd as sxe
    model = _gpt2()
    ids = torch.randint(0, 300, (1, 8))
    with torch.no_grad():
        ref = model(ids, use_cache=False).logits
    eng = sxe.init_inference(model, dtype=torch.float32, replace_with_kernel_inject=True,
                             weight_quantization={"post_init_quant": {"c_fc": {"num_bits": 8, "group_size": 64}}})
    assert eng.injected_layers == 2 and eng.injection_skipped is None
    fused = [m for m in model.modules() if isinstance(m, rm._Fused)]
    assert len(fused) == 2 and all(isinstance(m.w_qkv, rm._FusedQWeight) for m in fused)
    assert all(isinstance(m.w_out, rm._FusedQWeight) for m in fused)
    with torch.no_grad():
        out = eng(ids.to(eng.device), use_cache=False).logits
    rel = ((out.cpu() - ref).norm() / ref.norm()).item()
    assert rel < 2e-2, rel


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["gpt2", "bert"])
def test_real_head_dim_injection_runs_hip_flash(arch, monkeypatch):
    """Real GPT-2 / BERT-base geometry (768 hidden, 12 heads -> D = 64, S = 200): the injected layers
    run the HIP flash kernels (padded head dim / sequence), not SDPA."""
    from shuffle_exchange_amd.ops import attention as A
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    calls = {"hip": 0}
    real = torch.ops.sxe.flash_attn_fwd

    class _Spy:
        def __call__(self, *a, **k):
            calls["hip"] += 1
            return real(*a, **k)
    monkeypatch.setattr(A, "_sdpa", lambda *a, **k: (_ for _ in ()).throw(AssertionError("SDPA fallback")))
    torch.manual_seed(0)
    if arch == "gpt2":
        cfg = transformers.GPT2Config(vocab_size=512, n_positions=256, n_embd=768, n_layer=2, n_head=12)
        model = transformers.GPT2LMHeadModel(cfg).eval().to("cuda", torch.bfloat16)
    else:
        cfg = transformers.BertConfig(vocab_size=512, hidden_size=768, num_hidden_layers=2, num_attention_heads=12,
                                      intermediate_size=3072, max_position_embeddings=256)
        model = transformers.BertModel(cfg).eval().to("cuda", torch.bfloat16)
    ids = torch.randint(0, 512, (2, 200), device="cuda")
    with torch.no_grad():
        ref = model(ids).logits.float() if arch == "gpt2" else model(ids).last_hidden_state.float()
        replace_transformer_layer(model)
        monkeypatch.setattr(torch.ops.sxe, "flash_attn_fwd", _Spy(), raising=False)
        got = model(ids).logits.float() if arch == "gpt2" else model(ids).last_hidden_state.float()
    assert calls["hip"] == 2
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 2e-2, rel


def _decoder(arch, max_pos=64):
    torch.manual_seed(0)
    if arch == "llama":
        cfg = transformers.LlamaConfig(vocab_size=300, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=max_pos)
        return transformers.LlamaForCausalLM(cfg).eval()
    if arch == "qwen2":
        cfg = transformers.Qwen2Config(vocab_size=300, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=max_pos)
        return transformers.Qwen2ForCausalLM(cfg).eval()
    if arch == "mistral":
        cfg = transformers.MistralConfig(vocab_size=300, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                                         num_attention_heads=4, num_key_value_heads=1, max_position_embeddings=max_pos,
                                         sliding_window=None)
        return transformers.MistralForCausalLM(cfg).eval()
    if arch == "opt":
        cfg = transformers.OPTConfig(vocab_size=300, hidden_size=64, ffn_dim=128, num_hidden_layers=2,
                                     num_attention_heads=4, max_position_embeddings=max_pos, word_embed_proj_dim=64)
        return transformers.OPTForCausalLM(cfg).eval()
    if arch == "gptj":
        cfg = transformers.GPTJConfig(vocab_size=300, n_embd=64, n_layer=2, n_head=4, rotary_dim=8, n_positions=max_pos)
        return transformers.GPTJForCausalLM(cfg).eval()
    if arch == "bloom":
        cfg = transformers.BloomConfig(vocab_size=300, hidden_size=64, n_layer=2, n_head=4)
        return transformers.BloomForCausalLM(cfg).eval()
    if arch == "gptneo":
        cfg = transformers.GPTNeoConfig(vocab_size=300, hidden_size=64, num_layers=2, num_heads=4,
                                        attention_types=[[["global", "local"], 1]], window_size=4,
                                        max_position_embeddings=max_pos)
        return transformers.GPTNeoForCausalLM(cfg).eval()
    raise ValueError(arch)


@pytest.mark.parametrize("arch", ["llama", "qwen2", "mistral", "opt", "gptj", "bloom", "gptneo"])
def test_decoder_injection_logits_and_generate(arch):
    """Llama / Qwen2 / Mistral (GQA, RoPE, SwiGLU), OPT (biased QKV, pre-LN, ReLU), GPT-J (parallel
    residual, interleaved partial rotary), BLOOM (ALiBi, head-interleaved QKV) and GPT-Neo (unscaled
    scores, alternating global / local-window layers) injection: logits and greedy generation through
    the HF cache match the original modules (reference module_inject/containers/{llama,llama2,opt,
    gptj,bloom,gptneo}.py)."""
    model = _decoder(arch)
    ids = torch.randint(3, 300, (2, 10))
    with torch.no_grad():
        ref = model(ids, use_cache=False).logits
        ref_gen = model.generate(ids, max_new_tokens=6, do_sample=False, pad_token_id=0)
        n = replace_transformer_layer(model)
        got = model(ids, use_cache=False).logits
        got_gen = model.generate(ids, max_new_tokens=6, do_sample=False, pad_token_id=0)
    assert n == 2
    torch.testing.assert_close(got, ref, atol=5e-5, rtol=1e-4)
    assert torch.equal(got_gen, ref_gen)


def test_distilbert_injection_matches_hf():
    cfg = transformers.DistilBertConfig(vocab_size=200, dim=64, n_layers=2, n_heads=4, hidden_dim=128,
                                        max_position_embeddings=64)
    torch.manual_seed(0)
    model = transformers.DistilBertModel(cfg).eval()
    ids = torch.randint(3, 200, (2, 12))
    mask = torch.ones(2, 12, dtype=torch.long)
    mask[1, 8:] = 0
    with torch.no_grad():
        ref = model(ids, attention_mask=mask).last_hidden_state
        n = replace_transformer_layer(model)
        got = model(ids, attention_mask=mask).last_hidden_state
    assert n == 2
    torch.testing.assert_close(got[0], ref[0], atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(got[1, :8], ref[1, :8], atol=2e-5, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["llama", "opt", "gptj", "bloom", "gptneo"])
def test_decoder_injection_gpu_bf16(arch):
    """The new decoder policies on the MI355X in bf16 (HIP norm / GEMM / activation / flash kernels):
    logits close to the HF modules, greedy generation runs through the HF cache."""
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    model = _decoder(arch, max_pos=256).to("cuda", torch.bfloat16)  # positions must cover the 130 tokens
    ids = torch.randint(3, 300, (2, 130), device="cuda")
    assert ids.shape[1] + 8 <= 256
    with torch.no_grad():
        ref = model(ids, use_cache=False).logits.float()
        assert replace_transformer_layer(model) == 2
        got = model(ids, use_cache=False).logits.float()
        gen = model.generate(ids[:, :16], max_new_tokens=4, do_sample=False, pad_token_id=0)
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 3e-2, rel
    assert gen.shape == (2, 20)


def _clip(kind, dev="cpu", dtype=torch.float32):
    torch.manual_seed(0)
    if kind == "text":
        cfg = transformers.CLIPTextConfig(vocab_size=300, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                                          num_attention_heads=2, max_position_embeddings=64)
        return transformers.CLIPTextModel(cfg).eval().to(dev, dtype), cfg
    cfg = transformers.CLIPVisionConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                                        num_attention_heads=2, image_size=32, patch_size=8)
    return transformers.CLIPVisionModel(cfg).eval().to(dev, dtype), cfg


@pytest.mark.parametrize("kind", ["text", "vision"])
def test_clip_injection_matches_hf(kind):
    """CLIP text (causal) and vision towers (reference containers/clip.py): quick-GELU MLP, packed QKV."""
    model, cfg = _clip(kind)
    if kind == "text":
        inp = {"input_ids": torch.randint(3, 300, (2, 12))}
    else:
        inp = {"pixel_values": torch.randn(2, 3, 32, 32)}
    with torch.no_grad():
        ref = model(**inp).last_hidden_state
        n = replace_transformer_layer(model)
        got = model(**inp).last_hidden_state
    assert n == 2
    torch.testing.assert_close(got, ref, atol=5e-5, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["text", "vision"])
def test_clip_injection_gpu_bf16(kind):
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    model, cfg = _clip(kind, "cuda", torch.bfloat16)
    inp = ({"input_ids": torch.randint(3, 300, (2, 40), device="cuda")} if kind == "text"
           else {"pixel_values": torch.randn(2, 3, 32, 32, device="cuda", dtype=torch.bfloat16)})
    with torch.no_grad():
        ref = model(**inp).last_hidden_state.float()
        assert replace_transformer_layer(model) == 2
        got = model(**inp).last_hidden_state.float()
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 3e-2, rel
