"""FastGen model zoo parity: the ragged engine serving Hugging Face checkpoints of every family the
reference's inference/v2/model_implementations covers (Llama, Mistral, Mixtral, Qwen2, Qwen2-MoE,
Phi, Phi-3, Falcon (multi-query and new-architecture GQA), OPT) must reproduce the transformers
implementation's logits -- prefill of a ragged batch, then KV-cached decode steps -- on random tiny
configs (fp32, CPU reference kernels). Also covers loading from a checkpoint directory."""
import pytest
import torch

transformers = pytest.importorskip("transformers")


def _tiny(name):
    T = transformers
    common = dict(vocab_size=96, hidden_size=64, num_hidden_layers=2, num_attention_heads=4, pad_token_id=0,
                  bos_token_id=1, eos_token_id=2)
    if name == "llama":
        return T.LlamaForCausalLM(T.LlamaConfig(intermediate_size=96, num_key_value_heads=2, **common))
    if name == "llama31":
        rope = {"rope_type": "llama3", "rope_theta": 500000.0, "factor": 8.0, "low_freq_factor": 1.0,
                "high_freq_factor": 4.0, "original_max_position_embeddings": 32}
        return T.LlamaForCausalLM(T.LlamaConfig(intermediate_size=96, num_key_value_heads=2,
                                                rope_parameters=rope, **common))
    if name == "mistral":
        return T.MistralForCausalLM(T.MistralConfig(intermediate_size=96, num_key_value_heads=2, sliding_window=6,
                                                    **common))
    if name == "qwen2":
        return T.Qwen2ForCausalLM(T.Qwen2Config(intermediate_size=96, num_key_value_heads=2, **common))
    if name == "mixtral":
        return T.MixtralForCausalLM(T.MixtralConfig(intermediate_size=48, num_key_value_heads=2, num_local_experts=4,
                                                    num_experts_per_tok=2, **common))
    if name == "qwen2_moe":
        return T.Qwen2MoeForCausalLM(T.Qwen2MoeConfig(intermediate_size=96, num_key_value_heads=2, num_experts=4,
                                                      num_experts_per_tok=2, moe_intermediate_size=32,
                                                      shared_expert_intermediate_size=48, norm_topk_prob=True,
                                                      **common))
    if name == "phi":
        return T.PhiForCausalLM(T.PhiConfig(intermediate_size=96, partial_rotary_factor=0.5, **common))
    if name == "phi3":
        return T.Phi3ForCausalLM(T.Phi3Config(intermediate_size=96, num_key_value_heads=2, **common))
    if name == "falcon":
        return T.FalconForCausalLM(T.FalconConfig(vocab_size=96, hidden_size=64, num_hidden_layers=2,
                                                  num_attention_heads=4))
    if name == "falcon_new":
        return T.FalconForCausalLM(T.FalconConfig(vocab_size=96, hidden_size=64, num_hidden_layers=2,
                                                  num_attention_heads=4, num_kv_heads=2, new_decoder_architecture=True,
                                                  bias=True))
    if name == "opt":
        return T.OPTForCausalLM(T.OPTConfig(vocab_size=96, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                                            ffn_dim=96, word_embed_proj_dim=64, max_position_embeddings=64,
                                            pad_token_id=0))
    raise KeyError(name)


FAMILIES = ["llama", "llama31", "mistral", "qwen2", "mixtral", "qwen2_moe", "phi", "phi3", "falcon", "falcon_new",
            "opt"]


def _hf_last_logits(model, ids):
    with torch.no_grad():
        return model(torch.tensor([ids])).logits[0, -1].float()


def _engine(model_or_path, **kw):
    from shuffle_exchange_amd.inference.v2.engine_factory import build_hf_engine
    from shuffle_exchange_amd.inference.v2.engine_v2 import RaggedInferenceEngineConfig
    cfg = RaggedInferenceEngineConfig(kv_block_size=4, num_kv_blocks=64)
    return build_hf_engine(model_or_path, cfg, dtype=torch.float32, **kw)


@pytest.mark.parametrize("name", FAMILIES)
def test_ragged_engine_matches_transformers(name):
    torch.manual_seed(0)
    model = _tiny(name).eval()
    eng = _engine(model)
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(3, 96, (n,), generator=g).tolist() for n in (7, 11, 3)]
    # ragged prefill of three sequences in one put()
    logits = eng.put([0, 1, 2], prompts)
    for i, p in enumerate(prompts):
        ref = _hf_last_logits(model, p)
        assert torch.allclose(logits[i], ref, atol=2e-4, rtol=1e-4), (name, i, (logits[i] - ref).abs().max())
    # two KV-cached decode steps for sequences 0 and 2 together
    seqs = {0: list(prompts[0]), 2: list(prompts[2])}
    for step in range(2):
        toks = {u: int(torch.randint(3, 96, (1,), generator=g)) for u in seqs}
        out = eng.put(list(seqs), [[toks[u]] for u in seqs])
        for j, u in enumerate(seqs):
            seqs[u].append(toks[u])
            ref = _hf_last_logits(model, seqs[u])
            assert torch.allclose(out[j], ref, atol=2e-4, rtol=1e-4), (name, step, u, (out[j] - ref).abs().max())
    for u in (0, 1, 2):
        eng.flush(u)
    assert eng.free_blocks == eng.n_kv_blocks


def test_build_hf_engine_from_checkpoint_dir(tmp_path):
    torch.manual_seed(0)
    model = _tiny("qwen2").eval()
    model.save_pretrained(str(tmp_path))  # config.json + model.safetensors
    eng = _engine(str(tmp_path))
    ids = [5, 9, 17, 33, 2, 71]
    out = eng.put([7], [ids])
    assert torch.allclose(out[0], _hf_last_logits(model, ids), atol=2e-4, rtol=1e-4)
    gen = eng.generate([ids], max_new_tokens=4)
    ref = model.generate(torch.tensor([ids]), max_new_tokens=4, do_sample=False)[0, len(ids):].tolist()
    assert gen[0] == ref


def test_init_inference_kernel_inject_hf_model_generate():
    """v1 API (reference inference/engine.py + module_inject): init_inference on a transformers model
    with replace_with_kernel_inject routes generation through the ragged HF decoder."""
    import shuffle_exchange_amd as sxe
    torch.manual_seed(0)
    model = _tiny("mistral").eval()
    ref_model = _tiny("mistral").eval()
    ref_model.load_state_dict(model.state_dict())
    eng = sxe.init_inference(model, dtype=torch.float32, replace_with_kernel_inject=True)
    ids = torch.tensor([[5, 9, 17, 33, 2, 71, 8]])
    out = eng.generate(ids, max_new_tokens=5)
    ref = ref_model.generate(ids, max_new_tokens=5, do_sample=False)
    assert out.tolist() == ref.tolist()
