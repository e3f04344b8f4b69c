"""Inference-v2 module registry / heuristics: implementation selection by config, pinning, and the
ragged Llama model routing its attention / embedding / linear / MoE choices through it."""
import pytest
import torch


def test_registry_selection_and_pins():
    from shuffle_exchange_amd.inference.v2.modules import REGISTRIES, instantiate_attention, instantiate_linear
    from shuffle_exchange_amd.inference.v2.modules.implementations import AttentionConfig, LinearConfig
    assert {"quantized_weight_only", "blas_fp_linear"} <= set(REGISTRIES["linear"].names())
    w = torch.randn(32, 128)
    lin = instantiate_linear(LinearConfig(128, 32, torch.float32, None, "cpu"), w)
    assert lin.impl_name == "blas_fp_linear"
    x = torch.randn(3, 128)
    torch.testing.assert_close(lin(x), x @ w.t())
    q = instantiate_linear(LinearConfig(128, 32, torch.float32, "fp6", "cpu"), w)
    assert q.impl_name == "quantized_weight_only"
    assert torch.nn.functional.cosine_similarity(q(x).flatten(), (x @ w.t()).flatten(), dim=0) > 0.98
    # CPU: no flash prefill; an explicit pin of an unsupported implementation is an error
    a = instantiate_attention(AttentionConfig(128, 8, 2, torch.bfloat16, 0, "cpu"))
    assert a.impl_name == "dense_blocked_attention"
    with pytest.raises(ValueError):
        instantiate_attention(AttentionConfig(128, 8, 2, torch.bfloat16, 0, "cpu"),
                              pins={"attention": "dense_blocked_attention_flash_prefill"})


def test_ragged_llama_uses_registry():
    from shuffle_exchange_amd.inference.v2 import RaggedInferenceEngineConfig, build_engine
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.manual_seed(0)
    m = LlamaForCausalLM(llama_config("llama-tiny", num_hidden_layers=2, hidden_size=128, intermediate_size=256))
    e = build_engine(m, RaggedInferenceEngineConfig(num_kv_blocks=64, weight_quant="fp6"))
    impl = e._model.implementations
    assert impl["linear"] == "quantized_weight_only" and impl["embed"] == "ragged_embedding"
    ref = build_engine(m, RaggedInferenceEngineConfig(num_kv_blocks=64))
    assert ref._model.implementations["linear"] == "module"
    p = torch.randint(0, 512, (12,)).tolist()
    a, b = e.put([0], [p]), ref.put([0], [p])
    assert torch.nn.functional.cosine_similarity(a.float(), b.float()).item() > 0.97
