"""Ragged HF-decoder engine on the gfx950 kernels (bf16): flash prefill (>= 128 tokens, D=128),
paged decode, partial-rotary RoPE through the strided HIP kernel (Phi, D=64), exact-GELU bias-act
(Falcon), MoE with shared expert (Qwen2-MoE) -- against the transformers fp32 reference on CPU."""
import pytest
import torch

transformers = pytest.importorskip("transformers")
pytestmark = pytest.mark.gpu


def _model(name):
    T = transformers
    c = dict(vocab_size=256, num_hidden_layers=2, pad_token_id=0, bos_token_id=1, eos_token_id=2)
    if name == "llama":
        return T.LlamaForCausalLM(T.LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=2,
                                                num_key_value_heads=1, **c))
    if name == "phi":
        return T.PhiForCausalLM(T.PhiConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                                            partial_rotary_factor=0.5, **c))
    if name == "qwen2_moe":
        return T.Qwen2MoeForCausalLM(T.Qwen2MoeConfig(hidden_size=256, intermediate_size=512, num_attention_heads=2,
                                                      num_key_value_heads=2, num_experts=4, num_experts_per_tok=2,
                                                      moe_intermediate_size=128, shared_expert_intermediate_size=256,
                                                      **c))
    if name == "falcon":
        return T.FalconForCausalLM(T.FalconConfig(vocab_size=256, hidden_size=256, num_hidden_layers=2,
                                                  num_attention_heads=2))
    raise KeyError(name)


@pytest.mark.parametrize("name", ["llama", "phi", "qwen2_moe", "falcon"])
def test_hf_engine_gpu_matches_transformers(name):
    from shuffle_exchange_amd.inference.v2.engine_factory import build_hf_engine
    from shuffle_exchange_amd.inference.v2.engine_v2 import RaggedInferenceEngineConfig
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    torch.manual_seed(0)
    model = _model(name).eval()
    eng = build_hf_engine(model, RaggedInferenceEngineConfig(kv_block_size=64, num_kv_blocks=64),
                          dtype=torch.bfloat16, device="cuda")
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(3, 256, (n,), generator=g).tolist() for n in (200, 37)]
    out = eng.put([0, 1], prompts)
    for i, p in enumerate(prompts):
        with torch.no_grad():
            ref = model(torch.tensor([p])).logits[0, -1]
        rel = ((out[i].cpu() - ref).norm() / ref.norm()).item()
        assert rel < 3e-2, (name, i, rel)
    nxt = [int(out[0].argmax()), int(out[1].argmax())]
    out2 = eng.put([0, 1], [[nxt[0]], [nxt[1]]])
    for i, p in enumerate(prompts):
        with torch.no_grad():
            ref = model(torch.tensor([p + [nxt[i]]])).logits[0, -1]
        rel = ((out2[i].cpu() - ref).norm() / ref.norm()).item()
        assert rel < 3e-2, (name, "decode", i, rel)


@pytest.mark.parametrize("quant,tol", [("mxfp8", 0.16), ("mxfp6", 0.3), ("mxfp4", 0.6), ("int8", 0.06),
                                       ("int4", 0.6), ("fp6", 0.3)])
@pytest.mark.parametrize("name", ["llama", "qwen2_moe"])
def test_hf_engine_gpu_weight_quant(name, quant, tol):
    """Every inference weight format through the ragged engine on the GPU (prefill > 16 rows and
    single-token decode): OCP-MX weights on the block-scaled MFMA GEMM, int8/int4 on the mixed
    grouped kernel (experts included), FP6 bit planes -- logits stay within ~2x of the error the
    same formats show on the CPU path (random-init 256-wide models: mxfp8 0.08, mxfp6 0.15, mxfp4
    0.33, int8 0.02, int4 0.30, fp6 0.14 relative logit error vs fp32)."""
    from shuffle_exchange_amd.inference.v2.engine_factory import build_hf_engine
    from shuffle_exchange_amd.inference.v2.engine_v2 import RaggedInferenceEngineConfig
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    torch.manual_seed(0)
    model = _model(name).eval()
    eng = build_hf_engine(model, RaggedInferenceEngineConfig(kv_block_size=64, num_kv_blocks=64),
                          dtype=torch.bfloat16, device="cuda", weight_quant=quant)
    g = torch.Generator().manual_seed(3)
    prompt = torch.randint(3, 256, (150,), generator=g).tolist()
    out = eng.put([0], [prompt])
    with torch.no_grad():
        ref = model(torch.tensor([prompt])).logits[0, -1]
    assert ((out[0].cpu().float() - ref).norm() / ref.norm()).item() < tol
    nxt = int(out[0].argmax())
    out2 = eng.put([0], [[nxt]])
    with torch.no_grad():
        ref2 = model(torch.tensor([prompt + [nxt]])).logits[0, -1]
    assert ((out2[0].cpu().float() - ref2).norm() / ref2.norm()).item() < tol
