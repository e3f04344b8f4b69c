"""Ragged inference on the MI355X: the engine (flash prefill + paged decode + chunked continuation
through the HIP kernels, bf16) agrees with the model's own full-sequence forward."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _native():
    from shuffle_exchange_amd.ops import native
    native.require_hip()


def _model():
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=512, intermediate_size=1024, num_attention_heads=4,
                       num_key_value_heads=2, vocab_size=2048, num_hidden_layers=2, max_position_embeddings=4096)
    return LlamaForCausalLM(cfg).to("cuda", torch.bfloat16).eval()


def _cos(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return float(a @ b / (a.norm() * b.norm()))


def test_ragged_engine_gpu_matches_forward():
    from shuffle_exchange_amd.inference.v2 import RaggedInferenceEngineConfig, build_engine
    m = _model()
    eng = build_engine(m, RaggedInferenceEngineConfig(kv_block_size=64, num_kv_blocks=256))
    g = torch.Generator().manual_seed(1)
    hist = {1: torch.randint(0, 2048, (300,), generator=g),   # flash prefill (>=128, no history)
            2: torch.randint(0, 2048, (37,), generator=g),    # paged prefill
            3: torch.randint(0, 2048, (128,), generator=g)}
    lg = eng.put(list(hist), list(hist.values()))
    for j, u in enumerate(hist):
        with torch.no_grad():
            ref = m(hist[u][None].cuda())[0, -1].float()
        assert _cos(lg[j], ref) > 0.999
    for step in range(3):
        new = {1: torch.randint(0, 2048, (1,), generator=g), 2: torch.randint(0, 2048, (5,), generator=g),
               3: torch.randint(0, 2048, (130,), generator=g)}  # chunked continuation with history
        lg = eng.put(list(new), list(new.values()))
        for j, u in enumerate(new):
            hist[u] = torch.cat([hist[u], new[u]])
            with torch.no_grad():
                ref = m(hist[u][None].cuda())[0, -1].float()
            assert _cos(lg[j], ref) > 0.999, (step, u)


def test_generate_gpu():
    import shuffle_exchange_amd as sxe
    m = _model()
    eng = sxe.init_inference(m, dtype="bf16")
    prompt = torch.randint(0, 2048, (3, 16), generator=torch.Generator().manual_seed(2)).cuda()
    out = eng.generate(prompt, max_new_tokens=8)
    assert out.shape == (3, 24)
    assert torch.equal(out[:, :16], prompt)
