"""Inference engines on the CPU reference path: ragged v2 engine == full-sequence forward for
prefill, decode and chunked continuation (Llama and Mixtral), block accounting, scheduling
limits, init_inference + KV-cached generate == greedy full-recompute generate."""
import pytest
import torch


def _llama():
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.manual_seed(0)
    return LlamaForCausalLM(llama_config("llama-tiny", num_hidden_layers=2)).eval()


def _mixtral():
    from shuffle_exchange_amd.models import MixtralForCausalLM, mixtral_config
    torch.manual_seed(0)
    return MixtralForCausalLM(mixtral_config("mixtral-tiny", capacity_factor=64.0)).eval()  # dropless reference


@pytest.mark.parametrize("make", [_llama, _mixtral])
def test_ragged_engine_matches_full_forward(make):
    from shuffle_exchange_amd.inference.v2 import RaggedInferenceEngineConfig, build_engine
    m = make()
    eng = build_engine(m, RaggedInferenceEngineConfig(kv_block_size=8, num_kv_blocks=64))
    g = torch.Generator().manual_seed(1)
    hist = {1: torch.randint(0, 512, (13,), generator=g), 2: torch.randint(0, 512, (5,), generator=g),
            3: torch.randint(0, 512, (1,), generator=g)}
    lg = eng.put(list(hist), list(hist.values()))
    for step in range(3):
        new = {1: torch.randint(0, 512, (1,), generator=g), 2: torch.randint(0, 512, (4,), generator=g),
               3: torch.randint(0, 512, (9,), generator=g)}
        lg = eng.put(list(new), list(new.values()))
        for j, u in enumerate(new):
            hist[u] = torch.cat([hist[u], new[u]])
            with torch.no_grad():
                ref = m(hist[u][None])[0, -1].float()
            assert torch.allclose(lg[j], ref, atol=1e-4), (step, u, (lg[j] - ref).abs().max())
    used = eng.n_kv_blocks - eng.free_blocks
    assert used == sum((len(h) + 7) // 8 for h in hist.values())
    for u in hist:
        eng.flush(u)
    assert eng.free_blocks == eng.n_kv_blocks


def test_scheduling_limits():
    from shuffle_exchange_amd.inference.v2 import (RaggedInferenceEngineConfig, SchedulingError,
                                                   SchedulingResult, StateManagerConfig, build_engine)
    cfg = RaggedInferenceEngineConfig(kv_block_size=8, num_kv_blocks=4,
                                      state_manager=StateManagerConfig(max_ragged_batch_size=40,
                                                                       max_ragged_sequence_count=2))
    eng = build_engine(_llama(), cfg)
    assert eng.can_schedule([1], [33]) == SchedulingResult.KVCacheLimitExceeded
    assert eng.can_schedule([1, 2, 3], [1, 1, 1]) == SchedulingResult.BatchSequenceLimitExceeded
    assert eng.can_schedule([1], [41]) == SchedulingResult.BatchTokenLimitExceeded
    with pytest.raises(SchedulingError):
        eng.put([1], [torch.zeros(33, dtype=torch.long)])
    eng.put([1], [torch.zeros(10, dtype=torch.long)])
    assert eng.query(1, 100, 100) == (22, 2)  # 6 slots left in block 2 + 2 free blocks


def test_init_inference_generate_matches_recompute():
    import shuffle_exchange_amd as sxe
    m = _llama()
    eng = sxe.init_inference(m, dtype="fp32")
    prompt = torch.randint(0, 512, (2, 7), generator=torch.Generator().manual_seed(3))
    out = eng.generate(prompt, max_new_tokens=6)
    assert out.shape == (2, 13)
    ids = prompt.clone()
    for _ in range(6):
        with torch.no_grad():
            nxt = m(ids)[:, -1].argmax(-1, keepdim=True)
        ids = torch.cat([ids, nxt], dim=1)
    assert torch.equal(out.cpu(), ids)


def _case_v2_tp(rank, world, tp, nq, nkv):
    import torch
    from shuffle_exchange_amd.inference.v2 import RaggedInferenceEngineConfig, build_engine
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", num_attention_heads=nq, num_key_value_heads=nkv, hidden_size=128,
                       intermediate_size=256, vocab_size=301, num_hidden_layers=2)
    m = LlamaForCausalLM(cfg)
    eng = build_engine(m, RaggedInferenceEngineConfig(kv_block_size=8, num_kv_blocks=64,
                                                      tensor_parallel={"tp_size": tp}))
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, 301, (n,), generator=g) for n in (5, 11, 3)]
    first = eng.put([1, 2, 3], prompts)  # ragged prefill
    nxt = first.argmax(-1)
    second = eng.put([1, 2, 3], [t.view(1) for t in nxt])  # one decode step each
    gen = eng.generate([prompts[0].tolist()], max_new_tokens=4)
    return {"first": first, "second": second, "gen": gen, "kv_heads": eng.model.nkv}


@pytest.mark.parametrize("nq,nkv", [(4, 2), (4, 1)])
def test_v2_tensor_parallel_matches_tp1(nq, nkv):
    """InferenceEngineV2 with tensor_parallel.tp_size = 2 on gloo (reference llama_v2/model.py:156-191:
    all-reduce after o_proj / down_proj, all-gather of vocab-parallel logits; an odd vocab pads the
    last shard; kv heads replicated when tp exceeds them) == the tp = 1 engine: prefill + decode logits
    and greedy generation."""
    from .dist_utils import run_dist
    one = run_dist(_case_v2_tp, 1, 1, nq, nkv)[0]
    two = run_dist(_case_v2_tp, 2, 2, nq, nkv)
    for r in two:
        assert r["kv_heads"] == max(1, nkv // 2)
        assert torch.allclose(r["first"], one["first"], atol=1e-4), (r["first"] - one["first"]).abs().max()
        assert torch.allclose(r["second"], one["second"], atol=1e-4)
        assert r["gen"] == one["gen"]


def test_ragged_engine_rejects_positions_beyond_rope_table():
    """A sequence longer than the RoPE table raises instead of reading cos/sin out of bounds (the HIP
    RoPE kernels index the table unchecked)."""
    from shuffle_exchange_amd.inference.v2 import RaggedInferenceEngineConfig, build_engine
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=128, intermediate_size=256, num_attention_heads=4,
                       num_key_value_heads=2, vocab_size=100, num_hidden_layers=1, max_position_embeddings=64)
    eng = build_engine(LlamaForCausalLM(cfg).eval(), RaggedInferenceEngineConfig(kv_block_size=16, num_kv_blocks=16))
    eng.put([1], [torch.randint(0, 100, (60,))])
    with pytest.raises(ValueError, match="RoPE table"):
        eng.put([1], [torch.randint(0, 100, (10,))])
