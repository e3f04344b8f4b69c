"""InferenceEngineV2.serialize -> build_engine_from_ds_checkpoint round trips (reference
inference/v2/engine_v2.py:251, engine_factory.py:32-66): per-TP-rank parameter files + metadata,
rebuilt without the original model, give identical logits and generations -- for a Hugging Face
decoder (TP 1 and TP 2, bf16 and fp8 weight-only quantization) and the framework's own Llama."""
import pytest
import torch

from .dist_utils import run_dist

transformers = pytest.importorskip("transformers")


def _prompts():
    g = torch.Generator().manual_seed(1)
    return [torch.randint(3, 96, (n,), generator=g).tolist() for n in (7, 11, 3)]


def _run(eng):
    first = eng.put([0, 1, 2], _prompts())
    for u in (0, 1, 2):
        eng.flush(u)
    gen = eng.generate([_prompts()[1]], max_new_tokens=4)
    return first, gen


def _case(rank, world, tmp, quant, kind):
    from shuffle_exchange_amd.inference.v2 import RaggedInferenceEngineConfig, build_engine, build_hf_engine
    from shuffle_exchange_amd.inference.v2.engine_factory import build_engine_from_ds_checkpoint
    torch.manual_seed(0)
    cfg = RaggedInferenceEngineConfig(kv_block_size=4, num_kv_blocks=64, tensor_parallel={"tp_size": world})
    if kind == "hf":
        from tests.test_hf_inference import _tiny
        eng = build_hf_engine(_tiny("llama").eval(), cfg, dtype=torch.float32, weight_quant=quant)
    else:
        from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
        cfg.weight_quant = quant
        eng = build_engine(LlamaForCausalLM(llama_config("llama-tiny", vocab_size=96)).eval(), cfg)
    first, gen = _run(eng)
    eng.serialize(tmp)
    import torch.distributed as td
    if td.is_initialized():
        td.barrier()
    del eng
    eng2 = build_engine_from_ds_checkpoint(tmp, RaggedInferenceEngineConfig(kv_block_size=4, num_kv_blocks=64))
    first2, gen2 = _run(eng2)
    return {"first": first, "gen": gen, "first2": first2, "gen2": gen2}


@pytest.mark.parametrize("world,quant,kind", [(1, None, "hf"), (2, None, "hf"), (1, "fp8", "hf"),
                                              (1, None, "native"), (2, None, "native")])
def test_serialize_round_trip(tmp_path, world, quant, kind):
    res = run_dist(_case, world, str(tmp_path), quant, kind)
    for r in res:
        assert torch.equal(r["first"], r["first2"])
        assert r["gen"] == r["gen2"]
    files = sorted(p.name for p in tmp_path.iterdir())
    assert "ds_model_config.json" in files
    for rk in range(world):
        assert f"params_rank_{rk}.pt" in files and f"metadata_rank_{rk}.json" in files
    # the parameter files hold plain tensors only
    sd = torch.load(tmp_path / "params_rank_0.pt", weights_only=True)
    assert all(torch.is_tensor(v) for v in sd.values())
