"""Kernel-injected inference under tensor parallelism and checkpoint loading (gloo, CPU).

Reference: module_inject/replace_module.py:207-231 (the injected containers' q|k|v heads and MLP
columns sliced per rank, attention-out / MLP-out all-reduced), :418-473 and inference/engine.py:411-468
(checkpoint lists / JSON descriptors via runtime/state_dict_factory.py:21 ``SDLoaderFactory``, MP
merge / split). TP=2 injected logits and greedy generation equal the TP=1 injected model's; a
checkpoint saved as 2 MP shards loads into TP=1 and TP=2 engines; a misnamed key raises."""
import json
import os

import pytest
import torch

from .dist_utils import run_dist

transformers = pytest.importorskip("transformers")

ARCHS = ["llama", "gpt2", "opt", "gptj", "bloom", "gptneo", "neox"]


def _model(arch):
    torch.manual_seed(0)
    if arch == "gpt2":
        cfg = transformers.GPT2Config(vocab_size=300, n_positions=64, n_embd=64, n_layer=2, n_head=4)
        return transformers.GPT2LMHeadModel(cfg).eval()
    if arch == "neox":
        cfg = transformers.GPTNeoXConfig(vocab_size=300, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                                         intermediate_size=128, max_position_embeddings=64, rotary_pct=0.5)
        return transformers.GPTNeoXForCausalLM(cfg).eval()
    from tests.test_kernel_inject import _decoder
    return _decoder(arch)


def _case(rank, world, arch, tp, ckpt=None):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.module_inject import replace_module as rm
    model = _model(arch)
    kw = {"checkpoint": ckpt} if ckpt is not None else {}
    if ckpt is not None:  # weights come from the checkpoint, not from the seed
        with torch.no_grad():
            for p in model.parameters():
                p.add_(1.0)
    eng = sxe.init_inference(model, dtype=torch.float32, replace_with_kernel_inject=True, tensor_parallel={"tp_size": tp},
                             **kw)
    fused = [m for m in model.modules() if isinstance(m, rm._Fused)]
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(3, 300, (2, 10), generator=g)
    with torch.no_grad():
        logits = eng(ids, use_cache=False).logits
    gen = eng.generate(ids[:1], max_new_tokens=5)
    return {"logits": logits, "gen": gen, "n_fused": len(fused), "sharded": eng.tp_sharded_layers,
            "tp": [m._tp[1] if m._tp else 1 for m in fused]}


@pytest.mark.parametrize("arch", ARCHS)
def test_injected_tp2_matches_tp1(arch):
    one = run_dist(_case, 1, arch, 1)[0]
    two = run_dist(_case, 2, arch, 2)
    assert one["n_fused"] == 2
    for r in two:
        assert r["sharded"] == 2 and r["tp"] == [2, 2]
        d = (r["logits"] - one["logits"]).abs().max().item()
        assert d < 1e-4 * max(1.0, one["logits"].abs().max().item()), (arch, d)
        assert torch.equal(r["gen"], one["gen"]), arch


def _write_mp_shards(tmp, arch, n=2):
    """The model's weights as ``n`` MP shards: linear weights split along their output rows, the
    rest replicated (no tp_partitions metadata: the loader matches shapes against the model)."""
    model = _model(arch)
    sd = model.state_dict()
    d = os.path.join(tmp, "global_step7")
    os.makedirs(d, exist_ok=True)
    for r in range(n):
        shard = {}
        for k, v in sd.items():
            if v.dim() == 2 and k.endswith("weight") and v.shape[0] % n == 0 and "embed" not in k and "wte" not in k \
                    and "wpe" not in k:
                c = v.shape[0] // n
                shard[k] = v[r * c:(r + 1) * c].clone()
            else:
                shard[k] = v.clone()
        torch.save({"module": shard, "mp_world_size": n}, os.path.join(d, f"mp_rank_{r:02d}_model_states.pt"))
    with open(os.path.join(tmp, "latest"), "w") as f:
        f.write("global_step7")
    desc = {"type": "ds_model", "version": 1.0, "mp_size": n,
            "checkpoints": [f"global_step7/mp_rank_{r:02d}_model_states.pt" for r in range(n)]}
    with open(os.path.join(tmp, "ckpt.json"), "w") as f:
        json.dump(desc, f)
    return model


@pytest.mark.parametrize("source", ["dir", "json"])
def test_checkpoint_mp_merge_and_split(tmp_path, source):
    arch = "llama"
    _write_mp_shards(str(tmp_path), arch)
    src = str(tmp_path) if source == "dir" else str(tmp_path / "ckpt.json")
    ref = run_dist(_case, 1, arch, 1)[0]  # the seed's weights == the checkpoint's
    one = run_dist(_case, 1, arch, 1, src)[0]  # 2 shards merged into TP 1
    two = run_dist(_case, 2, arch, 2, src)  # merged, then split to TP 2
    assert torch.allclose(one["logits"], ref["logits"], atol=1e-5)
    for r in two:
        assert torch.allclose(r["logits"], ref["logits"], atol=1e-4)
        assert torch.equal(r["gen"], ref["gen"])


def test_checkpoint_misnamed_key_raises(tmp_path):
    import shuffle_exchange_amd as sxe
    model = _model("gpt2")
    sd = model.state_dict()
    k = next(k for k in sd if k.endswith("mlp.c_fc.weight"))
    sd[k.replace("c_fc", "c_fcx")] = sd.pop(k)
    path = str(tmp_path / "bad.pt")
    torch.save(sd, path)
    with pytest.raises(KeyError) as e:
        sxe.init_inference(_model("gpt2"), dtype=torch.float32, checkpoint=path)
    assert "c_fcx" in str(e.value) and "missing" in str(e.value)
    eng = sxe.init_inference(_model("gpt2"), dtype=torch.float32, checkpoint=path, load_strict=False)
    assert eng is not None


def test_sdloader_factory_json(tmp_path):
    from shuffle_exchange_amd.runtime.state_dict_factory import SDLoaderFactory
    model = _write_mp_shards(str(tmp_path), "gpt2")
    loader = SDLoaderFactory.get_sd_loader_json(str(tmp_path / "ckpt.json"))
    path, sd0 = loader.load(2, 0)
    assert path.endswith("mp_rank_00_model_states.pt")
    _, full = loader.load(1, 0, model=model)
    for k, v in model.state_dict().items():
        assert torch.equal(full[k], v), k
