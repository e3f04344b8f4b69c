"""AutoTP tensor parallelism on gloo: shard/unshard round trips (GQA-packed qkv, packed gate|up),
and TP (x DP) training == single-process training of the full model (Llama and GPT-2)."""
import pytest
import torch

from .dist_utils import run_dist


def test_shard_unshard_roundtrip():
    from shuffle_exchange_amd.module_inject.layers import shard_rows, unshard_rows
    w = torch.randn((8 + 2 * 4) * 16, 32)
    for layout in (None, ("chunks", 2), ("heads", [8, 4, 4], 16)):
        for tp in (1, 2, 4):
            parts = [shard_rows(w, layout, tp, r) for r in range(tp)]
            assert torch.equal(unshard_rows(parts, layout), w)
    # heads layout keeps whole heads together: rank 0 gets q heads 0..3, k heads 0..1, v heads 0..1
    p0 = shard_rows(w, ("heads", [8, 4, 4], 16), 2, 0)
    assert torch.equal(p0[:64], w[:64]) and torch.equal(p0[64:96], w[128:160])


def test_tp_parser_llama():
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    from shuffle_exchange_amd.module_inject.auto_tp import AutoTP
    m = LlamaForCausalLM(llama_config("llama-tiny"))
    plan = dict(AutoTP(m, None, tp_size=2).tp_parser())
    assert plan["layers.0.self_attn.qkv_proj"] == "col" and plan["layers.0.self_attn.o_proj"] == "row"
    assert plan["layers.0.mlp.gate_up_proj"] == "col" and plan["layers.0.mlp.down_proj"] == "row"
    assert not any("lm_head" in k or "embed" in k for k in plan)


def _model(kind):
    torch.manual_seed(0)
    if kind == "llama":
        from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
        cfg = llama_config("llama-tiny", num_attention_heads=4, num_key_value_heads=2)
        return LlamaForCausalLM(cfg), cfg.vocab_size
    from shuffle_exchange_amd.models import GPT2LMHeadModel, gpt2_config
    cfg = gpt2_config("gpt2-tiny")
    return GPT2LMHeadModel(cfg), cfg.vocab_size


def _case_tp(rank, world, kind, tp, stage, steps):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.module_inject.auto_tp import gather_tp_state_dict
    from shuffle_exchange_amd.parallel import groups
    model, V = _model(kind)
    ds = {"train_micro_batch_size_per_gpu": 2, "tensor_parallel": {"autotp_size": tp},
          "zero_optimization": {"stage": stage}, "gradient_clipping": 1.0,
          "optimizer": {"type": "SGD", "params": {"lr": 0.2}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    dp, dpr = groups.get_data_parallel_world_size(), groups.get_data_parallel_rank()
    g = torch.Generator().manual_seed(3)
    losses = []
    for _ in range(steps):
        b = torch.randint(0, V, (dp * 2, 16), generator=g)
        local = b[dpr * 2:(dpr + 1) * 2]
        loss = eng(local, labels=local)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    sd = gather_tp_state_dict(eng.module) if stage < 3 else None
    return {"losses": losses, "sd": sd, "norm": eng.get_global_grad_norm()}


def _reference(kind, world, tp, steps):
    model, V = _model(kind)
    dp = world // tp
    opt = torch.optim.SGD(model.parameters(), lr=0.2)
    g = torch.Generator().manual_seed(3)
    losses, norm = [], None
    for _ in range(steps):
        b = torch.randint(0, V, (dp * 2, 16), generator=g)
        loss = model(b, labels=b)
        opt.zero_grad()
        loss.backward()
        norm = float(torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0))
        opt.step()
    return model.state_dict(), norm


@pytest.mark.parametrize("kind,world,tp,stage", [("llama", 2, 2, 1), ("gpt2", 2, 2, 2), ("llama", 4, 2, 2),
                                                 ("llama", 2, 2, 0)])
def test_autotp_training_matches_single_process(kind, world, tp, stage):
    res = run_dist(_case_tp, world, kind, tp, stage, 3)
    ref_sd, ref_norm = _reference(kind, world, tp, 3)
    for r in res:
        assert r["norm"] == pytest.approx(ref_norm, rel=1e-3)
        for k, v in ref_sd.items():
            got = r["sd"][k].float()
            d = (got - v.float()).abs().max().item()
            assert d <= 1e-4 * max(1.0, v.abs().max().item()), f"{k}: {d}"


def test_autotp_zero3_trains():
    res = run_dist(_case_tp, 2, "llama", 2, 3, 3)
    ref = run_dist(_case_tp, 2, "llama", 2, 1, 3)
    for a, b in zip(res[0]["losses"], ref[0]["losses"]):
        assert a == pytest.approx(b, rel=1e-4)


def _case_tp_save(rank, world, path):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.module_inject.auto_tp import gather_tp_state_dict
    model, V = _model("llama")
    ds = {"train_micro_batch_size_per_gpu": 2, "tensor_parallel": {"autotp_size": 2},
          "zero_optimization": {"stage": 1}, "optimizer": {"type": "SGD", "params": {"lr": 0.2}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    b = torch.randint(0, V, (2, 16), generator=torch.Generator().manual_seed(3))
    loss = eng(b, labels=b)
    eng.backward(loss)
    eng.step()
    eng.save_checkpoint(path, tag="t")
    return {k: v.cpu() for k, v in gather_tp_state_dict(eng.module).items()}


def test_tp_checkpoint_reshape(tmp_path):
    """AutoTP TP=2 checkpoint -> TP=1 (full weights equal the gathered TP model, incl. the packed
    GQA q|k|v and gate|up layouts) -> TP=2 again (shards equal the original files)."""
    from shuffle_exchange_amd.checkpoint.reshape import inspect_checkpoint, reshape_checkpoint, tp_full_state_dict
    full = run_dist(_case_tp_save, 2, str(tmp_path / "tp2"))[0]
    info = inspect_checkpoint(str(tmp_path / "tp2"))
    assert info.tp_degree == 2 and len(info.model_files) == 2
    sd1 = tp_full_state_dict(str(tmp_path / "tp2"))
    for k, v in full.items():
        assert torch.equal(sd1[k], v), k
    model, _ = _model("llama")
    model.load_state_dict(sd1)  # a plain single-GPU model loads the reshaped weights
    reshape_checkpoint(str(tmp_path / "tp2"), str(tmp_path / "tp1"), new_tp=1)
    reshape_checkpoint(str(tmp_path / "tp1"), str(tmp_path / "tp2b"), new_tp=2)
    for r in range(2):
        a = torch.load(tmp_path / "tp2" / "t" / f"mp_rank_{r:02d}_model_states.pt", weights_only=True)["module"]
        b = torch.load(tmp_path / "tp2b" / "t" / f"mp_rank_{r:02d}_model_states.pt", weights_only=True)["module"]
        assert a.keys() == b.keys()
        for k in a:
            assert torch.equal(a[k], b[k]), k
