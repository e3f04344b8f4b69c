"""engine.compile (DeepCompile counterpart): optimizer-state offload between steps leaves the
training trajectory unchanged; the HIP-graph forward (GPU) replays eval forwards exactly; the
schedule compiler (shuffle_exchange_amd/compile/) turns the traced ZeRO-3 step into a
ScheduleGraph whose passes -- selective_gather (keep groups resident within the memory budget:
fewer all-gathers per step), prefetch (gathers placed under the budget), offload_adam_states
(when the traced peak exceeds it) -- leave training numerics unchanged (gloo, world 2)."""
import pytest
import torch

from .dist_utils import run_dist


def _train(rank, world, compiled, stage):
    import shuffle_exchange_amd as sxe
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.GELU(), torch.nn.Linear(64, 8))
    cfg = {"train_micro_batch_size_per_gpu": 4, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
           "zero_optimization": {"stage": stage},
           "compile": {"deepcompile": True, "offload_opt_states": True, "double_buffer": False}}
    eng, _, _, _ = sxe.initialize(model=model, config=cfg)
    if compiled:
        eng.compile()
        assert eng.is_compiled
    g = torch.Generator().manual_seed(1)
    for _ in range(4):
        x = torch.randn(4, 16, generator=g)
        loss = eng(x).pow(2).mean()
        eng.backward(loss)
        eng.step()
    if compiled:
        st = [v for s in eng.optimizer.optimizer.state.values() for v in s.values()
              if torch.is_tensor(v) and v.numel() > 1]
        assert st and all(v.device.type == "cpu" for v in st)  # states parked on the host between steps
    return [p.detach().float().clone() for p in eng.module.parameters()]


@pytest.mark.parametrize("stage", [1, 3])
def test_compile_offload_opt_states_matches_eager(stage):
    a = run_dist(_train, 1, True, stage)[0]
    b = run_dist(_train, 1, False, stage)[0]
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y)


def _graph_eval(rank, world):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=256, intermediate_size=512, num_attention_heads=2,
                       num_key_value_heads=1, vocab_size=512, num_hidden_layers=2)
    model = LlamaForCausalLM(cfg)
    ds = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True}, "zero_optimization": {"stage": 1},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    eng.compile(backend="hipgraph")
    ids = torch.randint(0, 512, (2, 128), device="cuda")
    eng.eval()
    with torch.no_grad():
        ref = eng.module(ids).clone()
        out1 = eng(ids).clone()
        ids2 = torch.randint(0, 512, (2, 128), device="cuda")
        out2 = eng(ids2).clone()
        ref2 = eng.module(ids2)
    assert len(eng._fwd_graphs) == 1
    return [(out1 - ref).abs().max().item(), (out2 - ref2).abs().max().item()]


@pytest.mark.gpu
def test_compile_hipgraph_eval_forward():
    errs = run_dist(_graph_eval, 1)[0]
    assert max(errs) == 0.0, errs


def _case(rank, world, compile_cfg, steps=4):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd import comm as dist
    from ._dist_cases import full_params, global_batches, tiny_llama
    model, cfg = tiny_llama(0)
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 1,
          "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 0, "stage3_max_reuse_distance": 0},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    calls = {"n": 0}
    orig = dist.all_gather_into_tensor

    def counting(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)
    dist.all_gather_into_tensor = counting
    per_step, losses = [], []
    for i, b in enumerate(global_batches(cfg, world, 2, 16, steps)):
        if i == 1 and compile_cfg is not None:
            eng.compile(compile_kwargs=compile_cfg)
        c0 = calls["n"]
        local = b[rank * 2:(rank + 1) * 2]
        loss = eng(local, labels=local)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss))
        per_step.append(calls["n"] - c0)
    dist.all_gather_into_tensor = orig
    plan = getattr(eng, "compile_plan", None)
    out = {"losses": losses, "gathers": per_step, "params": {k: v for k, v in full_params(eng).items()}}
    if plan is not None:
        g = plan["graph"]
        out.update(keep=sorted(plan["keep"]), prefetch=plan["prefetch"], offload=plan["offload_opt_states"],
                   offload_act=plan["offload_activation"],
                   n_groups=len(g.gather_bytes), nodes=[(n.phase, n.fg) for n in g.nodes],
                   gather_bytes=dict(g.gather_bytes), budget=plan["budget"], peak=g.peak_bytes)
    return out


def test_schedule_compiler_keeps_groups_and_preserves_numerics():
    ref = run_dist(_case, 2, None)
    big = run_dist(_case, 2, {"deepcompile": True, "memory_budget": 1e12})
    for a, b in zip(ref, big):
        assert a["losses"] == b["losses"]
        for k in a["params"]:
            assert torch.equal(a["params"][k], b["params"][k]), k
    r0 = big[0]
    # a huge budget keeps every partitioned group: after compiling, a step only re-gathers the
    # kept groups once after the optimizer update (no forward / backward gathers)
    assert len(r0["keep"]) == r0["n_groups"] > 0
    assert r0["gathers"][-1] < ref[0]["gathers"][-1]
    assert ("fwd", r0["nodes"][0][1]) == r0["nodes"][0] and any(p == "bwd" for p, _ in r0["nodes"])
    assert r0["offload"] is False and r0["offload_act"] is False


def test_schedule_compiler_tight_budget_prefetch_and_offload():
    # budget below the traced peak: nothing kept, gathers still scheduled (at least one trigger
    # per remaining group), optimizer states offloaded; numerics unchanged
    ref = run_dist(_case, 2, None)
    tight = run_dist(_case, 2, {"deepcompile": True, "memory_budget": 1000})
    for a, b in zip(ref, tight):
        assert a["losses"] == b["losses"]
    r0 = tight[0]
    assert r0["keep"] == [] and r0["offload"] is True and r0["offload_act"] is True
    scheduled = [j for ph in ("fwd", "bwd") for lst in r0["prefetch"][ph].values() for j in lst]
    assert scheduled, r0["prefetch"]
    assert r0["gathers"][-1] == ref[0]["gathers"][-1]


def test_prefetch_pass_respects_budget_and_covers_gather_time():
    from shuffle_exchange_amd.compile.graph import Node, ScheduleGraph
    from shuffle_exchange_amd.compile.passes import prefetch, zero3_schedule
    nodes = [Node("fwd", i, 1.0, 0) for i in range(6)] + [Node("bwd", i, 2.0, 0) for i in reversed(range(6))]
    g = ScheduleGraph(nodes, {i: 100 for i in range(6)}, {i: 2.5 for i in range(6)}, peak_bytes=1000, device_bytes=0)
    plan = prefetch(g, zero3_schedule(g, {}, 0), budget=1000 + 250, slack=1.0)
    # forward: each gather needs 2.5 ms of cover = 3 nodes ahead, but only 2 x 100 B may be in
    # flight (250 B of headroom) -> issued 2 nodes ahead
    trig = {j: t for t, js in plan["prefetch"]["fwd"].items() for j in js}
    assert trig[5] == 3 and trig[4] == 2 and trig[3] == 1
    plan2 = prefetch(g, zero3_schedule(g, {}, 0), budget=1000 + 10_000, slack=1.0)
    trig2 = {j: t for t, js in plan2["prefetch"]["fwd"].items() for j in js}
    assert trig2[5] == 2 and trig2[4] == 1  # 3 nodes of 1 ms cover 2.5 ms


def test_compile_config_warns_on_no_effect_keys():
    """compile keys with no effect here (sync_*, symmetric_memory, keep_*) and unknown keys warn
    instead of being accepted silently."""
    from shuffle_exchange_amd.compile.config import CompileConfig
    c = CompileConfig.from_dict({"deepcompile": True, "symmetric_memory": True, "sync_after_reduce": True,
                                 "keep_all_input_tensors": True, "bogus_key": 1})
    assert set(c.ignored) == {"symmetric_memory", "sync_after_reduce", "keep_all_input_tensors", "bogus_key"}
    assert CompileConfig.from_dict({"deepcompile": True, "keep_int_input_tensors": True}).ignored == []
