"""DeepCompile FX graph compiler for ZeRO 0/1/2 (compile/fx_backend.py, compile/fx_graph.py;
reference compile/backend.py:217, compile/init_z1.py:18, compile/passes/zero1_compile.py).

Dynamo + AOT autograd graphs whose backward hands every parameter gradient to the ZeRO buckets by
an in-graph ``sxe_dc.reduce_grad`` node placed right after the gradient's producer. The compiled
engine must follow the eager engine's trajectory (gloo, world 2, with gradient accumulation), the
backward graph must hold one reduce per parameter, and those reduces must be spread through the
backward (the first gradient leaves long before the graph ends)."""
import pytest
import torch

from .dist_utils import run_dist


def _train(rank, world, compiled, stage, gas, model_kind):
    import shuffle_exchange_amd as sxe
    torch.manual_seed(0)
    if model_kind == "llama":
        from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
        cfg = llama_config("llama-tiny", hidden_size=64, intermediate_size=128, num_attention_heads=4,
                           num_key_value_heads=2, vocab_size=128, num_hidden_layers=2)
        model = LlamaForCausalLM(cfg)
    else:
        model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.GELU(), torch.nn.Linear(64, 64),
                                    torch.nn.GELU(), torch.nn.Linear(64, 8))
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": gas,
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
          "zero_optimization": {"stage": stage, "reduce_bucket_size": 2000,
                                "stage3_param_persistence_threshold": 0},
          "compile": {"deepcompile": True, "fx_zero3": True}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    if compiled:
        eng.compile()
    g = torch.Generator().manual_seed(1 + rank)
    losses = []
    for _ in range(3 * gas):
        if model_kind == "llama":
            ids = torch.randint(0, 128, (2, 16), generator=g)
            loss = eng(ids, labels=ids)
        else:
            loss = eng(torch.randn(2, 16, generator=g)).pow(2).mean()
        eng.backward(loss)
        eng.step()
        losses.append(float(loss))
    # ZeRO-3 parameters are partitioned (in graph mode a released parameter keeps its shape over freed
    # storage): read them consolidated
    out = {"params": [] if stage == 3 else [p.detach().float().clone() for p in eng.module.parameters()],
           "losses": losses}
    if compiled:
        fx = eng.compile_plan["fx"]
        out["reduced"] = fx.reduced
        out["graphs"] = {k: {kk: v[kk] for kk in ("params", "reduces", "order")} for k, v in fx.graphs.items()}
        out["profiled"] = all("bwd" in v["profile"] and v["profile"]["bwd"]["nodes"] > 0 for v in fx.graphs.values())
        if stage == 3:
            out["z3"] = {k: {kk: v.get(kk) for kk in ("fw", "bw", "reduces", "params")} for k, v in fx.graphs.items()}
            out["stats"] = dict(fx.stats)
    if stage == 3:
        from shuffle_exchange_amd.runtime.zero.stage3 import RELEASED
        released = [p for us in eng.optimizer.units for u in us if u.state == RELEASED for p in u.params]
        # between steps a released parameter reads as an empty tensor (eager ZeRO-3 semantics), in
        # graph mode too -- never as a full-shape view of freed storage
        out["released_numels"] = sorted({p.numel() for p in released})
        out["params"] = [v for _, v in sorted(eng._zero3_consolidated_16bit_state_dict().items())
                         if v.dtype.is_floating_point]
        if compiled:  # and the next compiled step still runs (relinked before the forward)
            x = torch.randint(0, 128, (2, 16), generator=g) if model_kind == "llama" else torch.randn(2, 16, generator=g)
            loss = eng(x, labels=x) if model_kind == "llama" else eng(x).pow(2).mean()
            eng.backward(loss)
            eng.step()
            out["after_extra_step"] = sorted({p.numel() for p in released})
    return out


@pytest.mark.parametrize("stage,gas", [(0, 1), (1, 2), (2, 2)])
def test_fx_compiled_matches_eager_mlp(stage, gas):
    comp = run_dist(_train, 2, True, stage, gas, "mlp")
    eager = run_dist(_train, 2, False, stage, gas, "mlp")
    for c, e in zip(comp, eager):
        for x, y in zip(c["params"], e["params"]):
            torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)
        n_params = 6
        assert c["reduced"] == n_params * 3 * gas  # every gradient of every micro-step went through the graph
        (gr,) = c["graphs"].values()
        assert gr["params"] == n_params and gr["reduces"] == n_params
        pos, length = gr["order"]
        assert min(pos) < length // 2  # the first gradient leaves early in the backward
        assert c["profiled"]
    assert comp[0]["params"][0].equal(comp[1]["params"][0])  # replicas agree


def test_fx_compiled_matches_eager_llama_zero2():
    comp = run_dist(_train, 2, True, 2, 1, "llama")
    eager = run_dist(_train, 2, False, 2, 1, "llama")
    for c, e in zip(comp, eager):
        assert c["losses"] == pytest.approx(e["losses"], rel=1e-4, abs=1e-5)
        for x, y in zip(c["params"], e["params"]):
            torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5)
        assert sum(g["reduces"] for g in c["graphs"].values()) >= len(c["params"])


@pytest.mark.gpu
@pytest.mark.parametrize("stage", [1, 3])
def test_fx_compiled_llama_gpu_matches_eager(stage):
    """bf16 Llama (4 layers) on the HIP kernels (traced through their fake kernels,
    ops/fake_kernels.py): the compiled ZeRO-1 / ZeRO-3 engine reproduces the eager losses, and the
    model traces without a graph break (a break inside the repeated decoder layer would split the
    model into per-layer frames)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from torch._dynamo.utils import counters

    def run(compiled):
        import shuffle_exchange_amd as sxe
        from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
        torch.manual_seed(0)
        cfg = llama_config("llama-tiny", hidden_size=256, intermediate_size=512, num_attention_heads=4,
                           num_key_value_heads=2, vocab_size=1024, num_hidden_layers=4)
        model = LlamaForCausalLM(cfg).to(torch.bfloat16)
        z = {"stage": stage}
        if stage == 3:
            z["stage3_param_persistence_threshold"] = 0
        ds = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True}, "zero_optimization": z,
              "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "compile": {"deepcompile": True, "fx_zero3": True}}
        eng, _, _, _ = sxe.initialize(model=model, config=ds)
        if compiled:
            eng.compile()
        g = torch.Generator(device="cuda").manual_seed(1)
        ids = torch.randint(0, 1024, (2, 256), device="cuda", generator=g)
        losses = []
        for _ in range(4):  # the same batch: the loss falls fast, so a missed update shows
            loss = eng(ids, labels=ids)
            eng.backward(loss)
            eng.step()
            losses.append(float(loss))
        n = eng.compile_plan["fx"].reduced if compiled else 0
        torch._dynamo.reset()
        return losses, n

    counters.clear()
    c, n = run(True)
    breaks = dict(counters["graph_break"])
    e, _ = run(False)
    assert n > 0
    assert not breaks, breaks
    assert c == pytest.approx(e, rel=2e-3)


def _train_se(rank, world, compiled, method):
    import shuffle_exchange_amd as sxe
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.GELU(), torch.nn.Linear(64, 8))
    ds = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
          "zero_optimization": {"stage": 2}, "compile": {"deepcompile": True}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds, method=method, slice_count=2, rings=2, shuffle_step=1)
    if compiled:
        eng.compile()
    g = torch.Generator().manual_seed(7 + rank)
    for _ in range(4):
        loss = eng(torch.randn(2, 16, generator=g)).pow(2).mean()
        eng.backward(loss)
        eng.step()
        eng.shuffle_exchange()
    return [p.detach().float().clone() for p in eng.module.parameters()]


@pytest.mark.parametrize("method", ["RR", "shuffle"])
def test_fx_compiled_shuffle_exchange_matches_eager(method):
    """The fork's Shuffle-exchange ZeRO-2 (slice_count 2 over 4 ranks) under the FX compiler: the
    in-graph reduces feed the slice-group reduce-scatter and the inter-slice averaging unchanged."""
    comp = run_dist(_train_se, 4, True, method)
    eager = run_dist(_train_se, 4, False, method)
    for c, e in zip(comp, eager):
        for x, y in zip(c, e):
            torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("model_kind,gas", [("mlp", 1), ("llama", 1), ("llama", 2)])
def test_fx_zero3_graph_compiler_matches_eager(model_kind, gas):
    """ZeRO-3 under the graph compiler (compile/fx_zero3.py): gather / prefetch / release nodes in
    the forward and backward FX graphs and the reduce-scatters fed by in-graph reduce nodes; the
    trajectory equals the eager ZeRO-3 engine's (gloo, world 2), with and without gradient
    accumulation."""
    comp = run_dist(_train, 2, True, 3, gas, model_kind)
    eager = run_dist(_train, 2, False, 3, gas, model_kind)
    for c, e in zip(comp, eager):
        assert c["losses"] == pytest.approx(e["losses"], rel=1e-4, abs=1e-5)
        for x, y in zip(c["params"], e["params"]):
            torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5)
        fw = sum(v["fw"]["fetch"] for v in c["z3"].values() if v.get("fw"))
        bw = sum(v["bw"]["fetch"] for v in c["z3"].values() if v.get("bw"))
        assert fw > 0 and bw > 0, c["z3"]
        assert sum(v["reduces"] for v in c["z3"].values()) >= 1
        assert c["stats"]["fetch"] > 0 and c["stats"]["release"] > 0
        assert c["released_numels"] == [0] and e["released_numels"] == [0], (c["released_numels"], e["released_numels"])
        assert c["after_extra_step"] == [0]


class _BreakingBlock(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(8, 8)

    def forward(self, x):
        x = self.lin(x)
        torch._dynamo.graph_break()
        return torch.relu(x)


def _train_breaks(rank, world, compiled, stage):
    import shuffle_exchange_amd as sxe
    torch.manual_seed(0)
    model = torch.nn.Sequential(_BreakingBlock(), _BreakingBlock(), _BreakingBlock(), torch.nn.Linear(8, 2))
    ds = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
          "zero_optimization": {"stage": stage, "stage3_param_persistence_threshold": 0},
          "compile": {"deepcompile": True, "fx_zero3": True}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    if compiled:
        eng.compile()
    g = torch.Generator().manual_seed(3 + rank)
    for _ in range(3):
        loss = eng(torch.randn(2, 8, generator=g)).sum()
        eng.backward(loss)
        eng.step()
    torch._dynamo.reset()
    if stage == 3:
        return [v for _, v in sorted(eng._zero3_consolidated_16bit_state_dict().items())]
    return [p.detach().clone() for p in eng.module.parameters()]


def test_fx_graph_break_in_repeated_module():
    """A graph break inside a repeated block makes Dynamo compile the block's frame once and run it
    for every instance with that instance's parameters as inputs; the in-graph reduce nodes are
    bound to parameter identities, so the compiler builds one graph per parameter set
    (compile/fx_backend.py ``ParamBoundGraph``) and the ZeRO-1 trajectory still equals eager."""
    comp = run_dist(_train_breaks, 2, True, 1)
    eager = run_dist(_train_breaks, 2, False, 1)
    for c, e in zip(comp, eager):
        for x, y in zip(c, e):
            torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


def test_fx_zero3_graph_break_is_loud():
    """ZeRO-3 graph mode has no module hooks: a module that a graph break leaves to eager execution
    would read a released parameter. The compiler traces with fullgraph=True, so the step fails at
    the break with Dynamo's own message."""
    with pytest.raises(RuntimeError, match="graph_break|Unsupported|graph break"):
        run_dist(_train_breaks, 2, True, 3)


def test_native_dispatch_predicates_trace_without_break():
    """The extension loader is lock-free once the load is decided: the dispatch predicates
    (``native.use_hip`` & co.) run inside compiled regions, and a lock there is a graph break."""
    from shuffle_exchange_amd.ops import native
    avail = native.cpu_available()
    f = torch.compile(lambda x: x + 1 if native.cpu_available() else x - 1, fullgraph=True, backend="eager")
    assert f(torch.zeros(2)).tolist() == ([1.0, 1.0] if avail else [-1.0, -1.0])
