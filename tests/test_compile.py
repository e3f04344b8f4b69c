"""engine.compile (DeepCompile counterpart): optimizer-state offload between steps leaves the
training trajectory unchanged; the HIP-graph forward (GPU) replays eval forwards exactly."""
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
