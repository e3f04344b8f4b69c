"""Domino (overlapped TP) on gloo: the two-micro-batch schedule with async forward all-reduces and
parked backward input-grad all-reduces trains exactly like plain AutoTP."""
import pytest
import torch

from .dist_utils import run_dist


def _case(rank, world, domino, steps):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    from shuffle_exchange_amd.module_inject.auto_tp import gather_tp_state_dict
    from shuffle_exchange_amd.runtime.domino import DominoLlamaDecoderLayer, apply_domino
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", num_attention_heads=4, num_key_value_heads=2)
    model = LlamaForCausalLM(cfg)
    ds = {"train_micro_batch_size_per_gpu": 4, "tensor_parallel": {"autotp_size": world},
          "zero_optimization": {"stage": 1}, "optimizer": {"type": "SGD", "params": {"lr": 0.2}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    if domino:
        apply_domino(eng.module)
        assert all(type(layer) is DominoLlamaDecoderLayer for layer in eng.module.layers)
    g = torch.Generator().manual_seed(3)
    losses = []
    for _ in range(steps):
        b = torch.randint(0, cfg.vocab_size, (4, 16), generator=g)
        loss = eng(b, labels=b)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    if domino:
        assert DominoLlamaDecoderLayer.overlapped_calls == steps * cfg.num_hidden_layers
    return {"losses": losses, "sd": gather_tp_state_dict(eng.module)}


def test_domino_matches_autotp():
    dom = run_dist(_case, 2, True, 3)
    ref = run_dist(_case, 2, False, 3)
    for a, b in zip(dom[0]["losses"], ref[0]["losses"]):
        assert a == pytest.approx(b, rel=1e-5)
    for k, v in ref[0]["sd"].items():
        d = (dom[0]["sd"][k].float() - v.float()).abs().max().item()
        assert d <= 1e-5 * max(1.0, v.abs().max().item()), k


def test_apply_domino_requires_tp():
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    from shuffle_exchange_amd.runtime.domino import apply_domino
    with pytest.raises(AssertionError):
        apply_domino(LlamaForCausalLM(llama_config("llama-tiny")))
