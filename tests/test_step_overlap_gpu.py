"""Opt-in overlapped device optimizer step (SXE_STEP_OVERLAP=1, zero/base.py): fused Adam per unit
on a side stream with per-unit waits in the next forward / gathers gives bit-identical parameters to
the one-launch update, for ZeRO-2 and ZeRO-3, with gradient accumulation."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(stage, overlap, monkeypatch):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    monkeypatch.setenv("SXE_STEP_OVERLAP", "1" if overlap else "0")
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=256, intermediate_size=512, num_attention_heads=4,
                       num_key_value_heads=2, vocab_size=1024, num_hidden_layers=2)
    model = LlamaForCausalLM(cfg).to("cuda", torch.bfloat16)
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2, "bf16": {"enabled": True},
          "zero_optimization": {"stage": stage, "reduce_bucket_size": 300000, "stage3_param_persistence_threshold": 0},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "gradient_clipping": 1.0}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(6):
        ids = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
        eng.backward(eng(ids, labels=ids))
        eng.step()
    if stage == 3:
        out = {k: v.clone() for k, v in eng._zero3_consolidated_16bit_state_dict().items()}
    else:
        eng.optimizer.wait_params()
        out = {n: p.detach().cpu().clone() for n, p in eng.module.named_parameters()}
    used = bool(getattr(eng.optimizer, "_step_stream", None) is not None)
    eng.destroy()
    from shuffle_exchange_amd.parallel import groups
    groups.reset()
    return out, used


@pytest.mark.parametrize("stage", [2, 3])
def test_overlapped_step_bit_identical(stage, monkeypatch):
    a, used_a = _train(stage, True, monkeypatch)
    b, used_b = _train(stage, False, monkeypatch)
    assert used_a and not used_b
    for k in b:
        assert torch.equal(a[k], b[k]), k
