"""Autotuner: memory pruning of infeasible stages, grid / random / model-based search find the best
(synthetic) configuration, and a real in-process experiment measures engine throughput."""
import pytest


def _synthetic(cfg):
    mbs = cfg["train_micro_batch_size_per_gpu"]
    st = cfg["zero_optimization"]["stage"]
    if mbs > 8:
        raise RuntimeError("OOM")
    return 100 * mbs - 10 * (mbs - 4) ** 2 + (5 if st == 2 else 0)


@pytest.mark.parametrize("tuner", ["gridsearch", "random", "model_based"])
def test_autotuner_finds_best(tuner, tmp_path):
    from shuffle_exchange_amd.autotuning import Autotuner
    at = Autotuner({"optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}}, results_dir=str(tmp_path), tuner_type=tuner,
                   tuner_num_trials=40, tuner_early_stopping=None, micro_batch_sizes=[1, 2, 4, 8, 16], stages=(0, 1, 2, 3))
    best = at.tune(_synthetic)
    assert best.overrides["train_micro_batch_size_per_gpu"] == 8
    assert (tmp_path / "summary.json").exists()


def test_memory_pruning():
    from shuffle_exchange_amd.autotuning import Autotuner, model_state_bytes
    at = Autotuner({}, num_params=70e9, world_size=8)
    assert 0 not in at.feasible_stages() and 3 in at.feasible_stages()
    assert model_state_bytes(8e9, 3, 8) < model_state_bytes(8e9, 1, 8)


def test_engine_metric_probe(tmp_path):
    import json
    import torch
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    m = LlamaForCausalLM(llama_config("llama-tiny", num_hidden_layers=1))
    mp = tmp_path / "metric.json"
    ds = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
          "autotuning": {"enabled": True, "metric_path": str(mp), "start_profile_step": 1, "end_profile_step": 3,
                         "exit_after_profile": False}}
    eng, _, _, _ = sxe.initialize(model=m, config=ds)
    for _ in range(4):
        ids = torch.randint(0, 512, (2, 16))
        loss = eng(ids, labels=ids)
        eng.backward(loss)
        eng.step()
    assert json.loads(mp.read_text())["throughput"] > 0
