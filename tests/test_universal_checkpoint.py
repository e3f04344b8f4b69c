"""Universal checkpoint: save on 4 ranks (ZeRO-2 / ZeRO-3), convert offline, resume on 2 ranks (and
on a different stage) -- continued training matches the uninterrupted 4-rank run's parameters at
the same global batch."""
import pytest
import torch

from .dist_utils import run_dist


def _cfg(stage, universal=False):
    return {"train_micro_batch_size_per_gpu": 2 if not universal else 4,
            "zero_optimization": {"stage": stage, "reduce_bucket_size": 30000, "stage3_param_persistence_threshold": 0},
            "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
            "checkpoint": {"load_universal": universal}}


def _case_save(rank, world, stage, d, steps_a, steps_b):
    import shuffle_exchange_amd as sxe
    from ._dist_cases import full_params, global_batches, tiny_llama
    model, cfg = tiny_llama(0)
    eng, _, _, _ = sxe.initialize(model=model, config=_cfg(stage))
    bs = global_batches(cfg, world, 2, 16, steps_a + steps_b)
    for i, b in enumerate(bs):
        local = b[rank * 2:(rank + 1) * 2]
        loss = eng(local, labels=local)
        eng.backward(loss)
        eng.step()
        if i == steps_a - 1:
            eng.save_checkpoint(d, tag="t")
    return full_params(eng)


def _case_resume(rank, world, stage, d, steps_a, steps_b):
    import shuffle_exchange_amd as sxe
    from ._dist_cases import full_params, global_batches, tiny_llama
    model, cfg = tiny_llama(7)
    eng, _, _, _ = sxe.initialize(model=model, config=_cfg(stage, universal=True))
    eng.load_checkpoint(d, tag="t_universal")
    bs = global_batches(cfg, 4, 2, 16, steps_a + steps_b)[steps_a:]
    for b in bs:  # same global batch (8 samples) split over 2 ranks x 4
        local = b[rank * 4:(rank + 1) * 4]
        loss = eng(local, labels=local)
        eng.backward(loss)
        eng.step()
    return full_params(eng)


@pytest.mark.parametrize("src_stage,dst_stage", [(2, 2), (3, 1), (1, 3)])
def test_universal_resume_on_fewer_ranks(tmp_path, src_stage, dst_stage):
    from shuffle_exchange_amd.checkpoint.universal import convert_to_universal
    ref = run_dist(_case_save, 4, src_stage, str(tmp_path), 2, 2)[0]
    convert_to_universal(str(tmp_path), str(tmp_path / "t_universal"), tag="t")
    got = run_dist(_case_resume, 2, dst_stage, str(tmp_path), 2, 2)[0]
    for k, v in ref.items():
        d = (got[k] - v).abs().max().item()
        assert d <= 2e-4 * max(1.0, v.abs().max().item()), (k, d)
