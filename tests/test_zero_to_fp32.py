"""Offline consolidation of ZeRO checkpoints (stages 0-3, Shuffle-exchange slices) into one fp32
state dict equals the live engine's full parameters."""
import pytest
import torch

from .dist_utils import run_dist


def _case_save(rank, world, stage, d, se):
    import shuffle_exchange_amd as sxe
    from ._dist_cases import full_params, global_batches, tiny_llama
    model, cfg = tiny_llama(0)
    ds = {"train_micro_batch_size_per_gpu": 2, "zero_optimization": {"stage": stage, "reduce_bucket_size": 30000,
                                                                     "stage3_param_persistence_threshold": 0},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}}
    kw = {"method": "RR", "slice_count": 2} if se else {}
    eng, _, _, _ = sxe.initialize(model=model, config=ds, **kw)
    for b in global_batches(cfg, world, 2, 16, 2):
        local = b[rank * 2:(rank + 1) * 2]
        loss = eng(local, labels=local)
        eng.backward(loss)
        eng.step()
    eng.save_checkpoint(d)
    return full_params(eng)


@pytest.mark.parametrize("stage,world,se", [(0, 2, False), (1, 2, False), (2, 2, False), (3, 2, False),
                                            (2, 4, True)])
def test_zero_to_fp32(tmp_path, stage, world, se):
    from shuffle_exchange_amd.utils.zero_to_fp32 import (convert_zero_checkpoint_to_fp32_state_dict,
                                                         get_fp32_state_dict_from_zero_checkpoint)
    live = run_dist(_case_save, world, stage, str(tmp_path), se)[0]
    sd = get_fp32_state_dict_from_zero_checkpoint(str(tmp_path))
    for k, v in live.items():
        assert torch.allclose(sd[k], v, atol=1e-6), k
    out = convert_zero_checkpoint_to_fp32_state_dict(str(tmp_path), str(tmp_path / "fp32" / "model.pt"))
    assert set(torch.load(out, weights_only=True)) >= set(live)
