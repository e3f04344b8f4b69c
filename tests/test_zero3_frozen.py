"""ZeRO-3 owns frozen parameters (reference partitioned_param_coordinator.py:300,437,544 fetches every
parameter of a submodule; partition_parameters.py:1685,1769 / stage3.py:1558 quantized non-trainable
weights): a zero.Init model with a LoRA-style frozen base trains at W=2 over gloo like the
single-process reference, each rank holds 1/W of the frozen weights, and save_16bit_model includes them."""
import pytest
import torch

from . import _dist_cases as C
from .dist_utils import run_dist


@pytest.mark.parametrize("quant", [False, True])
def test_zero3_frozen_params_zero_init_w2(tmp_path, quant):
    world, steps = 2, 3
    res = run_dist(C.case_zero3_frozen, world, steps, quant, str(tmp_path))
    r0, r1 = res[0], res[1]
    names = r0["frozen_names"]
    assert names and r0["n_frozen_units"] >= 2 and r0["released"]
    # each rank holds 1/W of the frozen weights (units pad to 256-byte aligned chunks)
    for r in (r0, r1):
        assert abs(r["frozen_shard"] - r["frozen_total"] / world) <= 64 * r["n_frozen_units"] * world
    if quant:
        assert r0["n_quant"] == r0["n_frozen_units"]
        # int8 + one fp32 scale per 128 (or 64) elements: well under the bit16 1/W share
        assert r0["frozen_bytes"] < 0.6 * 4 * r0["frozen_total"] / world
    else:
        assert r0["n_quant"] == 0
    ref, ref_losses = C.frozen_reference(r0["before"], names, steps, world)
    # ranks agree; frozen weights unchanged; trainable ones follow the reference
    for k in ref:
        torch.testing.assert_close(r0["after"][k], r1["after"][k])
    tol = dict(atol=2e-2, rtol=2e-2) if quant else dict(atol=2e-4, rtol=2e-4)
    for k in names:
        torch.testing.assert_close(r0["after"][k], r0["before"][k], **({} if not quant else tol))
    for k, v in ref.items():
        if k not in names:
            torch.testing.assert_close(r0["after"][k], v, **tol)
    mean = [(a + b) / 2 for a, b in zip(r0["losses"], r1["losses"])]
    for a, b in zip(mean, ref_losses):
        assert abs(a - b) < (2e-2 if quant else 1e-4), (mean, ref_losses)
    # the consolidated 16-bit export and the checkpoint fragments include the frozen weights
    assert set(names) <= set(r0["saved_keys"])
    for k in names:
        torch.testing.assert_close(r0["saved_frozen"][k], r0["after"][k])
    assert set(r0["frag_keys"]) == set(names) and r1["frag_keys"] == []
