"""ZeRO gradient delivery for tiled / recomputed sub-graphs (ALST ``TiledMLP`` and
``sequence_tiled_compute``) and for parameters without a gradient in some micro-steps.

Every tile but the last delivers a partial parameter gradient; the ZeRO hooks must keep summing it
and reduce the unit once with the total (reference ``ds_grad_is_ready``,
runtime/sequence_parallel/ulysses_sp.py:720-724,846-850, honoured at stage_1_and_2.py:1146 and
stage3.py:1280). Before the fix a unit completed by the first tile was reduced early and the later
tiles added into a fresh uninitialised staging buffer (1.3e-2 parameter error at ZeRO-2 with
reduce_bucket_size 1). All cases run 2 gloo ranks and compare against the untiled engine."""
import pytest
import torch

from .dist_utils import run_dist


class _SeqTiled(torch.nn.Module):
    """An MLP run through ``sequence_tiled_compute`` with explicit parameters."""

    def __init__(self, mlp, n):
        super().__init__()
        self.mlp, self.n = mlp, n

    def forward(self, x):
        from shuffle_exchange_amd.sequence.tiled import sequence_tiled_compute
        return sequence_tiled_compute(self.mlp, x, n_tiles=self.n, params=tuple(self.mlp.parameters()))


def _case(rank, world, stage, bucket, mode, gas):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.sequence import TiledMLP
    from ._dist_cases import full_params, global_batches, tiny_llama
    model, cfg = tiny_llama(0)
    if mode == "tiled_mlp":
        for layer in model.layers:
            layer.mlp = TiledMLP(layer.mlp, num_shards=4)
    elif mode == "seq_tiled":
        for layer in model.layers:
            layer.mlp = _SeqTiled(layer.mlp, 4)
    zero = {"stage": stage}
    if bucket is not None:
        zero["reduce_bucket_size"] = bucket
        if stage == 3:
            zero["stage3_param_persistence_threshold"] = 0
    ds = {"train_micro_batch_size_per_gpu": 1, "gradient_accumulation_steps": gas, "zero_optimization": zero,
          "optimizer": {"type": "SGD", "params": {"lr": 0.1}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    for b in global_batches(cfg, world * gas, 1, 16, 1):
        for m in range(gas):
            local = b[(m * world + rank):(m * world + rank) + 1]
            loss = eng(local, labels=local)
            eng.backward(loss)
            eng.step()
    return {k.replace(".mlp.mlp.", ".mlp."): v for k, v in full_params(eng).items()}


@pytest.mark.parametrize("stage,bucket", [(1, 1), (2, 1), (2, None), (3, 1), (3, None)])
@pytest.mark.parametrize("mode", ["tiled_mlp", "seq_tiled"])
def test_tiled_compute_matches_untiled_under_zero(stage, bucket, mode):
    ref = run_dist(_case, 2, stage, bucket, "plain", 1)[0]
    got = run_dist(_case, 2, stage, bucket, mode, 1)
    for r in got:
        assert set(r) == set(ref)
        err = max((r[k] - ref[k]).abs().max().item() for k in ref)
        assert err < 1e-6, err


def test_tiled_mlp_zero1_grad_accumulation():
    """ZeRO-1 across 2 accumulation micro-steps with tiles: same update as untiled."""
    ref = run_dist(_case, 2, 1, 1, "plain", 2)[0]
    for r in run_dist(_case, 2, 1, 1, "tiled_mlp", 2):
        err = max((r[k] - ref[k]).abs().max().item() for k in ref)
        assert err < 1e-6, err


class _Branchy(torch.nn.Module):
    """``b`` is used only on odd micro-steps, ``c`` never: their fp32 staging slots must read as
    zero, not as torch.empty garbage, when the ZeRO-1 fp32 accumulation carries across micro-steps."""

    def __init__(self):
        super().__init__()
        self.a = torch.nn.Parameter(torch.ones(64))
        self.b = torch.nn.Parameter(torch.ones(64))
        self.c = torch.nn.Parameter(torch.ones(64))
        self.calls = 0

    def forward(self, x):
        self.calls += 1
        y = (self.a * x).sum()
        if self.calls % 2 == 0:
            y = y + (self.b * x).sum()
        return y


def _case_branchy(rank, world, gas):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.utils.tensor_fragment import safe_get_full_fp32_param
    model = _Branchy()
    ds = {"train_micro_batch_size_per_gpu": 1, "gradient_accumulation_steps": gas, "bf16": {"enabled": True},
          "data_types": {"grad_accum_dtype": "fp32"},
          "zero_optimization": {"stage": 1, "reduce_bucket_size": 10_000},
          "optimizer": {"type": "SGD", "params": {"lr": 1.0}}, "zero_allow_untested_optimizer": True}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    # poison torch.empty (the staging allocator) so an unwritten slot reads NaN, as GPU memory can
    import shuffle_exchange_amd.runtime.zero.flat as flat_mod
    real_empty = torch.empty

    def poisoned(*a, **k):
        t = real_empty(*a, **k)
        return t.fill_(float("nan")) if t.is_floating_point() else t

    flat_mod.torch = type("T", (), {"__getattr__": lambda self, n: poisoned if n == "empty" else getattr(torch, n)})()
    for m in range(gas):
        x = torch.full((64,), float(rank + 1 + m), dtype=torch.bfloat16)
        loss = eng(x)
        eng.backward(loss)
        eng.step()
    return {n: safe_get_full_fp32_param(getattr(model, n)).clone() for n in "abc"}


def test_fp32_accum_unused_param_slots_are_zero():
    gas = 4
    out = run_dist(_case_branchy, 2, gas)
    # expected: a gets every micro-step, b only the odd ones (m = 1, 3), c nothing
    ga = sum(r + 1 + m for r in range(2) for m in range(gas)) / (2 * gas)
    gb = sum(r + 1 + m for r in range(2) for m in range(gas) if m % 2 == 1) / (2 * gas)
    for r in out:
        torch.testing.assert_close(r["a"], torch.full((64,), 1.0 - ga), atol=1e-5, rtol=0)
        torch.testing.assert_close(r["b"], torch.full((64,), 1.0 - gb), atol=1e-5, rtol=0)
        torch.testing.assert_close(r["c"], torch.ones(64), atol=0, rtol=0)
