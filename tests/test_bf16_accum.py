"""BF16_Optimizer semantics: fp32 gradient accumulation (data_types.grad_accum_dtype), the skipped
non-finite bf16 step (LR scheduler not advanced, skipped_steps counted) and config-key honesty.

Reference: runtime/engine.py:1074-1089 (grad_accum_dtype defaults), :1384-1386 (bf16 + ZeRO-1 +
fp32 accumulation -> BF16_Optimizer), :2376-2390 (no scheduler step on overflow),
runtime/config_utils.py:110 (extra keys forbidden)."""
import os

import pytest
import torch

from .dist_utils import run_dist

GAS = 8
N = 4096


class _Lin(torch.nn.Module):
    """loss = sum(w * c): dL/dw = c exactly, so the accumulated gradient is known in closed form."""

    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.zeros(N))

    def forward(self, c):
        return (self.w * c).sum()


def _micro_inputs(rank):
    g = torch.Generator().manual_seed(100 + rank)
    # values in [1, 2) with a full bf16 mantissa: summing 8 of them in bf16 rounds at every add
    return [(1.0 + torch.rand(N, generator=g)).to(torch.bfloat16) for _ in range(GAS)]


def _case_accum(rank, world, stage, accum):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.runtime.bf16_optimizer import BF16_Optimizer
    from shuffle_exchange_amd.utils.tensor_fragment import safe_get_full_fp32_param
    torch.manual_seed(0)
    model = _Lin()
    ds = {"train_micro_batch_size_per_gpu": 1, "gradient_accumulation_steps": GAS, "bf16": {"enabled": True},
          "zero_optimization": {"stage": stage, "reduce_bucket_size": 1000},
          "optimizer": {"type": "SGD", "params": {"lr": 1.0}}, "zero_allow_untested_optimizer": True}
    if accum is not None:
        ds["data_types"] = {"grad_accum_dtype": accum}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    for c in _micro_inputs(rank):
        loss = eng(c)
        eng.backward(loss)
        eng.step()
    return {"w": safe_get_full_fp32_param(model.w).clone(), "bf16opt": isinstance(eng.optimizer, BF16_Optimizer)}


def _expected(world):
    tot = torch.zeros(N, dtype=torch.float64)
    for r in range(world):
        for c in _micro_inputs(r):
            tot += c.double() / GAS
    return -(tot / world).float()


@pytest.mark.parametrize("stage,accum,bf16opt", [(1, "fp32", True), (0, None, False)])
def test_fp32_grad_accumulation_matches_fp32_reference(stage, accum, bf16opt):
    """ZeRO-1 with grad_accum_dtype=fp32 routes to BF16_Optimizer; bf16 ZeRO-0 accumulates in fp32
    by default. Over GAS=8 micro-steps on 2 gloo ranks the update equals the fp64 mean of every
    micro-gradient (to fp32 rounding)."""
    exp = _expected(2)
    for r in run_dist(_case_accum, 2, stage, accum):
        assert r["bf16opt"] == bf16opt
        torch.testing.assert_close(r["w"], exp, atol=2e-6, rtol=0)


def test_bf16_accumulation_is_measurably_worse():
    """Control: with grad_accum_dtype=bf16 the same run rounds at every micro-step (so the test above
    really discriminates the accumulation dtype)."""
    exp = _expected(2)
    r = run_dist(_case_accum, 2, 1, "bf16")[0]
    assert not r["bf16opt"]
    assert (r["w"] - exp).abs().max() > 1e-3


def _case_skip(rank, world, stage, ckdir):
    import shuffle_exchange_amd as sxe
    torch.manual_seed(0)
    model = _Lin()
    ds = {"train_micro_batch_size_per_gpu": 1, "bf16": {"enabled": True}, "gradient_clipping": 1.0,
          "zero_optimization": {"stage": stage},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
          "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0.0, "warmup_max_lr": 1e-2,
                                                       "warmup_num_steps": 10, "warmup_type": "linear"}}}
    eng, _, _, sched = sxe.initialize(model=model, config=ds)
    lrs, ws, sched_lrs = [], [], []
    for i in range(4):
        c = torch.ones(N, dtype=torch.bfloat16)
        if i == 2 and rank == 1:
            c[7] = float("inf")  # one rank's gradient is non-finite: every rank must skip
        loss = eng(c)
        eng.backward(loss)
        eng.step()
        # the scheduler object the user holds resolves the deferred advance too (not one step stale)
        sched_lrs.append(sched.get_last_lr()[0])
        lrs.append(eng.get_lr()[0])
        ws.append(model.w.detach().float().clone())
    eng.save_checkpoint(ckdir)
    return {"lrs": lrs, "sched_lrs": sched_lrs, "skipped": eng.skipped_steps, "ws": ws, "global": eng.global_steps}


@pytest.mark.parametrize("stage", [0, 1, 3])
def test_nonfinite_bf16_step_skips_scheduler(tmp_path, stage):
    res = run_dist(_case_skip, 2, stage, str(tmp_path / f"ck{stage}"))
    for r in res:
        assert r["skipped"] == 1
        assert r["global"] == 4
        # linear warm-up: lr advances after steps 1, 2, 4 only (step 3 was skipped)
        assert r["sched_lrs"] == pytest.approx(r["lrs"])
        l0, l1, l2, l3 = r["lrs"]
        assert l1 > l0 and l2 == pytest.approx(l1) and l3 > l2
        assert torch.equal(r["ws"][2], r["ws"][1])  # the skipped step left the weights alone
        assert torch.isfinite(r["ws"][3]).all()
    torch.testing.assert_close(res[0]["ws"][3], res[1]["ws"][3])


def test_bf16_optimizer_checkpoint_prefix(tmp_path):
    """BF16_Optimizer files carry the reference's bf16_ prefix (engine.py:2927)."""
    run_dist(_case_accum_ckpt, 1, str(tmp_path))
    names = os.listdir(tmp_path / "global_step1")
    assert any(n.startswith("bf16_zero_pp_rank_0") for n in names), names


def _case_accum_ckpt(rank, world, d):
    import shuffle_exchange_amd as sxe
    model = _Lin()
    ds = {"train_micro_batch_size_per_gpu": 1, "bf16": {"enabled": True}, "zero_optimization": {"stage": 1},
          "data_types": {"grad_accum_dtype": "fp32"}, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    loss = eng(torch.ones(N, dtype=torch.bfloat16))
    eng.backward(loss)
    eng.step()
    eng.save_checkpoint(d)
    eng.load_checkpoint(d)
    return True


def test_unknown_config_key_warns_and_strict_raises():
    from unittest import mock

    from shuffle_exchange_amd.runtime import config as C
    from shuffle_exchange_amd.runtime.config import SXEConfig
    with mock.patch.object(C.logger, "warning") as warn:
        cfg = SXEConfig({"train_micro_batch_size_per_gpu": 1, "zero_optimization": {"stage": 2,
                                                                                      "reduce_bucket_sise": 5}})
    assert cfg.unknown_keys == ["zero_optimization.reduce_bucket_sise"]
    assert any("did you mean 'reduce_bucket_size'" in str(c.args[0]) for c in warn.call_args_list)
    with pytest.raises(ValueError, match="reduce_bucket_sise"):
        SXEConfig({"train_micro_batch_size_per_gpu": 1, "strict_config": True,
                   "zero_optimization": {"reduce_bucket_sise": 5}})
    # root blocks owned by other subsystems are not "unknown"
    assert SXEConfig({"train_micro_batch_size_per_gpu": 1, "data_efficiency": {"enabled": False},
                      "strict_config": True}).unknown_keys == []


def test_grad_accum_dtype_defaults():
    from shuffle_exchange_amd.runtime.config import SXEConfig
    b = {"train_micro_batch_size_per_gpu": 1, "bf16": {"enabled": True}}
    assert SXEConfig(b).grad_accum_dtype == "fp32"  # bf16 without ZeRO
    assert SXEConfig({**b, "zero_optimization": {"stage": 1}}).grad_accum_dtype == "bf16"
    assert SXEConfig({**b, "zero_optimization": {"stage": 1},
                      "data_types": {"grad_accum_dtype": "fp32"}}).grad_accum_dtype == "fp32"
    with pytest.raises(Exception):
        SXEConfig({**b, "data_types": {"grad_accum_dtype": "int8"}})
