"""Resume from checkpoints in the REFERENCE's ZeRO layout (checkpoint/reference_format.py).

The reference is not importable here, so the files are synthesised with its key schema
(runtime/zero/stage_1_and_2.py:2472-2512, stage3 ``fp32_flat_groups``, checkpoint/constants.py) and
its pickled class paths (``deepspeed.runtime.fp16.loss_scaler.DynamicLossScaler``,
``deepspeed.runtime.zero.config.ZeroStageEnum``, ``deepspeed.utils.tensor_fragment.fragment_address``)
-- registered in a throw-away ``sys.modules`` only while writing. The loader runs in fresh gloo
processes that have no ``deepspeed`` module at all and reads with ``weights_only=True``. Parity
against files written by the reference itself: unpinned."""
import collections
import dataclasses
import enum
import os
import sys
import types

import pytest
import torch

from ._dist_cases import tiny_llama
from .dist_utils import run_dist


def _fake_reference_modules():
    mods = {}
    for name in ("deepspeed", "deepspeed.runtime", "deepspeed.runtime.fp16", "deepspeed.runtime.fp16.loss_scaler",
                 "deepspeed.runtime.zero", "deepspeed.runtime.zero.config", "deepspeed.utils",
                 "deepspeed.utils.tensor_fragment"):
        mods[name] = types.ModuleType(name)

    class DynamicLossScaler:
        def __init__(self):
            self.cur_scale, self.cur_iter, self.last_overflow_iter = 1024.0, 5, 2
            self.scale_factor, self.scale_window, self.min_scale = 2.0, 1000, 1
            self.delayed_shift, self.cur_hysteresis, self.consecutive_hysteresis = 2, 1, False
            self.dynamic, self.dtype = True, torch.half
    DynamicLossScaler.__module__ = "deepspeed.runtime.fp16.loss_scaler"
    DynamicLossScaler.__qualname__ = "DynamicLossScaler"

    class ZeroStageEnum(int, enum.Enum):
        disabled = 0
        optimizer_states = 1
        gradients = 2
        weights = 3
    ZeroStageEnum.__module__ = "deepspeed.runtime.zero.config"
    ZeroStageEnum.__qualname__ = "ZeroStageEnum"

    @dataclasses.dataclass
    class fragment_address:  # noqa: N801 - the reference's class name
        numel: int
        start: int
    fragment_address.__module__ = "deepspeed.utils.tensor_fragment"
    fragment_address.__qualname__ = "fragment_address"

    mods["deepspeed.runtime.fp16.loss_scaler"].DynamicLossScaler = DynamicLossScaler
    mods["deepspeed.runtime.zero.config"].ZeroStageEnum = ZeroStageEnum
    mods["deepspeed.utils.tensor_fragment"].fragment_address = fragment_address
    return mods, DynamicLossScaler, ZeroStageEnum, fragment_address


def _synthetic_state():
    model, _ = tiny_llama(0)
    g = torch.Generator().manual_seed(123)
    named = [(n, p.detach().float()) for n, p in model.named_parameters()]
    fp32 = {n: t + 0.01 * torch.randn(t.shape, generator=g) for n, t in named}
    m = {n: 1e-3 * torch.randn(t.shape, generator=g) for n, t in named}
    v = {n: 1e-5 * torch.rand(t.shape, generator=g) for n, t in named}
    return [n for n, _ in named], fp32, m, v


def write_reference_checkpoint(d, stage, dp, step=7, bf16_optimizer=False):
    """``bf16_optimizer``: the reference BF16_Optimizer's files (runtime/bf16_optimizer.py:467-477:
    no zero_stage / loss scaler keys, ``bf16_zero_pp_rank_*`` names, engine.py:2927)."""
    mods, DLS, ZSE, FA = _fake_reference_modules()
    names, fp32, m, v = _synthetic_state()
    saved = {k: sys.modules.get(k) for k in mods}
    sys.modules.update(mods)
    try:
        tag_dir = os.path.join(d, "global_step7")
        os.makedirs(tag_dir, exist_ok=True)
        with open(os.path.join(d, "latest"), "w") as f:
            f.write("global_step7")
        shapes = [collections.OrderedDict((n, fp32[n].shape) for n in names)]
        model_states = {"module": {n: fp32[n].to(torch.bfloat16) for n in names} if stage < 3 else None,
                        "buffer_names": [], "param_shapes": shapes, "frozen_param_shapes": None,
                        "shared_params": {}, "lr_scheduler": None, "global_steps": step, "global_samples": 4 * step,
                        "skipped_steps": 0, "dp_world_size": dp, "mp_world_size": 1, "ds_version": "0.16.0",
                        "ds_config": {"zero_optimization": {"stage": stage}}}
        if stage < 3:
            torch.save(model_states, os.path.join(tag_dir, "mp_rank_00_model_states.pt"))
            flat = {k: torch.cat([t[n].reshape(-1) for n in names]) for k, t in (("p", fp32), ("m", m), ("v", v))}
            total = flat["p"].numel()
            align = 2 * dp
            padded = -(-total // align) * align
            part = padded // dp
            for r in range(dp):
                lo, hi = r * part, (r + 1) * part
                pad = lambda t: torch.cat([t, t.new_zeros(padded - total)])[lo:hi]  # noqa: E731
                mapping = collections.OrderedDict()
                off = 0
                for n in names:
                    nn_ = fp32[n].numel()
                    a, b = max(off, lo), min(off + nn_, hi)
                    if a < b:
                        mapping[n] = FA(numel=b - a, start=a - lo)
                    off += nn_
                osd = {"loss_scaler": DLS(), "dynamic_loss_scale": True, "overflow": False, "clip_grad": 1.0,
                       "base_optimizer_state": {"state": {0: {"step": torch.tensor(float(step)), "exp_avg": pad(flat["m"]),
                                                              "exp_avg_sq": pad(flat["v"])}},
                                                "param_groups": [{"lr": 1e-3, "params": [0]}]},
                       "single_partition_of_fp32_groups": [pad(flat["p"])[:max(0, min(hi, total) - lo)]],
                       "zero_stage": ZSE(stage), "group_paddings": [padded - total if r == dp - 1 else 0],
                       "partition_count": [dp], "ds_version": "0.16.0", "param_slice_mappings": [mapping]}
                prefix = ""
                if bf16_optimizer:
                    for k in ("loss_scaler", "dynamic_loss_scale", "overflow", "zero_stage"):
                        osd.pop(k)
                    prefix = "bf16_"
                torch.save({"optimizer_state_dict": osd, "ds_config": {}, "ds_version": "0.16.0"},
                           os.path.join(tag_dir, f"{prefix}zero_pp_rank_{r}_mp_rank_00_optim_states.pt"))
        else:
            for r in range(dp):
                torch.save(dict(model_states, module={}),
                           os.path.join(tag_dir, f"zero_pp_rank_{r}_mp_rank_00_model_states.pt"))
                parts = {}
                for key, src in (("p", fp32), ("m", m), ("v", v)):
                    pieces = []
                    for n in names:
                        t = src[n].reshape(-1)
                        ps = -(-t.numel() // dp)
                        t = torch.cat([t, t.new_zeros(ps * dp - t.numel())])
                        pieces.append(t[r * ps:(r + 1) * ps])
                    parts[key] = torch.cat(pieces)
                osd = {"zero_stage": ZSE(3), "loss_scaler": DLS(), "dynamic_loss_scale": True, "overflow": False,
                       "partition_count": dp, "fp32_flat_groups": [parts["p"]],
                       "optimizer_state_dict": {"state": {0: {"step": torch.tensor(float(step)), "exp_avg": parts["m"],
                                                              "exp_avg_sq": parts["v"]}},
                                                "param_groups": [{"lr": 1e-3, "params": [0]}]}}
                torch.save({"optimizer_state_dict": osd, "ds_config": {}, "ds_version": "0.16.0"},
                           os.path.join(tag_dir, f"zero_pp_rank_{r}_mp_rank_00_optim_states.pt"))
    finally:
        for k, old in saved.items():
            if old is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = old
    return fp32, m, v


def _case_resume(rank, world, ckdir, stage):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.utils.tensor_fragment import safe_get_full_fp32_param, safe_get_full_optimizer_state
    assert "deepspeed" not in sys.modules
    model, _ = tiny_llama(5)  # different init: everything must come from the checkpoint
    ds = {"train_micro_batch_size_per_gpu": 1, "zero_optimization": {"stage": stage,
                                                                       "stage3_param_persistence_threshold": 0},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    path, client = eng.load_checkpoint(ckdir)
    out = {"fp32": {}, "m": {}, "v": {}, "steps": eng.global_steps}
    for n, p in eng.module.named_parameters():
        out["fp32"][n] = safe_get_full_fp32_param(p).clone()
        out["m"][n] = safe_get_full_optimizer_state(p, "exp_avg").clone()
        out["v"][n] = safe_get_full_optimizer_state(p, "exp_avg_sq").clone()
    return out


@pytest.mark.parametrize("saved_stage,saved_dp,load_stage,load_world", [(2, 2, 2, 2), (1, 4, 3, 2), (3, 2, 1, 1),
                                                                        (3, 3, 3, 2)])
def test_resume_from_reference_layout_checkpoint(tmp_path, saved_stage, saved_dp, load_stage, load_world):
    """A reference-layout ZeRO-{1,2,3} checkpoint written at one dp degree resumes here under another
    stage / world size: fp32 masters, Adam moments and global_steps all restored exactly."""
    fp32, m, v = write_reference_checkpoint(str(tmp_path), saved_stage, saved_dp)
    res = run_dist(_case_resume, load_world, str(tmp_path), load_stage)
    for r in res:
        assert r["steps"] == 7
        for n in fp32:
            assert torch.allclose(r["fp32"][n], fp32[n], atol=1e-7), n
            assert torch.allclose(r["m"][n], m[n], atol=1e-9), n
            assert torch.allclose(r["v"][n], v[n], atol=1e-9), n


def test_resume_from_reference_bf16_optimizer_checkpoint(tmp_path):
    """Files of the reference's BF16_Optimizer (bf16_ prefix, ZeRO-1 schema without zero_stage) are
    detected as reference format and resume exactly."""
    from shuffle_exchange_amd.checkpoint.reference_format import is_reference_checkpoint
    fp32, m, v = write_reference_checkpoint(str(tmp_path), 1, 2, bf16_optimizer=True)
    assert is_reference_checkpoint(str(tmp_path))
    for r in run_dist(_case_resume, 2, str(tmp_path), 1):
        assert r["steps"] == 7
        for n in fp32:
            assert torch.allclose(r["fp32"][n], fp32[n], atol=1e-7), n
            assert torch.allclose(r["m"][n], m[n], atol=1e-9), n


def test_zero_to_fp32_reads_reference_layout(tmp_path):
    from shuffle_exchange_amd.utils.zero_to_fp32 import get_fp32_state_dict_from_zero_checkpoint
    for stage in (2, 3):
        d = tmp_path / f"s{stage}"
        fp32, _, _ = write_reference_checkpoint(str(d), stage, 3)
        sd = get_fp32_state_dict_from_zero_checkpoint(str(d))
        assert set(sd) == set(fp32)
        for n in fp32:
            assert torch.equal(sd[n], fp32[n]), n


def test_reference_files_load_with_weights_only(tmp_path):
    """The pickled reference classes resolve to inert stand-ins; a plain weights_only load refuses."""
    from shuffle_exchange_amd.checkpoint.reference_format import load_file
    write_reference_checkpoint(str(tmp_path), 2, 1)
    f = tmp_path / "global_step7" / "zero_pp_rank_0_mp_rank_00_optim_states.pt"
    with pytest.raises(Exception):
        torch.load(f, weights_only=True)
    osd = load_file(f)["optimizer_state_dict"]
    assert osd["loss_scaler"].state()["cur_scale"] == 1024.0
    assert int(osd["zero_stage"]) == 2


def _case_universal(rank, world, udir):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.utils.tensor_fragment import safe_get_full_fp32_param, safe_get_full_optimizer_state
    model, _ = tiny_llama(5)
    ds = {"train_micro_batch_size_per_gpu": 1, "zero_optimization": {"stage": 2},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "checkpoint": {"load_universal": True}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    eng.load_checkpoint(os.path.dirname(udir), tag=os.path.basename(udir))
    return {n: (safe_get_full_fp32_param(p).clone(), safe_get_full_optimizer_state(p, "exp_avg").clone())
            for n, p in eng.module.named_parameters()}


def test_reference_checkpoint_to_universal_and_resume(tmp_path):
    """ds_to_universal on a reference-layout ZeRO-3 checkpoint (dp 3), resumed as ZeRO-2 on 2 ranks."""
    from shuffle_exchange_amd.checkpoint.universal import convert_to_universal
    fp32, m, _ = write_reference_checkpoint(str(tmp_path / "ck"), 3, 3)
    udir = tmp_path / "uni" / "global_step7"
    convert_to_universal(str(tmp_path / "ck"), str(udir))
    assert (udir / "zero" / "lm_head.weight" / "fp32.pt").exists()
    for r in run_dist(_case_universal, 2, str(udir)):
        for n in fp32:
            assert torch.allclose(r[n][0], fp32[n], atol=1e-7), n
            assert torch.allclose(r[n][1], m[n], atol=1e-9), n
