"""ZeRO-3 partitioned over 2 ranks that share ONE MI355X (also with the deferred reduce-scatter and
params retained across micro-steps, as bench.py runs it) (gloo host collectives; RCCL needs one GPU
per rank): exercises the GPU side of stage 3 -- all-gather / reduce-scatter side streams, events,
record_stream fencing, kept-for-backward units, TN weight-gradient path into bf16 staging -- and
compares with the single-rank result on the same GPU."""
import os

import pytest
import torch

from . import _dist_cases as C
from .dist_utils import run_dist

pytestmark = pytest.mark.gpu


def _case(rank, world, reuse, stage=3, se=None, defer=False, offload_param=False):
    os.environ["LOCAL_RANK"] = "0"  # both ranks on GPU 0
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=256, intermediate_size=512, num_attention_heads=2,
                       num_key_value_heads=1, vocab_size=1024, num_hidden_layers=2)
    with sxe.zero.Init(dtype=torch.bfloat16):
        model = LlamaForCausalLM(cfg)
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2, "bf16": {"enabled": True},
          "zero_optimization": {"stage": stage, "stage3_param_persistence_threshold": 0,
                                "stage3_max_reuse_distance": reuse, "stage3_defer_reduce": defer,
                                "stage3_retain_params_in_step": defer},
          "optimizer": {"type": "SGD", "params": {"lr": 0.05}}}
    if offload_param:
        ds["zero_optimization"]["offload_param"] = {"device": "cpu", "pin_memory": True}
    eng, _, _, _ = sxe.initialize(model=model, config=ds, **(se or {}))
    g = torch.Generator().manual_seed(7)
    for _ in range(2):
        for _ in range(2):
            ids = torch.randint(0, cfg.vocab_size, (2 * world, 128), generator=g)
            local = ids[rank * 2:(rank + 1) * 2].cuda()
            loss = eng(local, labels=local)
            eng.backward(loss)
            eng.step()
    torch.cuda.synchronize()
    return {"params": C.full_params(eng), "S": getattr(eng.optimizer, "S", None)}


@pytest.mark.parametrize("reuse,defer", [(0, False), (10**12, False), (10**12, True)])
def test_zero3_two_ranks_one_gpu_matches_single_rank(reuse, defer):
    try:
        two = run_dist(_case, 2, reuse, 3, None, defer)
    except RuntimeError as e:
        if "gloo" in str(e).lower() and "cuda" in str(e).lower():
            pytest.skip(f"gloo without GPU tensor support on this build: {str(e)[-200:]}")
        raise
    one = run_dist(_case, 1, reuse)[0]
    assert two[0]["S"] == 2 and one["S"] == 1
    for k, v in one["params"].items():
        a, b = two[0]["params"][k].float(), v.float()
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert rel < 2e-2, (k, rel)
        assert torch.equal(two[0]["params"][k], two[1]["params"][k]), k


@pytest.mark.parametrize("stage", [2, 3])
def test_shuffle_exchange_rr_four_ranks_one_gpu(stage):
    """Shuffle-exchange RR (slice_count=2 -> 2 slices of 2 ranks) on the GPU code path (device-side
    bf16 slice averaging after each step, side streams): every rank ends with identical parameters
    (the CPU tests pin RR == DP-SGD numerically)."""
    se = {"method": "RR", "slice_count": 2}
    four = run_dist(_case, 4, 0, stage, se)
    for k in four[0]["params"]:
        for r in range(1, 4):
            assert torch.equal(four[0]["params"][k], four[r]["params"][k]), (k, r)


def test_shuffle_exchange_rr_with_offload_param_one_gpu():
    """Shuffle-exchange RR with ZeRO-3 offload_param: the bit16 shards live in pinned host memory
    and are averaged across slices through a device pack buffer (H2D, collective, D2H); every rank
    ends identical and equal to the same run without the offload."""
    se = {"method": "RR", "slice_count": 2}
    off = run_dist(_case, 4, 0, 3, se, False, True)
    dev = run_dist(_case, 4, 0, 3, se, False, False)
    for k in off[0]["params"]:
        for r in range(1, 4):
            assert torch.equal(off[0]["params"][k], off[r]["params"][k]), (k, r)
        a, b = off[0]["params"][k].float(), dev[0]["params"][k].float()
        assert ((a - b).norm() / (b.norm() + 1e-12)).item() < 1e-2, k


def _case_init_mem(rank, world):
    os.environ["LOCAL_RANK"] = "0"
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=1024, intermediate_size=4096, num_attention_heads=8,
                       num_key_value_heads=2, vocab_size=8192, num_hidden_layers=8)
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    with sxe.zero.Init(dtype=torch.bfloat16):
        model = LlamaForCausalLM(cfg)
    peak = torch.cuda.max_memory_allocated() - base
    held = torch.cuda.memory_allocated() - base
    layer = sum(p.ds_numel for p in model.layers[0].parameters()) * 2
    return {"peak": peak, "held": held, "full": cfg.num_params() * 2, "layer": layer}


def test_zero_init_gpu_memory_two_ranks():
    """zero.Init on the GPU: each of 2 ranks holds ~half the model after construction and never more
    than its half plus one module's whole parameters (+ allocator slack) while building it."""
    res = run_dist(_case_init_mem, 2)
    for r in res:
        assert r["held"] <= r["full"] / 2 + (4 << 20), r
        assert r["peak"] <= r["full"] / 2 + 2 * max(r["layer"], 8192 * 1024 * 2) + (16 << 20), r
        assert r["peak"] < 0.75 * r["full"], r


def _case_frozen(rank, world, quant):
    os.environ["LOCAL_RANK"] = "0"
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=256, intermediate_size=512, num_attention_heads=2,
                       num_key_value_heads=1, vocab_size=1024, num_hidden_layers=2)
    with sxe.zero.Init(dtype=torch.bfloat16):
        model = LlamaForCausalLM(cfg)
    frozen = C._freeze_lora_style(model)
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2, "bf16": {"enabled": True},
          "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 0,
                                "zero_quantized_nontrainable_weights": quant},
          "optimizer": {"type": "SGD", "params": {"lr": 0.05}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    before = C.full_params(eng)
    g = torch.Generator().manual_seed(7)
    for _ in range(2):
        for _ in range(2):
            ids = torch.randint(0, cfg.vocab_size, (2 * world, 128), generator=g)
            local = ids[rank * 2:(rank + 1) * 2].cuda()
            loss = eng(local, labels=local)
            eng.backward(loss)
            eng.step()
    torch.cuda.synchronize()
    opt = eng.optimizer
    return {"params": C.full_params(eng), "before": before, "frozen": frozen,
            "nq": sum(1 for u in opt.frozen_units if u.frozen_q), "nf": len(opt.frozen_units)}


@pytest.mark.parametrize("quant", [False, True])
def test_zero3_frozen_two_ranks_one_gpu(quant):
    """ZeRO-3 gather-only units for frozen weights on the GPU path (side-stream gathers, int8 shards
    dequantized by the HIP kernel), 2 ranks on one GPU vs the single-rank run."""
    two = run_dist(_case_frozen, 2, quant)
    one = run_dist(_case_frozen, 1, quant)[0]
    assert two[0]["nf"] >= 2 and two[0]["nq"] == (two[0]["nf"] if quant else 0) and one["nq"] == 0
    for k, v in one["params"].items():
        a, b = two[0]["params"][k].float(), v.float()
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert rel < (3e-2 if quant else 2e-2), (k, rel)
        assert torch.equal(two[0]["params"][k], two[1]["params"][k]), k
    for k in two[0]["frozen"]:
        a, b = two[0]["params"][k].float(), two[0]["before"][k].float()
        assert ((a - b).norm() / (b.norm() + 1e-12)).item() < (1e-2 if quant else 1e-6), k
