"""ZeRO-Offload / ZeRO-Infinity on the GPU path: the host-tier optimizer (C++ CPU Adam fed by the
streamed D2H / H2D staging ring, exact-size pinned buffers) trains a model on the MI355X to the
same parameters as the all-HBM fused HIP Adam; stage 3 with offload_param too; NVMe records."""
import os
import tempfile

import pytest
import torch

from . import _dist_cases as C
from .dist_utils import run_dist

pytestmark = pytest.mark.gpu


def _case(rank, world, stage, offload, nvme_dir=None):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=256, intermediate_size=512, num_attention_heads=2,
                       num_key_value_heads=1, vocab_size=1024, num_hidden_layers=2)
    with sxe.zero.Init(dtype=torch.bfloat16):
        model = LlamaForCausalLM(cfg)
    zc = {"stage": stage, "stage3_param_persistence_threshold": 0}
    if offload in ("cpu", "twin_flow", "cpu_opt"):
        zc["offload_optimizer"] = {"device": "cpu", "pin_memory": True, "ratio": 0.5 if offload == "twin_flow" else 1.0}
        if stage == 3 and offload != "cpu_opt":
            zc["offload_param"] = {"device": "cpu", "pin_memory": True}
    elif offload == "nvme":
        zc["offload_optimizer"] = {"device": "nvme", "nvme_path": nvme_dir}
    elif offload == "nvme_params":  # ZeRO-Infinity: parameter shards AND optimizer state on NVMe
        zc["offload_optimizer"] = {"device": "nvme", "nvme_path": nvme_dir}
        zc["offload_param"] = {"device": "nvme", "nvme_path": nvme_dir, "buffer_count": 3}
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2, "bf16": {"enabled": True},
          "gradient_clipping": 1.0, "zero_optimization": zc,
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-3, "weight_decay": 0.01}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    g = torch.Generator().manual_seed(7)
    for _ in range(3):
        for _ in range(2):
            ids = torch.randint(0, cfg.vocab_size, (2, 128), generator=g).cuda()
            loss = eng(ids, labels=ids)
            eng.backward(loss)
            eng.step()
    torch.cuda.synchronize()
    return C.full_params(eng)


@pytest.mark.parametrize("stage,offload", [(2, "cpu"), (3, "cpu"), (3, "nvme"), (3, "twin_flow"),
                                           (3, "nvme_params")])
def test_offload_matches_hbm_adam(stage, offload):
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        off = run_dist(_case, 1, stage, offload, d)[0]
    ref = run_dist(_case, 1, stage, "none")[0]
    for k, v in ref.items():
        a, b = off[k].float(), v.float()
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert rel < 5e-3, (k, rel)


@pytest.mark.parametrize("stage", [2, 3])
def test_offload_piecewise_d2h_matches_hbm_adam(stage, monkeypatch):
    """The host update walking a unit's gradient in D2H pieces as they land (SXE_OFFLOAD_D2H_PIECE,
    here 4096 elements: dozens of pieces per unit) trains to the same parameters."""
    monkeypatch.setenv("SXE_OFFLOAD_D2H_PIECE", "4096")
    off = run_dist(_case, 1, stage, "cpu")[0]
    monkeypatch.delenv("SXE_OFFLOAD_D2H_PIECE")
    ref = run_dist(_case, 1, stage, "none")[0]
    for k, v in ref.items():
        a, b = off[k].float(), v.float()
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert rel < 5e-3, (k, rel)


@pytest.mark.parametrize("window,kernel", [("0", "0"), ("2", "0"), ("2", "1"), ("0", "1")])
def test_offload_async_copy_schedules_match_sync(window, kernel, monkeypatch):
    """The asynchronous host tier (SXE_OFFLOAD_ASYNC) with a windowed gradient-D2H issue
    (SXE_OFFLOAD_ASYNC_WINDOW) and / or kernel-driven H2D of the updated shards
    (SXE_OFFLOAD_H2D_KERNEL, host_mem.hip h2d_copy_) trains to bit-identical parameters as the
    synchronous tier: same kernels, same order, only the copy scheduling differs."""
    ref = run_dist(_case, 1, 3, "cpu_opt")[0]
    monkeypatch.setenv("SXE_OFFLOAD_ASYNC", "1")
    monkeypatch.setenv("SXE_OFFLOAD_ASYNC_WINDOW", window)
    monkeypatch.setenv("SXE_OFFLOAD_H2D_KERNEL", kernel)
    got = run_dist(_case, 1, 3, "cpu_opt")[0]
    for k, v in ref.items():
        assert torch.equal(got[k], v), k


def test_h2d_copy_kernel():
    from shuffle_exchange_amd.ops import native
    from shuffle_exchange_amd.runtime.zero.offload import pinned_empty
    native.require_hip()
    src = pinned_empty(3 * 2**20 + 8, torch.bfloat16)
    src.copy_(torch.randn(src.numel()).bfloat16())
    dst = torch.empty(src.numel(), dtype=torch.bfloat16, device="cuda")
    torch.ops.sxe.h2d_copy_(dst, src)
    torch.cuda.synchronize()
    assert torch.equal(dst.cpu(), src)
