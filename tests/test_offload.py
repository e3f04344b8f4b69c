"""ZeRO-Offload / ZeRO-Infinity on gloo (world 2): optimizer state on the host (C++ CPU Adam) or
NVMe (C++ AIO engine), parameter offload for ZeRO-3; all must train to the same parameters as the
single-process torch.optim reference. Plus the AIO engine itself and offloaded checkpoints."""
import os

import pytest
import torch

from ._dist_cases import case_train, reference_train
from .dist_utils import run_dist

ADAM = {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.01}}


def _cfg(stage, device="cpu", nvme_path=None, offload_param=False, clip=0.0, ratio=1.0, param_device="cpu",
         buffer_count=5):
    z = {"stage": stage, "reduce_bucket_size": 20000,
         "offload_optimizer": {"device": device, "nvme_path": nvme_path, "pin_memory": True, "ratio": ratio}}
    if offload_param:
        z["offload_param"] = {"device": param_device, "pin_memory": True, "nvme_path": nvme_path,
                              "buffer_count": buffer_count}
        z["stage3_param_persistence_threshold"] = 10
    return {"train_micro_batch_size_per_gpu": 2, "zero_optimization": z, "optimizer": ADAM,
            "gradient_clipping": clip}


def _check(res, ref, tol=1e-4):
    # Adam amplifies summation-order noise on near-zero gradient entries; compare like test_zero_dist
    for r in res:
        for k, v in ref.items():
            d = (r["params"][k] - v).abs().max().item()
            assert d <= tol * max(1.0, v.abs().max().item()), f"{k}: {d}"


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_cpu_offload_matches_reference(stage):
    res = run_dist(case_train, 2, _cfg(stage), 3, 2, 16)
    _check(res, reference_train(ADAM, 3, 2, 2, 16))


def test_cpu_offload_with_clipping():
    res = run_dist(case_train, 2, _cfg(2, clip=1.0), 3, 2, 16)
    ref = reference_train(ADAM, 3, 2, 2, 16, clip=1.0)
    for r in res:
        for k, v in ref.items():
            assert (r["params"][k] - v).norm() / v.norm() < 1e-3, k


def test_nvme_offload_matches_reference(tmp_path):
    res = run_dist(case_train, 2, _cfg(2, "nvme", str(tmp_path)), 3, 2, 16)
    _check(res, reference_train(ADAM, 3, 2, 2, 16))
    assert any(f.endswith(".swp") for _, _, fs in os.walk(tmp_path) for f in fs)


def test_zero3_param_and_optimizer_offload(tmp_path):
    res = run_dist(case_train, 2, _cfg(3, "nvme", str(tmp_path), offload_param=True), 3, 2, 16)
    _check(res, reference_train(ADAM, 3, 2, 2, 16))


def _case_nvme_params(rank, world, nvme, opt_device, buffer_count):
    import shuffle_exchange_amd as sxe
    from ._dist_cases import full_params, global_batches, tiny_llama
    model, cfg = tiny_llama(0)
    ds = _cfg(3, opt_device, nvme, offload_param=True, param_device="nvme", buffer_count=buffer_count)
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    opt = eng.optimizer
    swapped = [u for us in opt.units for u in us if u.swap is not None]
    for b in global_batches(cfg, world, 2, 16, 3):
        local = b[rank * 2:(rank + 1) * 2]
        loss = eng(local, labels=local)
        eng.backward(loss)
        eng.step()
    sw = opt.pswap
    return {"params": full_params(eng), "n_swapped": len(swapped), "n_units": sum(len(us) for us in opt.units),
            "read": sw.bytes_read, "written": sw.bytes_written, "file": sw.file,
            "file_bytes": os.path.getsize(sw.file), "host_shards": sum(u._shard is not None for u in swapped)}


@pytest.mark.parametrize("opt_device,buffer_count", [("cpu", 2), ("nvme", 3)])
def test_zero3_nvme_parameter_tier(tmp_path, opt_device, buffer_count):
    """ZeRO-Infinity parameter swap (reference swap_tensor/partitioned_param_swapper.py:37): every
    non-persistent unit shard lives in the swap file (no host copy), is read back through a pool of
    `buffer_count` pinned buffers (2 forces eviction of dirty and in-flight buffers), and training
    matches the single-process reference."""
    res = run_dist(_case_nvme_params, 2, str(tmp_path), opt_device, buffer_count)
    _check(res, reference_train(ADAM, 3, 2, 2, 16))
    for r in res:
        assert r["n_swapped"] >= 2 and r["host_shards"] == 0
        # every forward + backward gather re-reads the shards; every step writes them back
        assert r["read"] > 3 * r["file_bytes"] and r["written"] >= 3 * r["file_bytes"]


def _case_nvme_param_no_host_opt(rank, world, nvme):
    import shuffle_exchange_amd as sxe
    from ._dist_cases import tiny_llama
    model, _ = tiny_llama(0)
    z = {"stage": 3, "offload_param": {"device": "nvme", "nvme_path": nvme}}
    try:
        sxe.initialize(model=model, config={"train_micro_batch_size_per_gpu": 1, "zero_optimization": z,
                                            "optimizer": ADAM})
    except ValueError as e:
        return str(e)
    return ""


def test_nvme_param_offload_needs_host_optimizer(tmp_path):
    """offload_param nvme is real or raises -- never a silent fallback to host memory."""
    assert "offload_optimizer" in run_dist(_case_nvme_param_no_host_opt, 1, str(tmp_path))[0]


@pytest.mark.parametrize("stage", [2, 3])
@pytest.mark.parametrize("ratio", [0.0, 0.4])
def test_twin_flow_partial_offload_matches_reference(stage, ratio):
    """offload_optimizer.ratio < 1 (Twin-Flow): part of every param group is stepped on the host,
    the rest in device memory; together they equal one AdamW over the global batch."""
    res = run_dist(case_train, 2, _cfg(stage, ratio=ratio), 3, 2, 16)
    _check(res, reference_train(ADAM, 3, 2, 2, 16))


def test_split_param_groups_by_ratio():
    from shuffle_exchange_amd.runtime.zero.offload import split_param_groups
    ps = [torch.nn.Parameter(torch.zeros(n)) for n in (10, 30, 20, 40)]
    opt = torch.optim.AdamW([{"params": ps[:3], "weight_decay": 0.1}, {"params": ps[3:], "weight_decay": 0.0}])
    split_param_groups(opt, 0.5)
    got = [([p.numel() for p in g["params"]], g["sxe_offload"], g["weight_decay"]) for g in opt.param_groups]
    assert got == [([10, 30], True, 0.1), ([20], False, 0.1), ([40], True, 0.0)]


def _case_offload_ckpt(rank, world, device, nvme, ckdir, ratio=1.0, nvme_params=False):
    import shuffle_exchange_amd as sxe
    from ._dist_cases import full_params, global_batches, tiny_llama
    cfg_a = (_cfg(3, device, nvme, offload_param=True, param_device="nvme", buffer_count=2) if nvme_params
             else _cfg(2, device, nvme, ratio=ratio))
    model, cfg = tiny_llama(0)
    eng, _, _, _ = sxe.initialize(model=model, config=cfg_a)
    batches = global_batches(cfg, world, 2, 16, 4)

    def run(e, bs):
        for b in bs:
            local = b[rank * 2:(rank + 1) * 2]
            loss = e(local, labels=local)
            e.backward(loss)
            e.step()
    run(eng, batches[:2])
    eng.save_checkpoint(ckdir, tag="t")
    run(eng, batches[2:])
    want = full_params(eng)
    model2, _ = tiny_llama(5)
    eng2, _, _, _ = sxe.initialize(model=model2, config=cfg_a)
    eng2.load_checkpoint(ckdir, tag="t")
    run(eng2, batches[2:])
    got = full_params(eng2)
    return {"ok": all(torch.allclose(want[k], got[k], atol=1e-6) for k in want)}


@pytest.mark.parametrize("device,ratio", [("cpu", 1.0), ("nvme", 1.0), ("cpu", 0.5)])
def test_offload_checkpoint_resume(tmp_path, device, ratio):
    nv = str(tmp_path / "nvme") if device == "nvme" else None
    res = run_dist(_case_offload_ckpt, 2, device, nv, str(tmp_path / "ck"), ratio)
    assert all(r["ok"] for r in res)


def test_nvme_param_tier_checkpoint_resume(tmp_path):
    """Save / load with the parameter shards on NVMe: the resumed run continues bit-exactly."""
    res = run_dist(_case_offload_ckpt, 2, "cpu", str(tmp_path / "nvme"), str(tmp_path / "ck"), 1.0, True)
    assert all(r["ok"] for r in res)


def test_aio_roundtrip(tmp_path):
    from shuffle_exchange_amd.ops.aio import AsyncIOHandle
    h = AsyncIOHandle(block_size=1 << 16, intra_op_parallelism=3)
    xs = [torch.randn(n) for n in (1, 4096, 1_000_003)]
    ids = [h.async_pwrite(x, tmp_path / f"{i}.bin") for i, x in enumerate(xs)]
    h.wait_request(ids[-1]) if hasattr(h, "wait_request") else None
    assert h.wait() >= 0
    ys = [torch.empty_like(x) for x in xs]
    for i, y in enumerate(ys):
        h.async_pread(y, tmp_path / f"{i}.bin")
    h.wait()
    assert all(torch.equal(x, y) for x, y in zip(xs, ys))
    # file offsets
    big = torch.arange(8192, dtype=torch.float32)
    h.sync_pwrite(big[:4096], tmp_path / "o.bin", 0)
    h.sync_pwrite(big[4096:], tmp_path / "o.bin", 4096 * 4)
    back = torch.empty(4096)
    h.sync_pread(back, tmp_path / "o.bin", 4096 * 4)
    assert torch.equal(back, big[4096:])
    with pytest.raises(RuntimeError):
        h.sync_pread(torch.empty(10), tmp_path / "missing.bin")


def test_client_scheduler_survives_twin_flow_split():
    """A torch LR scheduler built on the client optimizer before initialize() keeps driving every
    split part of its groups (ADVICE: strict zip over base_lrs raised after the split)."""
    from shuffle_exchange_amd.runtime.zero.offload import expand_scheduler_groups, split_param_groups
    ps = [torch.nn.Parameter(torch.zeros(n)) for n in (10, 30, 20, 40)]
    opt = torch.optim.AdamW([{"params": ps[:3], "lr": 1.0}, {"params": ps[3:], "lr": 2.0}])
    sch = torch.optim.lr_scheduler.LambdaLR(opt, [lambda s: 0.5 ** s, lambda s: 0.1 * s])
    split_param_groups(opt, 0.5)
    expand_scheduler_groups(sch, opt)
    for _ in range(2):
        opt.step()
        sch.step()
    assert [g["lr"] for g in opt.param_groups] == [0.25, 0.25, 2.0 * 0.2]


def _case_async(rank, world, async_on, gas, clip):
    os.environ["SXE_OFFLOAD_ASYNC"] = "1" if async_on else "0"
    os.environ["SXE_OFFLOAD_TRACE"] = "1"
    import shuffle_exchange_amd as sxe
    from ._dist_cases import global_batches, tiny_llama, full_params
    model, cfg = tiny_llama(0)
    ds = _cfg(3, clip=clip)
    ds["gradient_accumulation_steps"] = gas
    ds["zero_optimization"]["stage3_param_persistence_threshold"] = 0
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    hs = eng.optimizer.host_step
    for b in global_batches(cfg, world * gas, 2, 16, 3):
        for m in range(gas):
            part = b[m * 2 * world:(m + 1) * 2 * world]
            x = part[rank * 2:(rank + 1) * 2]
            eng.backward(eng(x, labels=x))
            eng.step()
    was_async = hs._worker is not None or bool(hs.trace and "waits" in hs.trace[-1])
    return {"params": full_params(eng), "async": was_async}


@pytest.mark.parametrize("gas,clip", [(1, 0.0), (2, 1.0)])
def test_async_host_update_is_bit_identical(gas, clip):
    """ZeRO-3 + CPU optimizer offload: the asynchronous host update (worker thread, per-unit waits in
    the next forward) gives exactly the parameters of the synchronous one."""
    a = run_dist(_case_async, 2, True, gas, clip)
    s = run_dist(_case_async, 2, False, gas, clip)
    assert a[0]["async"] and not s[0]["async"]
    for ra, rs in zip(a, s):
        for k in rs["params"]:
            assert torch.equal(ra["params"][k], rs["params"][k]), k
