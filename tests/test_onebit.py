"""1-bit compressed communication (gloo): packing/error-feedback invariants, compressed all-reduce
converging to the true mean under error feedback, and the 1-bit Adam / 0/1 Adam / 1-bit LAMB
optimizers on the engine (warm-up == uncompressed single-process run; compressed phase keeps
replicas identical and trains)."""
import pytest
import torch

from .dist_utils import run_dist


def test_pack_ef_invariant():
    from shuffle_exchange_amd.runtime.comm.compressed import _pack_ef, _unpack_avg
    x = torch.randn(64)
    err = torch.zeros(64)
    scale = (x.norm() / 8).reshape(1)
    packed = _pack_ef(x, err, scale)
    out = torch.empty(64)
    _unpack_avg(packed.view(1, 8), scale, out)
    assert torch.allclose(out + err, x, atol=1e-6)  # decoded + error == input (exact EF split)
    assert torch.equal(out > 0, x >= 0)


def _case_allreduce(rank, world, iters):
    from shuffle_exchange_amd.runtime.comm.compressed import CompressedBackend
    be = CompressedBackend()
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(1000, generator=g)
    we, se = be.make_errors(x.numel(), x.device)
    acc = torch.zeros_like(x)
    first = None
    for i in range(iters):
        y = x.clone()
        be.compressed_allreduce(y, we, se)
        acc += y
        if first is None:
            first = y.clone()
    xs = [torch.empty_like(x) for _ in range(world)]
    torch.distributed.all_gather(xs, x)
    mean = torch.stack(xs).mean(0)
    return {"first_cos": float(torch.nn.functional.cosine_similarity(first, mean, dim=0)),
            "avg_err": float((acc / iters - mean).norm() / mean.norm()), "first": first}


def test_compressed_allreduce_error_feedback():
    res = run_dist(_case_allreduce, 4, 200)
    for r in res:
        assert r["first_cos"] > 0.5
        assert r["avg_err"] < 0.05
    for r in res[1:]:
        assert torch.equal(r["first"], res[0]["first"])  # every rank decodes the same tensor


def _case_engine(rank, world, name, freeze, steps, lr=1e-3, fixed=False):
    import shuffle_exchange_amd as sxe
    from ._dist_cases import full_params, global_batches, tiny_llama
    model, cfg = tiny_llama(0)
    params = {"lr": lr}
    if name == "ZeroOneAdam":
        params.update(var_freeze_step=freeze, var_update_scaler=16, local_step_scaler=1000, local_step_clipper=2)
    else:
        params["freeze_step"] = freeze
    ds = {"train_micro_batch_size_per_gpu": 2, "zero_optimization": {"stage": 0},
          "optimizer": {"type": name, "params": params}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    losses = []
    bs = global_batches(cfg, world, 2, 16, steps)
    for b in ([bs[0]] * steps if fixed else bs):
        local = b[rank * 2:(rank + 1) * 2]
        loss = eng(local, labels=local)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    return {"params": full_params(eng), "losses": losses, "active": eng.basic_optimizer.comm_active}


def _reference(name, freeze, steps, world):
    from shuffle_exchange_amd.runtime.fp16.onebit import OnebitAdam, OnebitLamb
    from ._dist_cases import global_batches, tiny_llama
    model, cfg = tiny_llama(0)
    cls = {"OneBitAdam": OnebitAdam, "OneBitLamb": OnebitLamb}[name]
    opt = cls(model.parameters(), lr=1e-3, freeze_step=freeze)
    for b in global_batches(cfg, world, 2, 16, steps):
        loss = model(b, labels=b)
        opt.zero_grad()
        loss.backward()
        opt.step()
    return {n: p.detach().clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("name", ["OneBitAdam", "OneBitLamb"])
def test_onebit_warmup_equals_uncompressed(name):
    res = run_dist(_case_engine, 2, name, 1000, 3)
    ref = _reference(name, 1000, 3, 2)
    for r in res:
        assert not r["active"]
        for k, v in ref.items():
            assert torch.allclose(r["params"][k], v, atol=2e-5), k


@pytest.mark.parametrize("name", ["OneBitAdam", "ZeroOneAdam", "OneBitLamb"])
def test_onebit_compressed_phase(name):
    res = run_dist(_case_engine, 2, name, 4, 12, 1e-3, True)  # memorise one batch
    for r in res:
        assert r["active"]
        assert all(l == l for l in r["losses"])
    for k, v in res[0]["params"].items():
        assert torch.allclose(res[1]["params"][k], v, atol=1e-6), k  # replicas stay identical
    assert res[0]["losses"][-1] < res[0]["losses"][0]
