"""Deferred-completion collectives (comm/comm.py ``set_deferred_completion``, SXE_COMM_DEFER=1).

Every collective's output reads NaN until its consumer synchronises with it (device tensors: the
result lands on the issuing stream after a spin delay; async host ops: at ``Work.wait()``). The
gloo parity suites re-run under it prove that every consumer of an overlapped collective -- ZeRO-1/2
post-step all-gathers and reduce-scatters on the comm stream, ZeRO-3 gathers on the all-gather
stream and reduce-scatters on the reduce stream, Domino's async all-reduces, Gossip's
batch_isend_irecv, ring attention's P2P -- waits before reading, i.e. the code is correct when RCCL
completes asynchronously (which gloo and the single-rank shortcuts never exercise). A negative
control with the ZeRO-3 gather wait removed must fail."""
import os

import pytest
import torch

from . import _dist_cases as C
from .dist_utils import run_dist


def _case_async_unit(rank, world):
    from shuffle_exchange_amd import comm
    comm.set_deferred_completion(True)
    t = torch.full((4,), float(rank + 1))
    w = comm.all_reduce(t, async_op=True)
    before = bool(torch.isnan(t).all())
    w.wait()
    after = t.clone()
    send = torch.full((3,), 7.0 + rank)
    recv = torch.zeros(3)
    peer = 1 - rank
    ops = [comm.P2POp(torch.distributed.isend, send, peer), comm.P2POp(torch.distributed.irecv, recv, peer)]
    works = comm.batch_isend_irecv(ops)
    r_before = bool(torch.isnan(recv).all())
    for x in works:
        x.wait()
    vol = comm.get_comm_volume()
    return {"before": before, "after": after, "r_before": r_before, "recv": recv.clone(), "vol": vol}


def test_deferred_mode_hides_results_until_wait():
    for rank, r in enumerate(run_dist(_case_async_unit, 2)):
        assert r["before"] and r["r_before"]
        assert torch.equal(r["after"], torch.full((4,), 3.0))
        assert torch.equal(r["recv"], torch.full((3,), 7.0 + (1 - rank)))
        assert r["vol"]["all_reduce"] == (1, 16) and r["vol"]["send"] == (1, 12)


@pytest.fixture
def deferred(monkeypatch):
    monkeypatch.setenv("SXE_COMM_DEFER", "1")


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_zero_parity_under_deferred_completion(deferred, stage):
    world, steps, mbs, seq = 2, 2, 2, 16
    ds = {"train_micro_batch_size_per_gpu": mbs, "gradient_accumulation_steps": 2,
          "zero_optimization": {"stage": stage, "stage3_param_persistence_threshold": 0, "reduce_bucket_size": 4000,
                                "overlap_comm": True},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}}
    res = run_dist(C.case_train, world, ds, steps, mbs, seq)
    os.environ["SXE_COMM_DEFER"] = "0"
    ref = run_dist(C.case_train, world, ds, steps, mbs, seq)
    for k, v in ref[0]["params"].items():
        assert torch.isfinite(res[0]["params"][k]).all(), k
        torch.testing.assert_close(res[0]["params"][k], v, rtol=0, atol=0)


@pytest.mark.parametrize("method", ["RR", "Gossip"])
def test_shuffle_exchange_under_deferred_completion(deferred, method):
    world, steps, mbs, seq = 4, 2, 1, 16
    ds = {"train_micro_batch_size_per_gpu": mbs, "zero_optimization": {"stage": 2},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}}
    res = run_dist(C.case_train, world, ds, steps, mbs, seq, {"method": method, "slice_count": 2})
    os.environ["SXE_COMM_DEFER"] = "0"
    ref = run_dist(C.case_train, world, ds, steps, mbs, seq, {"method": method, "slice_count": 2})
    for r in range(world):
        for k, v in ref[r]["params"].items():
            torch.testing.assert_close(res[r]["params"][k], v, rtol=0, atol=0)


def test_domino_async_allreduce_under_deferred_completion(deferred):
    from .test_domino import _case
    res = run_dist(_case, 2, True, 2)
    os.environ["SXE_COMM_DEFER"] = "0"
    ref = run_dist(_case, 2, True, 2)
    assert res[0]["losses"] == ref[0]["losses"]
    for k, v in ref[0]["sd"].items():
        assert torch.equal(res[0]["sd"][k], v), k


def test_ring_attention_under_deferred_completion(deferred):
    from .test_ring_attention import _case_ring
    for r in run_dist(_case_ring, 2, True, "zigzag"):
        for k, v in r.items():
            if torch.is_tensor(v) and v.is_floating_point():
                assert torch.isfinite(v).all(), k


# ------------------------------------------------------------------------------------------- GPU
def _case_gpu(rank, world, stage, defer_reduce, drop_wait, deferred=True):
    os.environ["LOCAL_RANK"] = "0"
    from shuffle_exchange_amd import comm
    comm.set_deferred_completion(deferred, cycles=20_000_000)
    if drop_wait:  # negative control: the ZeRO-3 gather no longer makes the compute stream wait
        from shuffle_exchange_amd.runtime.zero import stage3 as S3

        def fetch_no_wait(self, fg, wait=True):
            for u in fg.units:
                if u.persistent:
                    continue
                if u.state == S3.RELEASED:
                    self._launch_gather(u)
                if wait and u.state == S3.INFLIGHT:
                    u.state = S3.AVAILABLE
        S3.ZeroStage3Optimizer._fetch = fetch_no_wait
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=256, intermediate_size=512, num_attention_heads=2,
                       num_key_value_heads=1, vocab_size=1024, num_hidden_layers=2)
    model = LlamaForCausalLM(cfg)
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2, "bf16": {"enabled": True},
          "zero_optimization": {"stage": stage, "stage3_param_persistence_threshold": 0, "overlap_comm": True,
                                "reduce_bucket_size": 200_000, "stage3_defer_reduce": defer_reduce},
          "optimizer": {"type": "SGD", "params": {"lr": 0.05}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    g = torch.Generator().manual_seed(7)
    losses = []
    for _ in range(2):
        for _ in range(2):
            ids = torch.randint(0, cfg.vocab_size, (2 * world, 128), generator=g)
            local = ids[rank * 2:(rank + 1) * 2].cuda()
            loss = eng(local, labels=local)
            eng.backward(loss)
            eng.step()
            losses.append(float(loss))
    torch.cuda.synchronize()
    return {"params": C.full_params(eng), "losses": losses}


@pytest.mark.gpu
@pytest.mark.parametrize("stage,defer_reduce", [(1, False), (2, False), (3, False), (3, True)])
def test_gpu_side_streams_wait_for_deferred_collectives(stage, defer_reduce):
    """2 ranks on one GPU (gloo), every collective completing ~8 ms late on its issuing stream:
    training stays finite and matches the undeferred run bitwise -- the comm-stream / all-gather /
    reduce-scatter consumers all wait on their events."""
    res = run_dist(_case_gpu, 2, stage, defer_reduce, False)
    ref = run_dist(_case_gpu, 2, stage, defer_reduce, False, False)
    for k, v in ref[0]["params"].items():
        assert torch.isfinite(res[0]["params"][k]).all(), k
        assert torch.equal(res[0]["params"][k], v), k


@pytest.mark.gpu
def test_gpu_missing_gather_wait_is_detected():
    """Negative control: with the wait on the ZeRO-3 gather event removed, the deferred collectives
    are read before they land -> non-finite loss or parameters differing from the reference."""
    bad = run_dist(_case_gpu, 2, 3, False, True)
    ref = run_dist(_case_gpu, 2, 3, False, False, False)
    finite = all(torch.isfinite(torch.tensor(bad[0]["losses"])))
    same = all(torch.equal(bad[0]["params"][k], v) for k, v in ref[0]["params"].items())
    assert not (finite and same)
