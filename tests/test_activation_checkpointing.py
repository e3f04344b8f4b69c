"""Activation checkpointing: recompute gives identical grads (incl. dropout via RNG replay), the
named RNG tracker, host offload of saved tensors, and TP-partitioned saved activations (gloo)."""
import torch

from .dist_utils import run_dist


def _block():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.GELU(), torch.nn.Dropout(0.3),
                               torch.nn.Linear(128, 64))


def _grads(use_ckpt, **cfg):
    from shuffle_exchange_amd.runtime.activation_checkpointing import checkpointing as ac
    ac.configure(None, **cfg)
    m = _block()
    x = torch.randn(64, 64, generator=torch.Generator().manual_seed(1), requires_grad=True)
    torch.manual_seed(42)
    y = ac.checkpoint(m, x) if use_ckpt else m(x)
    y.square().sum().backward()
    out = [x.grad.clone()] + [p.grad.clone() for p in m.parameters()]
    ac.configure(None, partition_activations=False, checkpoint_in_cpu=False)
    return out


def test_checkpoint_matches_plain_with_dropout():
    a = _grads(False)
    b = _grads(True)
    for x, y in zip(a, b):
        assert torch.allclose(x, y, atol=1e-6)


def test_rng_tracker_fork_is_reproducible():
    from shuffle_exchange_amd.runtime.activation_checkpointing.checkpointing import CudaRNGStatesTracker
    t = CudaRNGStatesTracker()
    t.add("mp", 123)
    base = torch.get_rng_state()
    with t.fork("mp"):
        a = torch.rand(4)
    with t.fork("mp"):
        b = torch.rand(4)
    assert not torch.equal(a, b)  # the tracked state advanced
    assert torch.equal(torch.get_rng_state(), base)  # the default stream is untouched
    t2 = CudaRNGStatesTracker()
    t2.add("mp", 123)
    with t2.fork("mp"):
        a2 = torch.rand(4)
    assert torch.equal(a, a2)


def _case_partitioned(rank, world):
    from shuffle_exchange_amd.parallel import groups
    from shuffle_exchange_amd.runtime.activation_checkpointing import checkpointing as ac
    groups.initialize(tensor_parallel_size=world)
    plain = _grads(False)
    part = _grads(True, partition_activations=True)
    return {"ok": all(torch.allclose(x, y, atol=1e-6) for x, y in zip(plain, part))}


def test_partition_activations_tp2():
    assert all(r["ok"] for r in run_dist(_case_partitioned, 2))


def _case_partitioned_counts(rank, world):
    """The partitioned path really stores 1/tp of the input."""
    from shuffle_exchange_amd.parallel import groups
    from shuffle_exchange_amd.runtime.activation_checkpointing import checkpointing as ac
    groups.initialize(tensor_parallel_size=world)
    p = ac._pack_partition(torch.randn(64, 64))
    return {"part": p.part.numel()}


def test_partition_stores_fraction():
    for r in run_dist(_case_partitioned_counts, 2):
        assert r["part"] == 64 * 64 // 2


def test_llama_ac_policies_give_identical_gradients():
    """Llama activation checkpointing policies (models/llama.py ac_policy): whole-layer ('full') and
    MLP-only ('mlp', keeps the attention outputs) recompute reproduce the un-checkpointed loss and
    gradients exactly."""
    import pytest
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    ids = torch.randint(0, 512, (2, 32), generator=torch.Generator().manual_seed(0))
    out = {}
    for name, kw in (("none", {}), ("full", {"activation_checkpointing": True}),
                     ("mlp", {"activation_checkpointing": True, "ac_policy": "mlp"})):
        torch.manual_seed(0)
        model = LlamaForCausalLM(llama_config("llama-tiny", **kw)).train()
        loss = model(ids, labels=ids)
        loss.backward()
        out[name] = (loss.detach(), [p.grad.clone() for p in model.parameters()])
    assert model.layers[0].ckpt_mlp
    for name in ("full", "mlp"):
        assert torch.equal(out[name][0], out["none"][0])
        for a, b in zip(out[name][1], out["none"][1]):
            torch.testing.assert_close(a, b, rtol=0, atol=0)
    with pytest.raises(ValueError):
        llama_config("llama-tiny", ac_policy="attention")
