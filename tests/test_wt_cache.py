"""Transposed-weight cache of the data-gradient GEMMs (ops/linear.py ``_transposed_weight``): the
transposes of a weight are reused across the micro-steps of one optimizer step, never across a
weight change (optimizer step, checkpoint load, LoRA fuse), never for a different tensor that
reuses an id, and never beyond the byte cap."""
import pytest
import torch

from shuffle_exchange_amd.ops import linear as L


@pytest.fixture
def counting(monkeypatch):
    calls = []

    def fake(t):
        calls.append(t)
        return t.t().contiguous()
    monkeypatch.setattr(L, "_transpose16", fake)
    monkeypatch.setattr(L, "WT_CACHE", True)
    L.invalidate_transposed_weights()
    yield calls
    L.invalidate_transposed_weights()


def test_cache_hits_until_invalidated(counting):
    w = torch.nn.Parameter(torch.randn(64, 32))
    a = L._transposed_weight(w)
    b = L._transposed_weight(w)
    assert a is b and len(counting) == 1 and torch.equal(a, w.t())
    L.invalidate_transposed_weights()
    with torch.no_grad():
        w.mul_(2)
    c = L._transposed_weight(w)
    assert len(counting) == 2 and torch.equal(c, w.t())


def test_cache_respects_identity_and_cap(counting, monkeypatch):
    w1 = torch.nn.Parameter(torch.randn(64, 32))
    L._transposed_weight(w1)
    w2 = torch.nn.Parameter(torch.randn(64, 32))
    assert torch.equal(L._transposed_weight(w2), w2.t())  # another tensor: its own transpose
    monkeypatch.setattr(L, "WT_CACHE_MAX_BYTES", 0)
    L.invalidate_transposed_weights()
    w3 = torch.nn.Parameter(torch.randn(8, 8))
    L._transposed_weight(w3)
    L._transposed_weight(w3)
    assert sum(1 for t in counting if t is w3) == 2  # over the cap: nothing is kept


def test_inplace_write_or_rebinding_misses(counting):
    """A write through the Parameter (version bump) or a rebind to other storage (ZeRO-3 gathers
    into a new buffer) is a miss even without an explicit invalidation."""
    w = torch.nn.Parameter(torch.randn(64, 32))
    L._transposed_weight(w)
    with torch.no_grad():
        w.add_(1.0)
    assert torch.equal(L._transposed_weight(w), w.t()) and len(counting) == 2
    w.data = torch.randn(64, 32)
    assert torch.equal(L._transposed_weight(w), w.t()) and len(counting) == 3
    assert L.transposed_weight_cache_bytes() == 64 * 32 * 4  # the stale entry's bytes were released


def _case_writers(rank, world):
    """Every bit16 weight writer outside the optimizer step drops the cache."""
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.ops import linear as lin
    from shuffle_exchange_amd.utils.tensor_fragment import safe_set_full_fp32_param, safe_set_local_fp32_param
    model = torch.nn.Linear(8, 8)
    ds = {"train_micro_batch_size_per_gpu": 1, "gradient_accumulation_steps": 2, "zero_optimization": {"stage": 1},
          "optimizer": {"type": "SGD", "params": {"lr": 0.1}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds, method="RR", slice_count=1)
    out = {}
    for name, fn in (("synchronization", eng.synchronization),
                     ("safe_set_full", lambda: safe_set_full_fp32_param(model.weight, torch.ones(8, 8))),
                     ("safe_set_local", lambda: safe_set_local_fp32_param(model.weight, torch.ones(64)))):
        lin._wt_cache[id(model.weight)] = (None, model.weight)
        fn()
        out[name] = len(lin._wt_cache)
    return out


def test_weight_writers_invalidate():
    from .dist_utils import run_dist
    (r,) = run_dist(_case_writers, 1)
    assert r == {"synchronization": 0, "safe_set_full": 0, "safe_set_local": 0}


def _case_engine(rank, world):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.ops import linear as lin
    seen = []
    for gas in (1, 2):
        model = torch.nn.Linear(8, 8)
        ds = {"train_micro_batch_size_per_gpu": 1, "gradient_accumulation_steps": gas,
              "optimizer": {"type": "SGD", "params": {"lr": 0.1}}}
        eng, _, _, _ = sxe.initialize(model=model, config=ds)
        seen.append(lin.WT_CACHE)
    w = torch.nn.Parameter(torch.randn(4, 4))
    lin._wt_cache[id(w)] = (None, w)
    for _ in range(2):
        eng.backward(eng(torch.randn(1, 8)).sum())
        eng.step()
    return {"seen": seen, "left": len(lin._wt_cache)}


def test_engine_enables_for_accumulation_and_clears_on_step():
    from .dist_utils import run_dist
    (r,) = run_dist(_case_engine, 1)
    assert r["seen"] == [False, True]
    assert r["left"] == 0  # the optimizer step invalidated the cache


@pytest.mark.gpu
def test_gpu_accumulation_with_cache_matches_uncached():
    """bf16 Llama layer at Llama-3-8B width (weights above the transposed-dgrad threshold), 2
    micro-steps x 2 optimizer steps: cached and recomputed transposes give bit-identical weights."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config

    def run(cache):
        torch.manual_seed(0)
        cfg = llama_config("llama3-8b", num_hidden_layers=1, vocab_size=4096)
        model = LlamaForCausalLM(cfg).to("cuda", torch.bfloat16)
        ds = {"train_micro_batch_size_per_gpu": 1, "gradient_accumulation_steps": 2, "bf16": {"enabled": True},
              "zero_optimization": {"stage": 1}, "optimizer": {"type": "AdamW", "params": {"lr": 1e-4}}}
        eng, _, _, _ = sxe.initialize(model=model, config=ds)
        L.WT_CACHE = cache
        g = torch.Generator(device="cuda").manual_seed(1)
        hits = 0
        for _ in range(4):
            ids = torch.randint(0, 4096, (1, 2048), device="cuda", generator=g)
            eng.backward(eng(ids, labels=ids))
            hits = max(hits, len(L._wt_cache))
            eng.step()
        return [p.detach().clone() for p in model.parameters()], hits

    a, hits = run(True)
    b, _ = run(False)
    assert hits > 0
    for x, y in zip(a, b):
        assert torch.equal(x, y)
