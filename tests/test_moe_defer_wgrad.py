"""Deferred expert weight gradients (moe/experts.py ``_GroupedMM`` + ZeRO-1/2 ``_grad_defer``): before
the accumulation boundary a single-rank expert unit keeps (x, dy) and writes its weight gradient once
at the boundary over all micro-steps' tokens. The result must equal writing every micro-step."""
import torch

from . import _dist_cases as C
from .dist_utils import run_dist


class _Target:
    """A stand-in for the optimizer's direct weight-gradient hooks of one parameter."""

    def __init__(self, w, boundary):
        self.buf = torch.full(w.shape, float("nan"))
        self.valid, self.done, self.boundary = False, 0, boundary
        w._sxe_grad_target = lambda p: (self.buf, self.valid)
        w._sxe_grad_done = self._done
        w._sxe_grad_defer = lambda p: not self.boundary[0]

    def _done(self, p):
        self.valid = True
        self.done += 1


def test_grouped_mm_defers_until_the_boundary():
    from shuffle_exchange_amd.moe import experts as E
    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(3, 16, 24))
    boundary = [False]
    t = _Target(w, boundary)
    xs = [torch.randn(3, 5, 16, requires_grad=True) for _ in range(3)]
    gs = [torch.randn(3, 5, 24) for _ in range(3)]
    for k, (x, g) in enumerate(zip(xs, gs)):
        boundary[0] = k == 2
        E.grouped_mm(x, w).backward(g)
        assert t.done == (1 if k == 2 else 0)
        torch.testing.assert_close(x.grad, torch.einsum("ecn,ekn->eck", g, w.detach()))
    ref = sum(torch.einsum("eck,ecn->ekn", x.detach(), g) for x, g in zip(xs, gs))
    torch.testing.assert_close(t.buf, ref)
    assert "_sxe_wstash" not in w.__dict__


def test_flush_writes_a_stash_no_boundary_backward_consumed():
    from shuffle_exchange_amd.moe import experts as E
    torch.manual_seed(1)
    w = torch.nn.Parameter(torch.randn(2, 8, 8))
    boundary = [False]
    t = _Target(w, boundary)
    x, g = torch.randn(2, 4, 8), torch.randn(2, 4, 8)
    E.grouped_mm(x, w).backward(g)
    assert t.done == 0 and len(w._sxe_wstash) == 1
    E.flush_deferred_wgrad(w)
    assert t.done == 1 and "_sxe_wstash" not in w.__dict__
    torch.testing.assert_close(t.buf, torch.einsum("eck,ecn->ekn", x, g))


def _case_mixtral_gas(rank, world, defer):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models.mixtral import MixtralForCausalLM, mixtral_config
    from shuffle_exchange_amd.moe import experts as E
    E.DEFER_WGRAD = defer
    torch.manual_seed(0)
    cfg = mixtral_config("mixtral-tiny", ep_size=world)
    model = MixtralForCausalLM(cfg)
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2, "zero_optimization": {"stage": 2},
          "optimizer": {"type": "AdamW", "params": {"lr": 3e-3}}, "gradient_clipping": 1.0}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    g = torch.Generator().manual_seed(11 + rank)
    for _ in range(2 * 2):
        ids = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
        loss = eng(ids, labels=ids)
        eng.backward(loss)
        eng.step()
    stashed = sum(1 for p in model.parameters() if p.__dict__.get("_sxe_wstash"))
    return {"params": {n: p.detach().float().clone() for n, p in model.named_parameters()}, "stashed": stashed}


def test_mixtral_zero2_gas2_deferred_equals_per_micro_step():
    """Mixtral-tiny, ZeRO-2, GAS 2, expert parallel over 2 gloo ranks (expert units are single-rank):
    deferred expert weight gradients == per-micro-step writes (fp32 sums in another order)."""
    on = run_dist(_case_mixtral_gas, 2, True)
    off = run_dist(_case_mixtral_gas, 2, False)
    for a, b in zip(on, off):
        assert a["stashed"] == 0
        for k, v in b["params"].items():
            torch.testing.assert_close(a["params"][k], v, rtol=1e-4, atol=1e-5)
