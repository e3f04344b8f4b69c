"""MoE: routing semantics, sparse dispatch == dense reference, expert-parallel all-to-all == single
process, and Mixtral training through the engine (gloo, CPU)."""
import pytest
import torch
import torch.nn.functional as F

from . import _dist_cases as C
from .dist_utils import run_dist


def _dense_reference(moe, x):
    """out[t] = sum_k gate_k * expert_{e_k}(x[t]) with the same routing decision."""
    layer = moe.deepspeed_moe
    xt = x.reshape(-1, x.shape[-1])
    r = layer.gate(xt)
    ex = layer.experts
    out = torch.zeros_like(xt)
    for t in range(xt.shape[0]):
        for j in range(r.expert.shape[1]):
            if not bool(r.keep[t, j]):
                continue
            e = int(r.expert[t, j])
            h = F.silu(xt[t] @ ex.w_gate_up[e][:, :ex.w_down.shape[1]]) * (xt[t] @ ex.w_gate_up[e][:, ex.w_down.shape[1]:])
            out[t] += r.weight[t, j] * (h @ ex.w_down[e])
    return out.view_as(x)


@pytest.mark.parametrize("k", [1, 2, 3])
def test_moe_matches_dense_reference(k):
    from shuffle_exchange_amd.moe import MoE
    from shuffle_exchange_amd.parallel import groups
    torch.manual_seed(0)
    groups.reset()
    moe = MoE(32, None, num_experts=4, ep_size=1, k=k, capacity_factor=4.0, min_capacity=64, use_rts=False,
              top2_2nd_expert_sampling=False, intermediate_size=48)
    moe._groups_ready = True
    x = torch.randn(2, 10, 32)
    torch.manual_seed(5)
    out, l_aux, counts = moe(x)
    torch.manual_seed(5)
    ref = _dense_reference(moe, x)
    assert torch.allclose(out, ref, atol=1e-5), (out - ref).abs().max()
    assert counts.sum().item() == 20 * k
    assert l_aux.item() > 0


def test_capacity_drops_tokens():
    from shuffle_exchange_amd.moe.sharded_moe import top2gating
    logits = torch.zeros(16, 4)
    logits[:, 0] = 5.0  # every token prefers expert 0
    logits[:, 1] = 4.0
    r = top2gating(logits, capacity_factor=0.5, min_capacity=1, top2_2nd_expert_sampling=False)
    # capacity = ceil(16/4 * 0.5 * 2) = 4 -> only 4 tokens fit in expert 0 and 4 in expert 1
    assert r.capacity == 4
    assert int(r.keep[:, 0].sum()) == 4 and int(r.keep[:, 1].sum()) == 4
    assert bool(r.keep[:4, 0].all())  # first tokens keep their slot (positional priority)


def test_expert_parallel_matches_single_process():
    res = run_dist(C.case_moe_ep, 2)
    single = C.moe_single_reference()
    for r in res:
        assert torch.allclose(r["out"], single["out"], atol=1e-5)
    # each rank holds half of the experts: its grads equal the single-process grads of those experts
    for rank, r in enumerate(res):
        sl = slice(rank * 2, rank * 2 + 2)
        assert torch.allclose(r["g_up"], single["g_up"][sl], atol=1e-5)
        assert torch.allclose(r["g_down"], single["g_down"][sl], atol=1e-5)


@pytest.mark.parametrize("stage", [0, 2])
def test_mixtral_trains_with_expert_parallelism(stage):
    res = run_dist(C.case_mixtral_train, 2, stage)
    for r in res:
        assert r["losses"][-1] < r["losses"][0]
