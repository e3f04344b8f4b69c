"""Mixture-of-Experts routing, dispatch and expert-parallel all-to-all.

Parity: reference deepspeed/moe/sharded_moe.py -- ``top1gating`` :183, ``top2gating`` :290,
``topkgating`` :374 (capacity, random token selection, noisy gating, drop-tokens, aux loss),
``TopKGate`` :450, ``MOELayer.forward`` :587-678 and ``_AllToAll`` :96-108.

MI355X-first data path (instead of the reference's dense [tokens, experts, capacity] one-hot
einsums, which cost O(S*E*C) memory and FLOPs):
  * gating yields a *sparse* assignment list -- (token, expert, slot, weight) for each of the k
    choices -- with slot = expert * capacity + position-in-expert (positions by a cumulative count,
    identical to the reference's cumsum locations, so the same tokens are dropped);
  * dispatch = one row gather into a contiguous [E, C, H] buffer; the EP all-to-all moves
    whole [E_local, C, H] blocks (one RCCL all_to_all_single over xGMI, full-mesh on one node);
  * local experts run as ONE batched GEMM over [E_local, ep*C, H] (equal capacity per expert);
  * combine = one weighted row gather + index_add back to token order.
"""
import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import comm as dist

exp_selection_uniform_map = {}
gumbel_map = {}


def gumbel_rsample(shape, device):
    g = gumbel_map.get(device)
    if g is None:
        one = torch.tensor(1.0, device=device)
        zero = torch.tensor(0.0, device=device)
        g = torch.distributions.gumbel.Gumbel(zero, one).rsample
        gumbel_map[device] = g
    return g(shape)


def multiplicative_jitter(x, device, epsilon=1e-2):
    if epsilon == 0:
        return x
    u = torch.empty_like(x).uniform_(1.0 - epsilon, 1.0 + epsilon)
    return x * u


def _capacity(num_tokens, num_experts, capacity_factor, min_capacity, tp=1):
    c = max(int(math.ceil(num_tokens / num_experts * capacity_factor)), int(min_capacity))
    # tensor-parallel non-expert layers: the capacity is split over the TP ranks before the a2a
    # (mappings.drop_tokens), so it is padded to a multiple of tp (reference sharded_moe.py:220)
    return -(-c // tp) * tp


class Routing:
    """Sparse routing decision: for each of the S*k assignments (token-major):
    ``expert`` [S,k] int64, ``location`` [S,k] int64 (position inside the expert's capacity),
    ``keep`` [S,k] bool (False = dropped by capacity), ``weight`` [S,k] float (combine weight),
    plus ``capacity``, ``l_aux`` and ``exp_counts`` (pre-drop tokens per expert)."""

    def __init__(self, expert, location, keep, weight, capacity, l_aux, exp_counts):
        self.expert, self.location, self.keep, self.weight = expert, location, keep, weight
        self.capacity, self.l_aux, self.exp_counts = capacity, l_aux, exp_counts

    def slots(self):
        return self.expert * self.capacity + self.location


def _positions(expert_idx, E, mask=None):
    """Cumulative position of each (token, choice) inside its expert, choice-major like the
    reference (all first choices are placed before all second choices)."""
    S, k = expert_idx.shape
    oh = F.one_hot(expert_idx.t().reshape(-1), E).to(torch.int32)  # [k*S, E], choice-major
    if mask is not None:
        oh = oh * mask.t().reshape(-1, 1).to(oh.dtype)
    # scan along the contiguous dimension ([E, k*S]): the outer-dim int64 scan of [k*S, E] was
    # 1.5 ms per MoE layer on MI355X at 8K tokens
    loc = torch.cumsum(oh.t().contiguous(), dim=1).t() - 1
    loc = (loc * oh).sum(1).view(k, S).t()
    return loc.to(torch.int64)


def _max_capacity(exp_counts, ep_group, num_tokens, tp=1):
    new_cap = exp_counts.max().to(torch.int64).reshape(1)
    if ep_group is not None and dist.get_world_size(ep_group) > 1:
        dist.all_reduce(new_cap, op=dist.ReduceOp.MAX, group=ep_group)
    c = max(1, int(min(int(new_cap.item()), num_tokens)))
    return -(-c // tp) * tp


def top1gating(logits, capacity_factor, min_capacity, used_token=None, noisy_gate_policy=None, drop_tokens=True,
               use_rts=True, ep_group=None, tp=1):
    from ..ops.moe import topk_softmax
    logits_w_noise = logits + gumbel_rsample(logits.shape, logits.device) if noisy_gate_policy == "RSample" else None
    gates, top = topk_softmax(logits, 1)
    S, E = gates.shape
    capacity = _capacity(S, E, capacity_factor, min_capacity, tp)
    idx1 = torch.argmax(logits_w_noise, dim=1) if logits_w_noise is not None else top[:, 0]
    mask1 = F.one_hot(idx1, E)
    if used_token is not None:
        mask1 = mask1 * used_token.unsqueeze(1).to(mask1.dtype)
    exp_counts = mask1.sum(0).detach()
    if not drop_tokens:
        capacity = _max_capacity(exp_counts, ep_group, S, tp)
    me = gates.mean(0)
    ce = mask1.float().mean(0)
    l_aux = (me * ce).sum() * E
    if use_rts:
        # random token selection: priority among a expert's tokens is random, not positional
        uniform = torch.rand(mask1.shape, device=logits.device)
        scores = (mask1 * uniform).masked_fill(mask1 == 0, -1.0)
        # keep the top-`capacity` random scores per expert
        kth = torch.topk(scores, k=min(capacity, S), dim=0).values[-1:]
        keep1 = (scores >= kth) & (mask1 > 0)
        mask1 = mask1 * keep1.to(mask1.dtype)
    loc = _positions(idx1.unsqueeze(1), E, (mask1.sum(1) > 0).unsqueeze(1))
    keep = (mask1.sum(1) > 0).unsqueeze(1) & (loc < capacity)
    gate1 = (gates * F.one_hot(idx1, E)).sum(1, keepdim=True)
    return Routing(idx1.unsqueeze(1), loc.clamp(max=capacity - 1), keep, gate1, capacity, l_aux, exp_counts)


def top2gating(logits, capacity_factor, min_capacity, drop_tokens=True, ep_group=None, top2_2nd_expert_sampling=True,
               tp=1):
    gates = F.softmax(logits, dim=1)
    S, E = gates.shape
    idx1 = torch.argmax(gates, dim=1)
    mask1 = F.one_hot(idx1, E)
    lg = logits + gumbel_rsample(logits.shape, logits.device) if top2_2nd_expert_sampling else logits
    idx2 = torch.argmax(lg.masked_fill(mask1.bool(), float("-inf")), dim=1)
    mask2 = F.one_hot(idx2, E)
    me = gates.mean(0)
    ce = mask1.float().mean(0)
    l_aux = (me * ce).mean() * E * E
    exp_counts = (mask1 + mask2).sum(0).detach()
    idx = torch.stack([idx1, idx2], dim=1)
    loc = _positions(idx, E)
    if drop_tokens:
        capacity = _capacity(S, E, capacity_factor * 2, min_capacity, tp)
    else:
        capacity = _max_capacity(exp_counts, ep_group, S, tp)
    keep = loc < capacity
    g = torch.stack([(gates * mask1).sum(1), (gates * mask2).sum(1)], dim=1) * keep
    denom = g.sum(1, keepdim=True).clamp(min=torch.finfo(g.dtype).eps)
    g = g / denom
    return Routing(idx, loc.clamp(max=capacity - 1), keep, g, capacity, l_aux, exp_counts)


def topkgating(logits, k, capacity_factor, min_capacity, drop_tokens=True, ep_group=None, drop_policy="probs", tp=1):
    from ..ops.moe import topk_softmax
    gates, top_idx = topk_softmax(logits, k)  # one HIP launch on GPU (softmax + top-k per token)
    top_gate = torch.gather(logits, 1, top_idx)
    S, E = gates.shape
    mask = torch.zeros_like(gates, dtype=torch.bool).scatter_(1, top_idx, True)
    exp_counts = mask.sum(0).detach()
    me = gates.mean(0)
    ce = mask.float().mean(0)
    l_aux = (me * ce).mean() * E * E / k
    if drop_tokens:
        capacity = _capacity(S, E, capacity_factor * k, min_capacity, tp)
        if drop_policy == "probs":
            topk_masked = torch.zeros_like(logits).scatter(1, top_idx, top_gate)
            cidx = torch.topk(topk_masked, k=min(capacity, S), dim=0, sorted=False)[1]
            cmask = torch.zeros_like(mask).scatter_(0, cidx, True)
            mask = mask & cmask
        elif drop_policy != "position":
            raise ValueError(f"Invalid drop_policy: {drop_policy}")
    else:
        capacity = _max_capacity(exp_counts, ep_group, S, tp)
    # positions along the token axis per expert (the reference's cumsum over tokens)
    locs = (torch.cumsum(mask.to(torch.int32).t().contiguous(), dim=1).t() - 1).to(torch.int64)
    loc_k = torch.gather(locs, 1, top_idx)
    keep_k = torch.gather(mask, 1, top_idx) & (loc_k < capacity)
    gates_k = torch.gather(gates, 1, top_idx) * keep_k
    gates_k = gates_k / gates_k.sum(1, keepdim=True).clamp(min=torch.finfo(gates_k.dtype).eps)
    return Routing(top_idx, loc_k.clamp(min=0, max=capacity - 1), keep_k, gates_k, capacity, l_aux, exp_counts)


class TopKGate(nn.Module):
    def __init__(self, model_dim, num_experts, k=1, capacity_factor=1.0, eval_capacity_factor=1.0, min_capacity=8,
                 noisy_gate_policy=None, drop_tokens=True, use_rts=True, ep_group=None, top2_2nd_expert_sampling=True,
                 drop_policy="probs"):
        super().__init__()
        self.wg = nn.Linear(model_dim, num_experts, bias=False).float()
        self.k = k
        self.capacity_factor = capacity_factor
        self.eval_capacity_factor = eval_capacity_factor
        self.min_capacity = min_capacity
        self.noisy_gate_policy = noisy_gate_policy
        self.drop_tokens = drop_tokens
        self.use_rts = use_rts
        self.ep_group = ep_group
        self.top2_2nd_expert_sampling = top2_2nd_expert_sampling
        self.drop_policy = drop_policy
        self.tp = 1

    def _set_ep_group(self, g, tp=1):
        self.ep_group = g
        self.tp = tp

    def forward(self, x, used_token=None):
        # gating in fp32 (reference sharded_moe.py:500-524)
        xf = x.float()
        if self.noisy_gate_policy == "Jitter" and self.training:
            xf = multiplicative_jitter(xf, device=x.device)
        logits = F.linear(xf, self.wg.weight.float())
        cf = self.capacity_factor if self.training else self.eval_capacity_factor
        if self.k == 1:
            return top1gating(logits, cf, self.min_capacity, used_token,
                              self.noisy_gate_policy if self.training else None, self.drop_tokens, self.use_rts,
                              self.ep_group, self.tp)
        if self.k == 2:
            return top2gating(logits, cf, self.min_capacity, self.drop_tokens, self.ep_group,
                              self.top2_2nd_expert_sampling and self.training, self.tp)
        return topkgating(logits, self.k, cf, self.min_capacity, self.drop_tokens, self.ep_group, self.drop_policy,
                          self.tp)


class _AllToAll(torch.autograd.Function):
    """Equal-split all_to_all_single over the expert-parallel group; backward is the inverse."""

    @staticmethod
    def forward(ctx, group, x):
        ctx.group = group
        x = x.contiguous()
        out = torch.empty_like(x)
        dist.all_to_all_single(out, x, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        out = torch.empty_like(g)
        dist.all_to_all_single(out, g, group=ctx.group)
        return None, out


def all_to_all(group, x):
    if group is None or dist.get_world_size(group) == 1:
        return x
    return _AllToAll.apply(group, x)


class MOELayer(nn.Module):
    """gate -> dispatch -> a2a -> experts -> a2a -> combine (reference sharded_moe.py:587-678).

    Tensor-parallel non-expert layers (``tp_group``): every TP rank routes the same tokens, keeps
    its 1/tp share of each expert's capacity for the a2a (``drop_tokens``) and all-gathers the
    shares after the return a2a. With expert TP (``expert_tp``) the EP group lives inside one TP
    slice and the TP peers of a rank hold the other column/row shards of the SAME experts: the
    shares are all-gathered before the experts (which run copy_to_tp / reduce_from_tp inside)
    and dropped again after them. Without it, the EP group spans the TP ranks (different experts
    per TP rank) and each expert sees only its share."""

    def __init__(self, gate: TopKGate, experts, ep_group_name, ep_size, num_local_experts):
        super().__init__()
        self.gate = gate
        self.experts = experts
        self.ep_group = None
        self.ep_group_name = ep_group_name
        self.ep_size = ep_size
        self.num_local_experts = num_local_experts
        self.l_aux = None
        self.exp_counts = None
        self.wall_clock_breakdown = False
        self.tp_group = None
        self.tp = 1
        self.expert_tp = False

    def _set_ep_group(self, ep_group, tp_group=None, expert_tp=False):
        self.ep_group = ep_group
        self.tp_group = tp_group
        self.tp = dist.get_world_size(tp_group) if tp_group is not None else 1
        self.expert_tp = bool(expert_tp) and self.tp > 1
        self.gate._set_ep_group(ep_group, self.tp)

    def forward(self, x, used_token=None):
        shape = x.shape
        H = shape[-1]
        xt = x.reshape(-1, H)
        S = xt.shape[0]
        r = self.gate(xt, used_token)
        E = self.ep_size * self.num_local_experts
        C = r.capacity
        k = r.expert.shape[1]
        from ..ops.moe import combine, dispatch, routing_tables
        # slots[t, c] = expert * C + position (-1 dropped) and its inverse slot_src[E * C]: dispatch
        # and combine are then atomic-free row gathers (csrc/kernels/moe.hip on the GPU)
        slots, slot_src = routing_tables(r.expert, r.location, r.keep, C, E)
        disp = dispatch(xt, slots, slot_src)
        ep, nle, tp = self.ep_size, self.num_local_experts, self.tp
        from .mappings import drop_tokens, gather_tokens
        Cl = C // tp  # capacity share of this TP rank
        if tp > 1:
            disp = drop_tokens(disp.view(E, C, H), 1, self.tp_group)
        # [E, Cl, H] -> a2a over EP: rank j receives, from every rank, the rows for its local experts
        disp = all_to_all(self.ep_group, disp.reshape(ep, nle * Cl, H))
        Ce = Cl
        if self.expert_tp:  # the TP peers hold the other shards of these experts: all see every token
            disp = gather_tokens(disp.view(ep * nle, Cl, H), 1, self.tp_group)
            Ce = C
        # local experts see [E_local, ep*Ce, H]
        disp = disp.reshape(ep, nle, Ce, H).transpose(0, 1).reshape(nle, ep * Ce, H)
        out = self.experts(disp)
        out = out.view(nle, ep, Ce, H).transpose(0, 1).reshape(ep * nle, Ce, H)
        if self.expert_tp:
            out = drop_tokens(out, 1, self.tp_group)
        out = all_to_all(self.ep_group, out.reshape(ep, nle * Cl, H))
        if tp > 1:
            out = gather_tokens(out.view(E, Cl, H), 1, self.tp_group)
        out = out.reshape(E * C, H)
        comb = combine(out, slots, slot_src, r.weight)
        self.l_aux = r.l_aux
        self.exp_counts = r.exp_counts
        return comb.view(shape)
