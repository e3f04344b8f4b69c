"""Token drop / gather across the tensor-parallel group for MoE layers.

Parity: reference deepspeed/moe/mappings.py -- ``_DropTokens`` :88 / ``_GatherTokens`` :71 (and
their use in sharded_moe.py:615-665). When the non-expert part of the model is tensor-parallel,
every TP rank holds the same tokens; each rank keeps only its 1/tp share of the dispatched
capacity before the expert all-to-all (correctness for replicated experts, and 1/tp of the a2a
bytes over xGMI), and the shares are all-gathered again afterwards.

Drop's backward is a gather and gather's backward is a drop (no reduction): the incoming
gradient is identical on all TP ranks, so each rank's slice of it is exact.
"""
import torch

from .. import comm as dist


def _drop(x, dim, group):
    n = dist.get_world_size(group)
    if n == 1:
        return x
    assert x.shape[dim] % n == 0, f"dimension {dim} ({x.shape[dim]}) not divisible by tp {n}"
    c = x.shape[dim] // n
    return x.narrow(dim, dist.get_rank(group) * c, c).contiguous()


def _gather(x, dim, group):
    n = dist.get_world_size(group)
    if n == 1:
        return x
    x = x.movedim(dim, 0).contiguous()
    out = x.new_empty((n * x.shape[0],) + tuple(x.shape[1:]))
    dist.all_gather_into_tensor(out, x, group=group)
    return out.movedim(0, dim).contiguous()


class _DropTokens(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dim, group):
        ctx.dim, ctx.group = dim, group
        return _drop(x, dim, group)

    @staticmethod
    def backward(ctx, g):
        return _gather(g, ctx.dim, ctx.group), None, None


class _GatherTokens(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dim, group):
        ctx.dim, ctx.group = dim, group
        return _gather(x, dim, group)

    @staticmethod
    def backward(ctx, g):
        return _drop(g, ctx.dim, ctx.group), None, None


def drop_tokens(x, dim, group):
    if group is None or dist.get_world_size(group) == 1:
        return x
    return _DropTokens.apply(x, dim, group)


def gather_tokens(x, dim, group):
    if group is None or dist.get_world_size(group) == 1:
        return x
    return _GatherTokens.apply(x, dim, group)
