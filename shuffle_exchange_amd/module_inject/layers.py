"""Tensor-parallel linear layers (Megatron column / row split) for training and inference.

Parity: reference module_inject/layers.py -- ``RowParallel`` / ``ColumnParallel`` autograd
functions :64-153, ``LinearAllreduce`` :388, ``LinearLayer`` :465, ``LmHeadLinearAllreduce``,
``GatherReplacedLayerParams`` :655 (gather shards for checkpointing).

Column-parallel (``LinearLayer``): weight rows split over TP ranks, identity forward on the input
and an all-reduce of the input gradient in backward. Row-parallel (``LinearAllreduce``): weight
columns split, partial products all-reduced in forward, identity backward. Both run their GEMM
through ``ops.linear`` so the weight-grad GEMM still lands in the ZeRO buffers.
On one MI355X node TP all-reduces ride RCCL over xGMI; the reduction stream is the compute
stream (the result is needed immediately), so TP degree should stay within a node.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import comm as dist
from ..ops.linear import linear


class _CopyToTP(torch.autograd.Function):
    """Identity forward, all-reduce of the gradient (input of a column-parallel layer)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromTP(torch.autograd.Function):
    """All-reduce forward, identity backward (output of a row-parallel layer)."""

    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous()
        dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherFromTP(torch.autograd.Function):
    """All-gather along the last dim forward, split backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        ws = dist.get_world_size(group)
        ctx.rank = dist.get_rank(group)
        parts = [torch.empty_like(x) for _ in range(ws)]
        dist.all_gather(parts, x.contiguous(), group=group)
        return torch.cat(parts, dim=-1)

    @staticmethod
    def backward(ctx, g):
        ws = dist.get_world_size(ctx.group)
        return g.chunk(ws, dim=-1)[ctx.rank].contiguous(), None


class _ColumnParallelLinear(torch.autograd.Function):
    """Column-parallel GEMM whose backward overlaps the input-gradient all-reduce with the
    weight-gradient GEMM: dX = dY W is computed first and its all-reduce is launched
    asynchronously (RCCL runs on its own stream over xGMI) before dW = dY^T X is issued on the
    compute stream. Without ``handles`` the wait is at the end of this backward; with a
    ``handles`` list (Domino) the Work is parked there and waited by ``wait_grad_handles``
    further down the graph, so it also overlaps the other micro-batch's backward.
    (Reference: runtime/domino/async_linear.py:14-36 ``DominoAsyncColumnParallelLinearImpl``.)"""

    @staticmethod
    def forward(ctx, x, weight, bias, group, handles):
        ctx.save_for_backward(x, weight)
        ctx.group, ctx.handles, ctx.has_bias = group, handles, bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, gy):
        from ..ops.linear import write_weight_grad
        x, w = ctx.saved_tensors
        dx = dw = db = None
        work = None
        if ctx.needs_input_grad[0]:
            dx = torch.matmul(gy, w).contiguous()
            work = dist.all_reduce(dx, group=ctx.group, async_op=True)
        gy2 = gy.reshape(-1, gy.shape[-1])
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, x.shape[-1])
            if not write_weight_grad(w, gy2, x2):
                dw = gy2.t() @ x2
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = gy2.sum(0)
        if work is not None:
            if ctx.handles is not None:
                ctx.handles.append(work)
            else:
                work.wait()
        return dx, dw, db, None, None


class _WaitGradHandles(torch.autograd.Function):
    """Identity; its backward waits for the input-grad all-reduces parked by the column-parallel
    layers that consume this tensor (reference runtime/domino/transformer.py:50-70 ``NoOper``)."""

    @staticmethod
    def forward(ctx, x, handles):
        ctx.handles = handles
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        while ctx.handles:
            ctx.handles.pop().wait()
        return g, None


def wait_grad_handles(x, handles):
    return _WaitGradHandles.apply(x, handles)


def copy_to_tp(x, group):
    return _CopyToTP.apply(x, group)


def reduce_from_tp(x, group):
    return _ReduceFromTP.apply(x, group)


def gather_from_tp(x, group):
    return _GatherFromTP.apply(x, group)


class TensorParallelLinearBase(nn.Module):
    _sxe_lower_precision_safe = True  # torch_autocast: GEMM weights may communicate in bf16 / fp16
    is_tensor_parallel = True

    def __init__(self, weight, bias, group, full_shape, split_dim, layout=None):
        super().__init__()
        self.weight = nn.Parameter(weight)
        self.bias = nn.Parameter(bias) if bias is not None else None
        self.tp_group = group
        self.tp_world_size = dist.get_world_size(group) if group is not None else 1
        self.tp_rank = dist.get_rank(group) if group is not None else 0
        self.full_shape = tuple(full_shape)
        self.split_dim = split_dim
        self.layout = layout
        self.weight.tensor_model_parallel = True
        self.weight.partition_dim = split_dim

    @property
    def in_features(self):
        return self.weight.shape[1]

    @property
    def out_features(self):
        return self.weight.shape[0]


class LinearLayer(TensorParallelLinearBase):
    """Column parallel: y_local = x W_local^T (+ b_local); optional all-gather of the output."""

    def __init__(self, weight, bias, group, full_shape, layout=None, gather_output=False):
        super().__init__(weight, bias, group, full_shape, 0, layout)
        if self.bias is not None:
            self.bias.tensor_model_parallel = True
        self.gather_output = gather_output

    def forward(self, x, skip_bias=False, grad_handles=None):
        b = None if skip_bias else self.bias
        if self.tp_group is not None and self.tp_world_size > 1 and torch.is_grad_enabled() and (
                x.requires_grad or self.weight.requires_grad):
            y = _ColumnParallelLinear.apply(x, self.weight, b, self.tp_group, grad_handles)
        else:
            y = linear(x, self.weight, b)
        if self.gather_output and self.tp_world_size > 1:
            y = gather_from_tp(y, self.tp_group)
        return y


class LinearAllreduce(TensorParallelLinearBase):
    """Row parallel: y = all_reduce(x_local W_local^T) + b (bias added once, after the reduce)."""

    def __init__(self, weight, bias, group, full_shape, layout=None):
        super().__init__(weight, bias, group, full_shape, 1, layout)

    def forward(self, x, skip_bias=False):
        y = linear(x, self.weight)
        if self.tp_group is not None and self.tp_world_size > 1:
            y = reduce_from_tp(y, self.tp_group)
        if self.bias is not None and not skip_bias:
            y = y + self.bias
        return y

    def forward_partial(self, x):
        """x_local W_local^T without the reduction (Domino launches it asynchronously)."""
        return linear(x, self.weight)


class LmHeadLinearAllreduce(LinearAllreduce):
    """Row-parallel LM head used by inference AutoTP (hidden split, logits all-reduced)."""

    def forward(self, x):
        k = self.weight.shape[1]
        x_local = x[..., self.tp_rank * k:(self.tp_rank + 1) * k]
        return super().forward(x_local)


# ------------------------------------------------------------------------------------ sharding
def shard_rows(w, layout, tp, rank):
    """Slice the output rows of W for column parallelism. ``layout``:
    None -> contiguous split; ("chunks", n) -> split each of n equal row blocks (e.g. [gate|up]);
    ("heads", [n0, n1, ...], head_dim) -> split each section of heads (e.g. packed q|k|v with GQA)."""
    if layout is None:
        assert w.shape[0] % tp == 0, f"rows {w.shape[0]} not divisible by tp {tp}"
        return w.chunk(tp, dim=0)[rank]
    kind = layout[0]
    if kind == "chunks":
        blocks = w.chunk(layout[1], dim=0)
        return torch.cat([b.chunk(tp, dim=0)[rank] for b in blocks], dim=0)
    if kind == "heads":
        counts, d = layout[1], layout[2]
        out, o = [], 0
        for n in counts:
            sec = w[o * d:(o + n) * d]
            assert n % tp == 0, f"{n} heads not divisible by tp {tp}"
            out.append(sec.view(n, d, *w.shape[1:]).chunk(tp, dim=0)[rank].reshape(-1, *w.shape[1:]))
            o += n
        return torch.cat(out, dim=0)
    raise ValueError(f"unknown layout {layout}")


def unshard_rows(parts, layout):
    """Inverse of shard_rows: list of per-rank shards -> full weight."""
    tp = len(parts)
    if layout is None:
        return torch.cat(parts, dim=0)
    kind = layout[0]
    if kind == "chunks":
        n = layout[1]
        blocks = [p.chunk(n, dim=0) for p in parts]
        return torch.cat([torch.cat([blocks[r][i] for r in range(tp)], dim=0) for i in range(n)], dim=0)
    if kind == "heads":
        counts, d = layout[1], layout[2]
        secs = []
        offs = [0]
        for n in counts:
            offs.append(offs[-1] + (n // tp) * d)
        for i in range(len(counts)):
            secs.append(torch.cat([p[offs[i]:offs[i + 1]] for p in parts], dim=0))
        return torch.cat(secs, dim=0)
    raise ValueError(f"unknown layout {layout}")


def gather_full_weight(layer):
    """Full (unsharded) weight of a TP layer, on every rank of its group (for checkpoints)."""
    w = layer.weight.detach().contiguous()
    if layer.tp_world_size == 1:
        return w
    parts = [torch.empty_like(w) for _ in range(layer.tp_world_size)]
    dist.all_gather(parts, w, group=layer.tp_group)
    if layer.split_dim == 0:
        return unshard_rows(parts, layer.layout)
    return torch.cat(parts, dim=1)


class GatherReplacedLayerParams:
    """Context manager: temporarily materialise full weights of TP layers (reference :655)."""

    def __init__(self, params_or_modules, module=None, enabled=True):
        self.mods = [m for m in (params_or_modules if isinstance(params_or_modules, (list, tuple)) else
                                 [params_or_modules]) if isinstance(m, TensorParallelLinearBase)]
        self.enabled = enabled
        self.saved = []

    def __enter__(self):
        if not self.enabled:
            return self
        for m in self.mods:
            self.saved.append(m.weight.data)
            m.weight.data = gather_full_weight(m)
        return self

    def __exit__(self, *exc):
        for m, d in zip(self.mods, self.saved):
            m.weight.data = d
        self.saved = []
