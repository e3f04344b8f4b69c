"""Automatic tensor parallelism: find the Linear layers of a model and swap them for column / row
parallel shards.

Parity: reference module_inject/auto_tp.py -- ``AutoTP`` :193, ``tp_parser`` :285 (row-parallel
= layers whose output is added back into the residual stream: o_proj / down_proj / out_proj /
dense_4h_to_h / fc2 / c_proj ...), ``_replace`` :348, ``_replace_module``; training entry
``runtime/tensor_parallel/tp_manager.py:12`` and ``deepspeed.tp_model_init``.

Layout hints (new): a Linear may carry ``_tp_layout`` (``("chunks", n)`` for packed [gate|up] or
[q|k|v] of equal blocks, ``("heads", [nq, nkv, nkv], head_dim)`` for GQA-packed qkv) and
``_tp_row_parallel``; modules that track head counts expose ``tp_shard_(tp)``. Without hints the
reference's name heuristics decide. Embeddings, LM heads, MoE routers and expert weights stay
replicated (experts are expert-parallel instead).
"""
import torch
import torch.nn as nn

from .. import comm as dist
from ..utils.logging import log_dist
from .layers import LinearAllreduce, LinearLayer, TensorParallelLinearBase, shard_rows

ROW_PARALLEL_NAMES = {"o_proj", "down_proj", "out_proj", "c_proj", "mlp_proj", "dense_4h_to_h", "fc2", "wo", "w2",
                      "dense", "proj_out", "self_attn.dense", "attention.dense"}
KEEP_REPLICATED = {"lm_head", "embed_out", "wg", "gate", "router", "score", "classifier", "coefficient"}


class AutoTP:
    def __init__(self, module, tp_group, tp_size=None, linear_names=None, keep_replicated=None):
        self.module = module
        self.tp_group = tp_group
        self.tp_size = tp_size or (dist.get_world_size(tp_group) if tp_group is not None else 1)
        self.tp_rank = dist.get_rank(tp_group) if tp_group is not None else 0
        self.row_names = set(linear_names or ROW_PARALLEL_NAMES)
        self.keep = set(keep_replicated or KEEP_REPLICATED)

    @staticmethod
    def _leaf(name):
        return name.rsplit(".", 1)[-1]

    def _skip(self, name):
        parts = name.split(".")
        return self._leaf(name) in self.keep or "experts" in parts or "deepspeed_experts" in parts

    def tp_parser(self, model=None):
        """[(qualified name, "row" | "col")] for every Linear that will be sharded."""
        model = model or self.module
        out = []
        for name, m in model.named_modules():
            if not isinstance(m, nn.Linear) or isinstance(m, TensorParallelLinearBase) or self._skip(name):
                continue
            two = ".".join(name.split(".")[-2:])
            row = getattr(m, "_tp_row_parallel", False) or self._leaf(name) in self.row_names or two in self.row_names
            out.append((name, "row" if row else "col"))
        return out

    def _replace(self, m, kind):
        w = m.weight.data
        b = m.bias.data if m.bias is not None else None
        layout = getattr(m, "_tp_layout", None)
        if kind == "col":
            ws = shard_rows(w, layout, self.tp_size, self.tp_rank).contiguous()
            bs = shard_rows(b, layout, self.tp_size, self.tp_rank).contiguous() if b is not None else None
            new = LinearLayer(ws, bs, self.tp_group, tuple(w.shape), layout=layout)
        else:
            assert w.shape[1] % self.tp_size == 0, f"in_features {w.shape[1]} not divisible by tp {self.tp_size}"
            ws = w.chunk(self.tp_size, dim=1)[self.tp_rank].contiguous()
            new = LinearAllreduce(ws, b.clone() if b is not None else None, self.tp_group, tuple(w.shape))
        new.weight.requires_grad_(m.weight.requires_grad)
        return new

    def replace_module(self):
        if self.tp_size == 1:
            return self.module
        plan = self.tp_parser()
        for name, kind in plan:
            parent_name, _, leaf = name.rpartition(".")
            parent = self.module.get_submodule(parent_name) if parent_name else self.module
            setattr(parent, leaf, self._replace(getattr(parent, leaf), kind))
        for m in self.module.modules():
            if hasattr(m, "tp_shard_") and not getattr(m, "_tp_sharded", False):
                m.tp_shard_(self.tp_size)
                m._tp_sharded = True
        log_dist(f"AutoTP: tp={self.tp_size}, {sum(k == 'col' for _, k in plan)} column-parallel and "
                 f"{sum(k == 'row' for _, k in plan)} row-parallel linears", ranks=[0])
        return self.module


def broadcast_within_tp(model, tp_group, src_global_rank):
    """Identical starting weights on every TP rank before sharding. Expert weights are left alone:
    without expert TP the TP ranks hold different experts (and expert-TP shards are cut from
    each rank's own full init)."""
    from ..moe.utils import is_moe_param
    with torch.no_grad():
        for p in list(model.parameters()) + list(model.buffers()):
            if isinstance(p, nn.Parameter) and is_moe_param(p):
                continue
            dist.broadcast(p.data, src=src_global_rank, group=tp_group)


def tp_model_init(model, tp_size, dtype=None, tp_group=None):
    """Shard ``model`` for tensor-parallel training (reference ``deepspeed.tp_model_init``)."""
    from ..parallel import groups
    if tp_group is None:
        if groups.get_tensor_model_parallel_world_size() != tp_size:
            groups.initialize(tensor_parallel_size=tp_size)
        tp_group = groups.get_tensor_model_parallel_group()
    ranks = groups.group_ranks("model") if tp_group is groups.get_tensor_model_parallel_group() else \
        dist.group_ranks(tp_group)
    if tp_size > 1:
        broadcast_within_tp(model, tp_group, min(ranks))
    AutoTP(model, tp_group, tp_size).replace_module()
    if dtype is not None:
        model.to(dtype)
    model._sxe_tp_size = tp_size
    return model


def gather_tp_state_dict(model):
    """Full (unsharded) state dict of an AutoTP model, identical on every TP rank."""
    from .layers import gather_full_weight
    sd = {}
    for name, m in model.named_modules():
        if isinstance(m, TensorParallelLinearBase):
            sd[name + ".weight"] = gather_full_weight(m)
            if m.bias is not None:
                if m.split_dim == 0 and m.tp_world_size > 1:
                    parts = [torch.empty_like(m.bias) for _ in range(m.tp_world_size)]
                    dist.all_gather(parts, m.bias.detach().contiguous(), group=m.tp_group)
                    from .layers import unshard_rows
                    sd[name + ".bias"] = unshard_rows(parts, m.layout)
                else:
                    sd[name + ".bias"] = m.bias.detach()
    for k, v in model.state_dict().items():
        sd.setdefault(k, v.detach())
    return sd
