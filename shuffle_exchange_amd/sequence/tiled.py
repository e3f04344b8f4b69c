"""Arctic Long Sequence Training (ALST) helpers: tiled compute along the sequence, sequence-parallel
loss, and the HF-transformers Ulysses attention adapter.

Parity: reference runtime/sequence_parallel/ulysses_sp.py -- ``UlyssesSPAttentionHF`` :47 /
``register_with_transformers`` :337, ``SequenceTiledCompute`` :608, ``TiledMLP`` :757,
``TiledFusedLogitsLoss`` :915; sequence/cross_entropy.py ``vocab_sequence_parallel_cross_entropy``
:11-60.

``TiledMLP`` / ``SequenceTiledCompute`` keep only one tile of the intermediate activations alive:
forward runs tiles under no_grad, backward recomputes each tile with grad and back-propagates it
immediately (parameter grads accumulate across tiles). For Llama-3-8B at 32k tokens the
[T, 2*14336] gate/up activation shrinks from 1.8 GB to 1.8 GB / n_tiles.
"""
import math

import torch

from .. import comm as dist


class _TiledCompute(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fn, n_tiles, x, *params):
        ctx.fn, ctx.n_tiles, ctx.n_params = fn, n_tiles, len(params)
        # parameters whose gradients the tiles accumulate: explicit, else the module's own
        ctx.grad_params = [p for p in (params or (fn.parameters() if isinstance(fn, torch.nn.Module) else ()))
                           if p.requires_grad]
        ctx.save_for_backward(x)
        with torch.no_grad():
            outs = [fn(t) for t in x.chunk(n_tiles, dim=-2)]
        return torch.cat(outs, dim=-2)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        dx = torch.empty_like(x)
        xs, gs, dxs = x.chunk(ctx.n_tiles, dim=-2), g.chunk(ctx.n_tiles, dim=-2), dx.chunk(ctx.n_tiles, dim=-2)
        params = ctx.grad_params
        last = len(xs) - 1
        try:
            for t, (xt, gt, dxt) in enumerate(zip(xs, gs, dxs)):
                # every tile but the last delivers a PARTIAL parameter gradient: the ZeRO hooks and the
                # direct weight-grad writers leave it summing in .grad (reference ds_grad_is_ready,
                # runtime/sequence_parallel/ulysses_sp.py:720-724,846-850; honoured at
                # stage_1_and_2.py:1146 / stage3.py:1280), so a unit is reduced once, with the total
                for p in params:
                    p._sxe_grad_partial = t < last
                xt = xt.detach().requires_grad_(True)
                with torch.enable_grad():
                    y = ctx.fn(xt)
                torch.autograd.backward(y, gt)
                dxt.copy_(xt.grad)
        finally:
            for p in params:
                p._sxe_grad_partial = False
        return (None, None, dx) + (None,) * ctx.n_params


def sequence_tiled_compute(fn, x, n_tiles=None, tile_tokens=None, params=()):
    """fn over ``x`` [..., S, H] in sequence tiles; parameters of ``fn`` get their grads through the
    per-tile recompute in backward."""
    S = x.shape[-2]
    if n_tiles is None:
        n_tiles = max(1, math.ceil(S / tile_tokens)) if tile_tokens else 1
    n_tiles = max(1, min(n_tiles, S))
    if n_tiles == 1 or not torch.is_grad_enabled():
        return fn(x)
    return _TiledCompute.apply(fn, n_tiles, x, *params)


SequenceTiledCompute = sequence_tiled_compute


class TiledMLP(torch.nn.Module):
    """Wrap an MLP module: ``TiledMLP(mlp, num_shards)`` (reference signature ``TiledMLP.apply``)."""

    def __init__(self, mlp, num_shards=None, tile_tokens=8192):
        super().__init__()
        self.mlp = mlp
        self.num_shards = num_shards
        self.tile_tokens = tile_tokens

    def forward(self, x):
        return sequence_tiled_compute(self.mlp, x, self.num_shards, self.tile_tokens)


def tiled_fused_logits_loss(h, weight, labels, ignore_index=-100, tile_tokens=8192, reduction="mean"):
    """LM head + CE without materialising [T, V] logits (TiledFusedLogitsLoss)."""
    from ..ops.cross_entropy import fused_linear_cross_entropy
    return fused_linear_cross_entropy(h, weight, labels, ignore_index, tile_tokens, reduction)


class _GatherSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        ws = dist.get_world_size(group)
        ctx.rank, ctx.n = dist.get_rank(group), x.shape[0]
        out = torch.empty(ws * x.shape[0], *x.shape[1:], dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x.contiguous(), group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        return g[ctx.rank * ctx.n:(ctx.rank + 1) * ctx.n], None


def vocab_sequence_parallel_cross_entropy(logits, target, sp_group=None, ignore_index=-100):
    """Per-token CE of this rank's sequence shard, all-gathered over the SP group so every rank holds
    the full [S_total, ...] loss vector (reference sequence/cross_entropy.py)."""
    from ..ops.cross_entropy import cross_entropy
    # logits: [S_local, B, V] (reference layout) or [B, S_local, V]
    loss = cross_entropy(logits, target, ignore_index=ignore_index, reduction="none")
    if sp_group is None or dist.get_world_size(sp_group) == 1:
        return loss
    seq_first = loss.dim() == 2 and logits.dim() == 3 and logits.shape[0] == target.shape[0] and \
        target.shape[0] != logits.shape[1]
    if not seq_first and loss.dim() == 2:
        return _GatherSeq.apply(loss.transpose(0, 1).contiguous(), sp_group).transpose(0, 1)
    return _GatherSeq.apply(loss, sp_group)


# ----------------------------------------------------------------------------------- HF adapter
class UlyssesSPAttentionHF:
    """Drop-in HF ``attention_interface``: q/k/v arrive per rank as [B, H, S_local, D]; heads are
    scattered / sequence gathered with one all-to-all each way around the core attention."""

    def __init__(self, attn_fn, sp_group, num_heads, num_kv_heads, head_dim):
        self.attn_fn = attn_fn
        self.group = sp_group
        self.p = dist.get_world_size(sp_group) if sp_group is not None else 1
        self.nq, self.nkv, self.d = num_heads, num_kv_heads, head_dim

    def __call__(self, module, query, key, value, attention_mask=None, *args, **kwargs):
        from .layer import _SeqAllToAll
        p = self.p
        if p == 1:
            return self.attn_fn(module, query, key, value, attention_mask, *args, **kwargs)
        if key.shape[1] % p:  # GQA with fewer kv heads than ranks: replicate kv heads
            rep = p // math.gcd(key.shape[1], p)
            key = key.repeat_interleave(rep, dim=1)
            value = value.repeat_interleave(rep, dim=1)
        q, k, v = (_SeqAllToAll.apply(self.group, t.transpose(1, 2), True).transpose(1, 2)
                   for t in (query, key, value))
        out = self.attn_fn(module, q, k, v, None, *args, **kwargs)
        o, rest = (out[0], out[1:]) if isinstance(out, tuple) else (out, ())
        # HF attention functions return [B, S, H, D]
        o = _SeqAllToAll.apply(self.group, o, False)
        return (o,) + tuple(rest) if isinstance(out, tuple) else o


def register_with_transformers(model_config, core_attn_implementation="sdpa", sequence_parallel_size=1,
                               sp_group=None, name="ulysses"):
    """Register ``UlyssesSPAttentionHF`` as an HF attention implementation named ``name`` and return
    the configured callable (set ``config._attn_implementation = name`` on the model)."""
    from transformers.modeling_utils import ALL_ATTENTION_FUNCTIONS
    core = ALL_ATTENTION_FUNCTIONS[core_attn_implementation]
    if sp_group is None:
        from ..parallel import groups
        groups.initialize(sequence_parallel_size=sequence_parallel_size)
        sp_group = groups.get_sequence_parallel_group()
    hd = getattr(model_config, "head_dim", None) or model_config.hidden_size // model_config.num_attention_heads
    fn = UlyssesSPAttentionHF(core, sp_group, model_config.num_attention_heads,
                              getattr(model_config, "num_key_value_heads", model_config.num_attention_heads), hd)
    ALL_ATTENTION_FUNCTIONS.register(name, fn)
    return fn
