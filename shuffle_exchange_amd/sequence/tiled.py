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
def sxe_flash_attention_forward(module, query, key, value, attention_mask=None, dropout=0.0, scaling=None,
                                is_causal=None, **kwargs):
    """HF ``ALL_ATTENTION_FUNCTIONS`` entry running the gfx950 flash kernel (ops/attention.py):
    q/k/v [B, H, S, D] in, ([B, S, H, D], None) out -- the HF attention-function convention. A
    causal (or absent) mask runs the fused causal kernel; an explicit non-causal 4-D mask, dropout
    or an uncovered shape falls back to SDPA with the mask."""
    from ..ops.attention import attention, hip_paddable, hip_supported
    causal = getattr(module, "is_causal", True) if is_causal is None else bool(is_causal)
    q, k, v = (t.transpose(1, 2) for t in (query, key, value))
    plain = attention_mask is None or attention_mask.dim() != 4
    if (query.is_cuda and plain and not dropout and (hip_supported(q, k, v) or hip_paddable(q, k, v))):
        return attention(q, k, v, causal=causal, softmax_scale=scaling), None
    if key.shape[1] != query.shape[1]:
        rep = query.shape[1] // key.shape[1]
        key, value = key.repeat_interleave(rep, 1), value.repeat_interleave(rep, 1)
    m = attention_mask if (attention_mask is not None and attention_mask.dim() == 4) else None
    o = torch.nn.functional.scaled_dot_product_attention(query, key, value, attn_mask=m, dropout_p=dropout,
                                                         is_causal=causal and m is None, scale=scaling)
    return o.transpose(1, 2), None


class UlyssesSPAttentionHF:
    """Drop-in HF ``attention_interface``: q/k/v arrive per rank as [B, H, S_local, D]; heads are
    scattered / sequence gathered with one all-to-all each way around the core attention.

    Reference runtime/sequence_parallel/ulysses_sp.py:47-335. As there, ``position_ids`` (needed
    unsharded by packed-sample core attention) are all-gathered over the SP group before the core
    call (:269-272), and ``skip_all_but_last_attention_debug_mode`` runs only every
    ``num_hidden_layers``-th core attention, feeding the query through for the others (:295-315:
    memory-fit checks at long sequence lengths; the loss is meaningless). A 2-D padding mask
    [B, S_local] is all-gathered to [B, S] the same way; a 4-D mask built by HF for the LOCAL shard
    cannot describe the global sequence and is dropped (the core runs causal)."""

    def __init__(self, attn_fn, sp_group, num_heads, num_kv_heads, head_dim, num_hidden_layers=1):
        self.attn_fn = attn_fn
        self.group = sp_group
        self.p = dist.get_world_size(sp_group) if sp_group is not None else 1
        self.nq, self.nkv, self.d = num_heads, num_kv_heads, head_dim
        if self.nq % self.p:
            raise ValueError(f"attention head count {self.nq} is not divisible by SP size {self.p}")
        if not (self.nkv % self.p == 0 or self.p % self.nkv == 0):
            raise ValueError(f"KV head count {self.nkv} and SP size {self.p}: one must divide the other")
        self.num_hidden_layers = max(1, int(num_hidden_layers))
        self.skip_all_but_last_attention_debug_mode = False
        self.rotating_layer_counter = 0

    def _gather_seq(self, t, dim):
        parts = [torch.empty_like(t) for _ in range(self.p)]
        dist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.cat(parts, dim=dim)

    def __call__(self, module, query, key, value, attention_mask=None, *args, **kwargs):
        from .layer import _SeqAllToAll
        p = self.p
        if p == 1:
            return self.attn_fn(module, query, key, value, attention_mask, *args, **kwargs)
        if kwargs.get("position_ids") is not None:
            kwargs["position_ids"] = self._gather_seq(kwargs["position_ids"], 1)
        if attention_mask is not None:
            attention_mask = self._gather_seq(attention_mask, 1) if attention_mask.dim() == 2 else None
        if key.shape[1] % p:  # GQA with fewer kv heads than ranks: replicate kv heads
            rep = p // math.gcd(key.shape[1], p)
            key = key.repeat_interleave(rep, dim=1)
            value = value.repeat_interleave(rep, dim=1)
            if hasattr(module, "num_key_value_groups"):
                module.num_key_value_groups = query.shape[1] // key.shape[1]
        q, k, v = (_SeqAllToAll.apply(self.group, t.transpose(1, 2), True).transpose(1, 2)
                   for t in (query, key, value))
        if self.skip_all_but_last_attention_debug_mode:
            self.rotating_layer_counter = (self.rotating_layer_counter + 1) % self.num_hidden_layers
            if self.rotating_layer_counter != 0:
                out = (q.transpose(1, 2), None)  # bogus data of the right shape
            else:
                out = self.attn_fn(module, q, k, v, attention_mask, *args, **kwargs)
        else:
            out = self.attn_fn(module, q, k, v, attention_mask, *args, **kwargs)
        o, rest = (out[0], out[1:]) if isinstance(out, tuple) else (out, ())
        # HF attention functions return [B, S, H, D]
        o = _SeqAllToAll.apply(self.group, o.contiguous(), False)
        return (o,) + tuple(rest) if isinstance(out, tuple) else o


def register_with_transformers(model_config, core_attn_implementation=None, sequence_parallel_size=1,
                               sp_group=None, name="ulysses"):
    """Register ``UlyssesSPAttentionHF`` as an HF attention implementation named ``name`` and return
    the configured callable (set ``config._attn_implementation = name`` on the model). The default
    core attention is the gfx950 flash kernel (registered as ``"sxe_flash"``); pass e.g. ``"sdpa"``
    for an HF one."""
    from transformers.modeling_utils import ALL_ATTENTION_FUNCTIONS
    ALL_ATTENTION_FUNCTIONS.register("sxe_flash", sxe_flash_attention_forward)
    core = ALL_ATTENTION_FUNCTIONS[core_attn_implementation or "sxe_flash"]
    if sp_group is None:
        from ..parallel import groups
        groups.initialize(sequence_parallel_size=sequence_parallel_size)
        sp_group = groups.get_sequence_parallel_group()
    hd = getattr(model_config, "head_dim", None) or model_config.hidden_size // model_config.num_attention_heads
    fn = UlyssesSPAttentionHF(core, sp_group, model_config.num_attention_heads,
                              getattr(model_config, "num_key_value_heads", model_config.num_attention_heads), hd,
                              getattr(model_config, "num_hidden_layers", 1))
    ALL_ATTENTION_FUNCTIONS.register(name, fn)
    return fn


class AutogradComputeMLP(torch.autograd.Function):
    """Run ``fn(self, x)`` without keeping its activations: forward under no_grad, backward
    recomputes it with grad (reference ulysses_sp.py:864). Parameter gradients arrive in one
    delivery, so ZeRO sees them once. Usage: ``AutogradComputeMLP.apply(mlp_forward, mlp, x)``."""

    @staticmethod
    def forward(ctx, fn, self, x):
        ctx.fn, ctx.self = fn, self
        ctx.save_for_backward(x)
        with torch.no_grad():
            return fn(self, x)

    @staticmethod
    def backward(ctx, *grads):
        (x,) = ctx.saved_tensors
        x1 = x.detach().requires_grad_(x.requires_grad)
        with torch.enable_grad():
            out = ctx.fn(ctx.self, x1)
        torch.autograd.backward(out, grads[0])
        return None, None, x1.grad


class UlyssesSPFwdLossBwdWithLogits:
    """One Ulysses-SP training micro-step from a data-parallel batch whose logits the loss needs
    whole (reference ulysses_sp.py:1064): the SP ranks all-gather their batches (variable sequence
    lengths allowed), then run them one after another -- each sharded over the SP group along the
    sequence, forward, loss from the shifted labels of this rank's shard (tiled over
    ``num_loss_logit_shards`` when the logits are large), SP-weighted mean by the count of
    non-ignored labels per shard, backward -- with the gradient-accumulation boundary only after
    the last. Returns the mean loss."""

    def __init__(self, model, model_unwrapped, device, num_loss_logit_shards="auto", **kwargs):
        from ..parallel import groups
        self.model = model
        self.model_unwrapped = model_unwrapped
        self.device = device
        self.num_loss_logit_shards = num_loss_logit_shards
        self.kwargs = kwargs
        self.sp_group = groups.get_sequence_parallel_group()
        self.sp_world_size = groups.get_sequence_parallel_world_size()
        self.sp_rank = groups.get_sequence_parallel_rank()

    def _gather_batches(self, batch):
        n = self.sp_world_size
        seqlen = torch.tensor([batch["input_ids"].shape[1]], dtype=torch.int64, device=self.device)
        lens = [torch.zeros_like(seqlen) for _ in range(n)]
        dist.all_gather(lens, seqlen, group=self.sp_group)
        lens = [int(x.item()) for x in lens]
        micro = [{} for _ in range(n)]
        for k, v in batch.items():
            v = v.to(self.device)
            L = max(lens)
            pad = torch.nn.functional.pad(v, (0, L - v.shape[1]), value=-100 if k == "labels" else 0)
            parts = [torch.empty_like(pad) for _ in range(n)]
            dist.all_gather(parts, pad.contiguous(), group=self.sp_group)
            for r in range(n):
                micro[r][k] = parts[r][:, :lens[r]]
        return micro

    def _loss(self, logits, shift_labels):
        from ..ops.cross_entropy import cross_entropy
        if bool((shift_labels == -100).all()):
            return (logits.sum() * 0.0).float()
        V = logits.shape[-1]
        shards = self.num_loss_logit_shards
        if shards == "auto":
            shards = max(1, math.ceil(logits.numel() * 4 / 2**30))  # ~1 GB of fp32 logits per shard
        lg, lb = logits.reshape(-1, V), shift_labels.reshape(-1)
        n = (lb != -100).sum().clamp_min(1)
        total = sum(cross_entropy(a, b, ignore_index=-100, reduction="sum")
                    for a, b in zip(lg.chunk(shards), lb.chunk(shards)))
        return total / n

    def sp_fwd_loss_bwd(self, batch):
        if not (batch["input_ids"].shape == batch["position_ids"].shape == batch["labels"].shape):
            raise ValueError("input_ids, position_ids and labels must have the same shape for Ulysses SP")
        micro = self._gather_batches(batch)
        n = self.sp_world_size
        self.model.set_gradient_accumulation_boundary(False)
        losses = []
        for sub in range(n):
            b = dict(micro[sub])
            S = b["input_ids"].shape[1]
            if S % n:
                raise ValueError(f"sub-step {sub}: seqlen {S} is not divisible by the SP size {n}")
            c = S // n
            labels = torch.nn.functional.pad(b.pop("labels"), (0, 1), value=-100)
            shift = labels[..., 1:]
            # exact per-shard counts of the shifted labels that contribute (the reference subtracts one
            # per shard as an approximation; the shift drops one label per SEQUENCE, in the last shard)
            counts = [int((shift[:, c * r:c * (r + 1)] != -100).sum().item()) for r in range(n)]
            b = {k: v[:, c * self.sp_rank:c * (self.sp_rank + 1)] for k, v in b.items()}
            shift = shift[:, c * self.sp_rank:c * (self.sp_rank + 1)]
            if sub == n - 1:
                self.model.set_gradient_accumulation_boundary(True)
            out = self.model(**b)
            logits = getattr(out, "logits", out)
            loss = self._loss(logits, shift)
            tot = max(1, sum(counts))
            # this framework's SP gradient convention: each SP rank back-propagates its shard's SHARE
            # of the sample loss and the ZeRO reduction sums the SP ranks (engine sp_scale); the
            # reference back-propagates the all-gathered total on every rank and divides by sp
            share = loss * (counts[self.sp_rank] / tot)
            full = share.detach().clone()
            dist.all_reduce(full, group=self.sp_group)
            self.model.backward(share.reshape(()))
            losses.append(float(full))
        return sum(losses) / len(losses) if losses else float("nan")

