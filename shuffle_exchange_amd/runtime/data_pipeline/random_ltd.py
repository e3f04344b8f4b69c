"""Random layerwise token dropping (random-LTD).

Parity: reference runtime/data_pipeline/data_routing/basic_layer.py (``RandomLayerTokenDrop``),
scheduler.py (``RandomLTDScheduler``: kept-token count growing from min_value to max_value every
``require_steps`` / ``seq_per_step``), and ops/random_ltd (``token_sort_`` / ``token_gather`` /
``token_scatter_``): the gather / scatter are single ``index_select`` / ``index_copy`` launches on
the token axis (HBM-bound copies the vendor kernels already run at bandwidth).
"""
import torch
import torch.nn as nn


class RandomLTDScheduler:
    def __init__(self, config):
        sc = config.get("random_ltd_schedule", config)
        self.min_value = sc["min_value"]
        self.max_value = sc["max_value"]
        cfg = sc.get("schedule_config", {})
        self.seq_per_step = cfg.get("seq_per_step", 16)
        self.require_steps = cfg.get("require_steps", 100)
        self.current = self.min_value
        self.consumed_layer_tokens = 0
        # token selection draws from a stream keyed by (seed, global step, micro-step, layer) instead
        # of the global RNG: an activation-checkpoint recompute of the wrapped layer (which restores
        # only the global RNG) draws the SAME tokens as its forward, and a resumed run -- whose step
        # counters come from the checkpoint -- drops the same tokens as an uninterrupted one. Outside
        # an engine (no begin_micro_step) the key falls back to a running draw counter.
        self.seed = int(config.get("seed", 1234))
        self.draws = 0
        self._key = None
        self._counted = set()

    def begin_micro_step(self, global_step, micro_step):
        """Called by the engine once per training forward (never by a recompute)."""
        self._key = (int(global_step), int(micro_step))
        self._counted = set()

    def generator(self, device, layer_id=0):
        g = torch.Generator(device=device)
        if self._key is None:
            g.manual_seed((self.seed * 1_000_003 + self.draws) % (1 << 62))
            self.draws += 1
            return g
        step, micro = self._key
        g.manual_seed(((self.seed * 1_000_003 + step) * 4_099 + micro) * 257 + int(layer_id) & ((1 << 62) - 1))
        return g

    def count_tokens(self, layer_id, n):
        """consumed_layer_tokens, once per (micro-step, layer): a recompute does not count again."""
        if self._key is None:
            self.consumed_layer_tokens += n
            return
        if layer_id not in self._counted:
            self._counted.add(layer_id)
            self.consumed_layer_tokens += n

    def get_current_seq(self):
        return self.current

    def update_seq(self, global_step):
        steps = global_step // max(1, self.require_steps)
        self.current = min(self.max_value, self.min_value + steps * self.seq_per_step)
        return self.current

    def state_dict(self):
        return {"current": self.current, "consumed_layer_tokens": self.consumed_layer_tokens, "draws": self.draws}

    def load_state_dict(self, sd):
        self.current = sd["current"]
        self.consumed_layer_tokens = sd.get("consumed_layer_tokens", 0)
        self.draws = sd.get("draws", 0)


def token_sort_(idx):
    return torch.sort(idx, dim=-1).values


def gather_tokens(x, idx):
    """x: [B, S, H], idx: [B, k] sorted token ids -> [B, k, H] (HIP row gather, ops/rows.py)."""
    from ...ops.rows import gather_tokens as _g
    return _g(x, idx)


def scatter_tokens(full, part, idx):
    """Write part [B, k, H] back into full [B, S, H] at idx (out of place; HIP row scatter)."""
    from ...ops.rows import scatter_tokens as _s
    return _s(full, part, idx)


class RandomLayerTokenDrop(nn.Module):
    """Wraps a layer f(x [B, S, H], ...) so that during training it only processes ``k`` random
    tokens per sequence (sorted, so causal order is kept); the other tokens pass through unchanged.

    Positional arguments shaped like the hidden states (this framework's fused-residual stream:
    ``layer(x, res, rope, position_ids)`` -> ``(x, res)``) are gathered and scattered alongside, so
    a dropped token keeps x + res; a ``position_ids`` of None becomes the kept tokens' ORIGINAL
    positions (RoPE must not see the compacted order). Parity: reference
    data_routing/basic_layer.py ``RandomLayerTokenDrop``."""

    def __init__(self, layer, scheduler=None):
        super().__init__()
        self.layer = layer
        self.scheduler = scheduler
        self.reserved_length = None
        import inspect
        try:
            names = list(inspect.signature(layer.forward).parameters)
        except (TypeError, ValueError):
            names = []
        self._pos_arg = names.index("position_ids") if "position_ids" in names else None

    def init_config(self, config, scheduler, layer_id=0):
        self.scheduler = scheduler
        self.layer_id = layer_id

    def forward(self, x, *args, **kwargs):
        k = self.reserved_length if self.reserved_length is not None else (
            self.scheduler.get_current_seq() if self.scheduler is not None else x.shape[1])
        if not self.training or k >= x.shape[1]:
            return self.layer(x, *args, **kwargs)
        B, S, _ = x.shape
        lid = getattr(self, "layer_id", 0)
        gen = self.scheduler.generator(x.device, lid) if hasattr(self.scheduler, "generator") else None
        idx = token_sort_(torch.rand(B, S, device=x.device, generator=gen).topk(k, dim=1).indices)
        if hasattr(self.scheduler, "count_tokens"):
            self.scheduler.count_tokens(lid, B * k)
        elif self.scheduler is not None:
            self.scheduler.consumed_layer_tokens += B * k
        args = list(args)
        full = {0: x}
        for j, a in enumerate(args):
            if torch.is_tensor(a) and a.dim() == 3 and a.shape[:2] == (B, S):
                full[j + 1] = a
                args[j] = gather_tokens(a, idx)
        pj = self._pos_arg
        if pj is not None and pj - 1 < len(args) and pj >= 1:
            pos = args[pj - 1]
            if pos is None:
                pos = torch.arange(S, device=x.device).unsqueeze(0).expand(B, S)
            if torch.is_tensor(pos) and pos.shape[-1] == S:
                args[pj - 1] = torch.gather(pos.expand(B, S), 1, idx)
        elif "position_ids" in kwargs or pj is not None:
            pos = kwargs.get("position_ids")
            if pos is None:
                pos = torch.arange(S, device=x.device).unsqueeze(0).expand(B, S)
            kwargs["position_ids"] = torch.gather(pos.expand(B, S), 1, idx)
        out = self.layer(gather_tokens(x, idx), *args, **kwargs)
        if torch.is_tensor(out):
            return scatter_tokens(x, out, idx)
        outs = list(out)
        for j, o in enumerate(outs):
            if not (torch.is_tensor(o) and o.dim() == 3 and o.shape[:2] == (B, k)):
                continue
            src = full.get(j, x if j == 0 else None)
            if src is None:
                # an output stream the layer created (the fused residual of the first layer, whose
                # input residual is None): dropped tokens carry zero in it, so x + res == x for them
                src = torch.zeros((B, S) + tuple(o.shape[2:]), dtype=o.dtype, device=o.device)
            outs[j] = scatter_tokens(src, o, idx)
        return type(out)(outs) if isinstance(out, tuple) else outs


def convert_to_random_ltd(model, layer_ids, scheduler):
    """Wrap the decoder layers ``layer_ids`` (indices into the model's first ModuleList) with
    ``RandomLayerTokenDrop`` in place; returns the wrapped count (reference
    data_routing/helper.py ``convert_to_random_ltd``)."""
    for mod in model.modules():
        for name, child in mod.named_children():
            if isinstance(child, nn.ModuleList) and len(child) > 0:
                n = 0
                for i in sorted(layer_ids):
                    if not isinstance(child[i], RandomLayerTokenDrop):
                        child[i] = RandomLayerTokenDrop(child[i], scheduler)
                        child[i].layer_id = i
                    n += 1
                return n
    return 0
