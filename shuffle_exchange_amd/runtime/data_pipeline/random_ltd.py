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

    def get_current_seq(self):
        return self.current

    def update_seq(self, global_step):
        steps = global_step // max(1, self.require_steps)
        self.current = min(self.max_value, self.min_value + steps * self.seq_per_step)
        return self.current

    def state_dict(self):
        return {"current": self.current, "consumed_layer_tokens": self.consumed_layer_tokens}

    def load_state_dict(self, sd):
        self.current = sd["current"]
        self.consumed_layer_tokens = sd.get("consumed_layer_tokens", 0)


def token_sort_(idx):
    return torch.sort(idx, dim=-1).values


def gather_tokens(x, idx):
    """x: [B, S, H], idx: [B, k] sorted token ids -> [B, k, H]."""
    return torch.gather(x, 1, idx.unsqueeze(-1).expand(-1, -1, x.shape[-1]))


def scatter_tokens(full, part, idx):
    """Write part [B, k, H] back into full [B, S, H] at idx (out of place)."""
    return full.scatter(1, idx.unsqueeze(-1).expand(-1, -1, full.shape[-1]), part)


class RandomLayerTokenDrop(nn.Module):
    """Wraps a layer f([B, S, H], ...) so that during training it only processes ``k`` random
    tokens per sequence (the rest pass through unchanged)."""

    def __init__(self, layer, scheduler=None):
        super().__init__()
        self.layer = layer
        self.scheduler = scheduler
        self.reserved_length = None

    def forward(self, x, *args, **kwargs):
        k = self.reserved_length if self.reserved_length is not None else (
            self.scheduler.get_current_seq() if self.scheduler is not None else x.shape[1])
        if not self.training or k >= x.shape[1]:
            return self.layer(x, *args, **kwargs)
        B, S, _ = x.shape
        idx = token_sort_(torch.rand(B, S, device=x.device).topk(k, dim=1).indices)
        part = self.layer(gather_tokens(x, idx), *args, **kwargs)
        part = part[0] if isinstance(part, tuple) else part
        return scatter_tokens(x, part, idx)
