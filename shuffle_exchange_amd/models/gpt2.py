"""GPT-2 (learned positions, LayerNorm, GELU MLP, tied LM head) on this repo's ops.

Used by the plumbing configuration of BASELINE.json ("GPT-2 small ZeRO-1 on CPU/gloo world_size=2")
and as the LayerNorm/GELU/bias path of the kernel set. Presets: gpt2 (124M), gpt2-medium, gpt2-large,
gpt2-tiny (tests).
"""
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.activation import bias_gelu
from ..ops.attention import attention
from ..ops.cross_entropy import cross_entropy
from ..ops.linear import Embedding, Linear
from ..ops.norm import LayerNorm
from ..runtime.zero.partition_parameters import local_shard


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    layer_norm_epsilon: float = 1e-5
    initializer_range: float = 0.02

    def num_params(self):
        h, L = self.n_embd, self.n_layer
        per = 4 * h * h + 4 * h + 8 * h * h + 5 * h + 4 * h
        return self.vocab_size * h + self.n_positions * h + L * per + 2 * h


PRESETS = {
    "gpt2": dict(),
    "gpt2-medium": dict(n_embd=1024, n_layer=24, n_head=16),
    "gpt2-large": dict(n_embd=1280, n_layer=36, n_head=20),
    "gpt2-tiny": dict(vocab_size=256, n_positions=64, n_embd=64, n_layer=2, n_head=4),
}


def gpt2_config(name, **kw):
    d = dict(PRESETS[name])
    d.update(kw)
    return GPT2Config(**d)


class GPT2Block(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        h = cfg.n_embd
        self.n_head = cfg.n_head
        self.head_dim = h // cfg.n_head
        self.ln_1 = LayerNorm(h, cfg.layer_norm_epsilon)
        std = cfg.initializer_range
        self.c_attn = Linear(h, 3 * h, init_std=std)
        self.c_proj = Linear(h, h, init_std=std)
        self.ln_2 = LayerNorm(h, cfg.layer_norm_epsilon)
        self.c_fc = Linear(h, 4 * h, init_std=std)
        self.mlp_proj = Linear(4 * h, h, init_std=std)
        self.c_attn._tp_layout = ("chunks", 3)
        self.c_proj._tp_row_parallel = True
        self.mlp_proj._tp_row_parallel = True

    def tp_shard_(self, tp):
        assert self.n_head % tp == 0
        self.n_head //= tp

    def forward(self, x):
        B, S, H = x.shape
        d = self.head_dim
        qkv = self.c_attn(self.ln_1(x)).view(B, S, 3, self.n_head, d)
        o = attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], causal=True)
        x = x + self.c_proj(o.reshape(B, S, self.n_head * d))
        m = bias_gelu(self.c_fc(self.ln_2(x), skip_bias=True), self.c_fc.bias)
        return x + self.mlp_proj(m)


class GPT2LMHeadModel(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.cfg = cfg
        self.wte = Embedding(cfg.vocab_size, cfg.n_embd, init_std=cfg.initializer_range)
        self.wpe = Embedding(cfg.n_positions, cfg.n_embd, init_std=cfg.initializer_range)
        self.h = nn.ModuleList([GPT2Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = LayerNorm(cfg.n_embd, cfg.layer_norm_epsilon)
        # weights initialise themselves in their constructors (world-size invariant under zero.Init)

    @torch.no_grad()
    def reset_parameters(self):
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                local_shard(m.weight).normal_(0.0, self.cfg.initializer_range)
            if isinstance(m, nn.Linear) and m.bias is not None:
                local_shard(m.bias).zero_()

    def forward(self, input_ids, labels=None):
        B, S = input_ids.shape
        pos = torch.arange(S, device=input_ids.device)
        x = self.wte(input_ids) + self.wpe(pos)[None]
        for blk in self.h:
            x = blk(x)
        logits = F.linear(self.ln_f(x), self.wte.weight)
        if labels is None:
            return logits
        tgt = torch.cat([labels[:, 1:], torch.full_like(labels[:, :1], -100)], dim=1)
        return cross_entropy(logits, tgt)
