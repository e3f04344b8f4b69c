"""Mixtral-style sparse MoE decoder (Llama attention + top-2 routed SwiGLU experts).

The expert FFN is ``moe.MoE`` (expert-parallel all-to-all over the EP group, batched expert GEMMs);
everything else is the Llama layer of ``models/llama.py``. The router load-balancing loss
(``router_aux_loss_coef`` x sum of per-layer aux losses) is added to the LM loss.
Presets: mixtral-8x7b (46.7B params: 32 layers, 8 experts, top-2) and mixtral-tiny (tests).
"""
from dataclasses import dataclass

import torch
import torch.nn as nn

from ..moe.layer import MoE
from ..ops.linear import Embedding
from ..runtime.activation_checkpointing.checkpointing import checkpoint
from ..ops.norm import RMSNorm
from .llama import LlamaAttention, LlamaConfig, LlamaForCausalLM, LMHeadLoss


@dataclass
class MixtralConfig(LlamaConfig):
    num_local_experts: int = 8
    num_experts_per_tok: int = 2
    ep_size: int = 1
    capacity_factor: float = 1.25
    router_aux_loss_coef: float = 0.02
    drop_tokens: bool = True
    min_capacity: int = 4
    top2_2nd_expert_sampling: bool = True  # reference MoE default (HF Mixtral routes top-2 greedily)
    enable_expert_tensor_parallelism: bool = False

    def num_params(self):
        h, i, L = self.hidden_size, self.intermediate_size, self.num_hidden_layers
        d = self.head_dim
        attn = h * (self.num_attention_heads + 2 * self.num_key_value_heads) * d + self.num_attention_heads * d * h
        per_layer = attn + self.num_local_experts * 3 * h * i + h * self.num_local_experts + 2 * h
        return L * per_layer + 2 * self.vocab_size * h + h

    def active_params_per_token(self):
        h, i, L = self.hidden_size, self.intermediate_size, self.num_hidden_layers
        d = self.head_dim
        attn = h * (self.num_attention_heads + 2 * self.num_key_value_heads) * d + self.num_attention_heads * d * h
        return L * (attn + self.num_experts_per_tok * 3 * h * i) + self.vocab_size * h


PRESETS = {
    "mixtral-8x7b": dict(vocab_size=32000, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                         num_attention_heads=32, num_key_value_heads=8, rope_theta=1e6, max_position_embeddings=32768),
    "mixtral-tiny": dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                         num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256,
                         num_local_experts=4),
    # 8-rank rehearsals: 8 experts (EP=8 legal, one expert per rank, like Mixtral-8x7B at N=8)
    "mixtral-tiny8": dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                          num_attention_heads=8, num_key_value_heads=8, max_position_embeddings=256,
                          num_local_experts=8),
}


def mixtral_config(name, **kw):
    d = dict(PRESETS[name])
    d.update(kw)
    return MixtralConfig(**d)


class MixtralDecoderLayer(nn.Module):
    def __init__(self, cfg: MixtralConfig):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.self_attn = LlamaAttention(cfg)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.block_sparse_moe = MoE(cfg.hidden_size, None, cfg.num_local_experts, cfg.ep_size,
                                    k=cfg.num_experts_per_tok, capacity_factor=cfg.capacity_factor,
                                    eval_capacity_factor=cfg.capacity_factor, min_capacity=cfg.min_capacity,
                                    drop_tokens=cfg.drop_tokens, intermediate_size=cfg.intermediate_size,
                                    top2_2nd_expert_sampling=cfg.top2_2nd_expert_sampling,
                                    enable_expert_tensor_parallelism=cfg.enable_expert_tensor_parallelism)

    def forward(self, x, residual, rope, position_ids=None):
        if residual is None:
            a, h = self.input_layernorm(x), x
        else:
            a, h = self.input_layernorm(x, residual)
        attn = self.self_attn(a, rope, position_ids)
        m, h2 = self.post_attention_layernorm(attn, h)
        out, l_aux, _ = self.block_sparse_moe(m)
        return out, h2, l_aux


class MixtralForCausalLM(LlamaForCausalLM):
    def __init__(self, cfg: MixtralConfig):
        nn.Module.__init__(self)
        self.cfg = cfg
        self.embed_tokens = Embedding(cfg.vocab_size, cfg.hidden_size, init_std=cfg.initializer_range)
        self.layers = nn.ModuleList([MixtralDecoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.lm_head = LMHeadLoss(cfg, None)
        self._rope = None
        self._init_remaining()

    def forward(self, input_ids, labels=None, position_ids=None):
        x = self.embed_tokens(input_ids)
        rope = self.rope(x.device)
        res = None
        aux = []
        for layer in self.layers:
            if self.cfg.activation_checkpointing and self.training and torch.is_grad_enabled():
                x, res, l_aux = checkpoint(layer, x, res, rope, position_ids)
            else:
                x, res, l_aux = layer(x, res, rope, position_ids)
            aux.append(l_aux)
        h = self.norm(x, res)[0]
        out = self.lm_head(h, labels)
        if labels is not None and self.cfg.router_aux_loss_coef:
            out = out + self.cfg.router_aux_loss_coef * torch.stack([a.float() for a in aux]).sum()
        return out
