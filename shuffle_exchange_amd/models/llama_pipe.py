"""Llama as a pipeline layer list (``LayerSpec``s) for ``PipelineModule``.

The residual stream travels between stages as the pair ``(x, residual)`` (the true hidden state is
``x + residual``), exactly as the fused add+RMSNorm of the non-pipelined model consumes it, so a
stage boundary costs no extra elementwise pass. The last stage emits logits; ``llama_pipe_loss``
is the matching ``loss_fn`` (next-token shift + the HIP cross-entropy kernel).
Weight initialisation is identical to ``LlamaForCausalLM`` when ``seed_layers`` is off and the
module is built from the same global seed on one stage (used by the equivalence tests).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.cross_entropy import cross_entropy
from ..ops.norm import RMSNorm
from ..ops.rope import RopeCache
from ..runtime.pipe.module import LayerSpec, TiedLayerSpec
from .llama import LlamaConfig, LlamaDecoderLayer

_ROPE = {}


def _rope(cfg, device):
    key = (cfg.head_dim, cfg.max_position_embeddings, cfg.rope_theta, str(device))
    if key not in _ROPE:
        _ROPE[key] = RopeCache(cfg.head_dim, cfg.max_position_embeddings, cfg.rope_theta, device)
    return _ROPE[key]


class EmbeddingPipe(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.weight = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden_size))
        nn.init.normal_(self.weight, 0.0, cfg.initializer_range)

    def forward(self, input_ids):
        x = F.embedding(input_ids, self.weight)
        return x, torch.zeros_like(x)


def _tied_head(embed, inputs):
    h = inputs
    return F.linear(h, embed.weight)


class DecoderLayerPipe(LlamaDecoderLayer):
    def __init__(self, cfg: LlamaConfig):
        super().__init__(cfg)
        self.cfg = cfg
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0.0, cfg.initializer_range)

    def forward(self, inputs):
        x, res = inputs
        return super().forward(x, res, _rope(self.cfg, x.device))


class FinalNormPipe(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)

    def forward(self, inputs):
        x, res = inputs
        return self.norm(x, res)[0]


class LMHeadPipe(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden_size))
        nn.init.normal_(self.weight, 0.0, cfg.initializer_range)

    def forward(self, h):
        return F.linear(h, self.weight)


def llama_pipe_loss(logits, labels, ignore_index=-100):
    tgt = torch.cat([labels[:, 1:], torch.full_like(labels[:, :1], ignore_index)], dim=1)
    return cross_entropy(logits, tgt, ignore_index=ignore_index)


def llama_pipeline_layers(cfg: LlamaConfig):
    if cfg.tie_word_embeddings:
        first = TiedLayerSpec("embed", EmbeddingPipe, cfg)
        last = TiedLayerSpec("embed", EmbeddingPipe, cfg, forward_fn=_tied_head)
    else:
        first, last = LayerSpec(EmbeddingPipe, cfg), LayerSpec(LMHeadPipe, cfg)
    return [first] + [LayerSpec(DecoderLayerPipe, cfg) for _ in range(cfg.num_hidden_layers)] + \
        [LayerSpec(FinalNormPipe, cfg), last]


def llama_pipeline_module(cfg: LlamaConfig, num_stages, partition_method="parameters", **kw):
    from ..runtime.pipe.module import PipelineModule
    return PipelineModule(llama_pipeline_layers(cfg), num_stages=num_stages, loss_fn=llama_pipe_loss,
                          partition_method=partition_method, **kw)
