"""Llama-family decoder (Llama-2/3, Mistral-style GQA) built on this repo's HIP ops.

MI355X-first layer anatomy (all hot elementwise work in HIP kernels, all GEMMs as large single
hipBLASLt calls):
  a, h   = rmsnorm(x + res)            fused residual-add + RMSNorm          (ops/norm.py)
  qkv    = a @ Wqkv^T                  ONE GEMM for q, k, v  -> [B, S, Hq+2Hkv, D]
  rope_(qkv[:, :, :Hq+Hkv])            in place, no transposes               (ops/rope.py)
  o      = attention(q, k, v)          [B, S, H, D] strided views, GQA       (ops/attention.py)
  m, h2  = rmsnorm(o @ Wo^T + h)
  out    = swiglu(m @ Wgu^T) @ Wd^T    ONE GEMM for gate|up; weight grads on  (ops/mlp.py)
                                       token-minor copies the gated kernels write
  loss   = fused_linear_cross_entropy(final_norm(...), Wlm)                  (ops/cross_entropy.py)

Reference counterparts: the inference-v2 Llama implementation
(deepspeed/inference/v2/model_implementations/llama_v2/model.py:133-199) and the HF models the
reference trains through ``deepspeed.initialize``. Config presets match Llama-3 8B / 70B.
"""
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.mlp import swiglu_mlp
from ..runtime.activation_checkpointing.checkpointing import checkpoint
from ..runtime.zero.partition_parameters import local_shard
from ..ops.attention import attention_qkv_rope, qkv_proj_attention
from ..ops.cross_entropy import fused_linear_cross_entropy
from ..ops.linear import Embedding, Linear, linear
from ..ops.norm import RMSNorm
from ..ops.rope import RopeCache
from ..sequence.layer import ulysses_qkv_attention
from ..sequence.ring_attention import ring_qkv_attention


def _sp_group():
    from ..parallel import groups
    return groups.get_sequence_parallel_group() if groups.get_sequence_parallel_world_size() > 1 else None


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 8
    head_dim: Optional[int] = None
    rope_theta: float = 500000.0
    rms_norm_eps: float = 1e-5
    max_position_embeddings: int = 8192
    tie_word_embeddings: bool = False
    initializer_range: float = 0.02
    activation_checkpointing: bool = False
    # what activation checkpointing recomputes: "full" = the whole decoder layer (attention
    # included); "mlp" = only the MLP sub-block (its gate_up / SwiGLU activations, ~70 % of a
    # layer's saved bytes, are recomputed by GEMMs; the flash-attention forward is NOT re-run)
    ac_policy: str = "full"
    # how many decoder layers (the first N) the checkpoint policy covers; None = all of them. 288 GB
    # of HBM often fits the activations of SOME layers: recomputing only the rest is faster (the
    # model-side analogue of activation_checkpointing.number_checkpoints, reference
    # runtime/activation_checkpointing/checkpointing.py:1007)
    ac_layers: Optional[int] = None
    loss_chunk_tokens: Optional[int] = None
    sequence_parallel: bool = False  # Ulysses: inputs are [B, S/sp] chunks of the SP group
    sp_mode: str = "ulysses"         # "ring" / "ring_zigzag": ring attention (context parallelism) over
                                     # the SP group, contiguous or zig-zag (sequence.ring_attention) shards
    fpdt_chunk_size: int = 0         # >0: FPDT chunked attention (global chunk length); inputs laid
                                     # out by sequence.fpdt_layer.FPDT_InputConstruct
    fpdt_offload: bool = False       # FPDT: keep the saved q/k/v/o chunks in pinned host memory
    extra: dict = field(default_factory=dict)

    def __post_init__(self):
        if self.ac_policy not in ("full", "mlp"):
            raise ValueError(f"ac_policy must be 'full' or 'mlp', got {self.ac_policy!r}")
        if self.head_dim is None:
            self.head_dim = self.hidden_size // self.num_attention_heads

    def num_params(self):
        h, i, v, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_hidden_layers
        d = self.head_dim
        qkv = h * (self.num_attention_heads + 2 * self.num_key_value_heads) * d
        per_layer = qkv + self.num_attention_heads * d * h + 3 * h * i + 2 * h
        emb = v * h * (1 if self.tie_word_embeddings else 2)
        return L * per_layer + emb + h

    def flops_per_token(self, seq_len):
        """Training FLOPs per token: 6 * non-embedding-params + causal attention (fwd 2*S*h per
        layer for QK^T and PV, halved by causality, x3 for fwd+bwd)."""
        n = self.num_params() - self.vocab_size * self.hidden_size  # exclude input embedding (lookup)
        attn = 3 * 2 * 2 * self.num_hidden_layers * seq_len * self.num_attention_heads * self.head_dim / 2
        return 6 * n + attn


PRESETS = {
    "llama3-8b": dict(),
    "llama3-70b": dict(hidden_size=8192, intermediate_size=28672, num_hidden_layers=80, num_attention_heads=64,
                       num_key_value_heads=8),
    "llama2-7b": dict(vocab_size=32000, hidden_size=4096, intermediate_size=11008, num_hidden_layers=32,
                      num_attention_heads=32, num_key_value_heads=32, rope_theta=10000.0, rms_norm_eps=1e-5,
                      max_position_embeddings=4096),
    "llama-tiny": dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256),
    # 8-rank rehearsals: 16 query / 8 KV heads so Ulysses SP=8 is legal (Llama-3-8B's 32/8 ratio halved)
    "llama-tiny8": dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                        num_attention_heads=16, num_key_value_heads=8, max_position_embeddings=256),
}


def llama_config(name, **overrides):
    d = dict(PRESETS[name])
    d.update(overrides)
    return LlamaConfig(**d)


class LlamaAttention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.nq, self.nkv, self.d = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        std = cfg.initializer_range
        self.qkv_proj = Linear(cfg.hidden_size, (self.nq + 2 * self.nkv) * self.d, bias=False, init_std=std)
        self.o_proj = Linear(self.nq * self.d, cfg.hidden_size, bias=False, init_std=std)
        # AutoTP: split q|k|v by heads (GQA-aware); nq/nkv become per-rank counts
        self.qkv_proj._tp_layout = ("heads", [self.nq, self.nkv, self.nkv], self.d)
        self.o_proj._tp_row_parallel = True

    def forward(self, x, rope: RopeCache, position_ids=None):
        B, S, _ = x.shape
        spg = _sp_group() if self.cfg.sequence_parallel else None
        if not self.cfg.fpdt_chunk_size and spg is None:
            # QKV projection + attention as one node: its weight gradient runs on token-minor
            # operands (ops/attention.py _QKVProjAttn)
            o = qkv_proj_attention(x, self.qkv_proj, self.nq, self.nkv, rope, position_ids, causal=True)
            return self.o_proj(o.reshape(B, S, self.nq * self.d))
        qkv = self.qkv_proj(x).view(B, S, self.nq + 2 * self.nkv, self.d)
        if self.cfg.fpdt_chunk_size:
            from ..sequence.fpdt_layer import fpdt_attention
            from .. import comm as dist
            p = dist.get_world_size(spg) if spg is not None else 1
            n = max(1, S * p // self.cfg.fpdt_chunk_size)
            o = fpdt_attention(qkv, self.nq, self.nkv, rope, spg, n, offload=self.cfg.fpdt_offload)
        elif spg is not None and self.cfg.sp_mode in ("ring", "ring_zigzag"):
            o = ring_qkv_attention(qkv, self.nq, self.nkv, rope, spg, position_ids, causal=True,
                                   layout="zigzag" if self.cfg.sp_mode == "ring_zigzag" else "contiguous")
        elif spg is not None:
            o = ulysses_qkv_attention(qkv, self.nq, self.nkv, rope, spg, position_ids, causal=True)
        else:
            o = attention_qkv_rope(qkv, self.nq, self.nkv, rope, position_ids, causal=True)
        return self.o_proj(o.reshape(B, S, self.nq * self.d))

    def tp_shard_(self, tp):
        assert self.nq % tp == 0 and self.nkv % tp == 0, "heads must divide the TP degree"
        self.nq //= tp
        self.nkv //= tp


class LlamaMLP(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        std = cfg.initializer_range
        self.gate_up_proj = Linear(cfg.hidden_size, 2 * cfg.intermediate_size, bias=False, init_std=std)
        self.down_proj = Linear(cfg.intermediate_size, cfg.hidden_size, bias=False, init_std=std)
        self.gate_up_proj._tp_layout = ("chunks", 2)
        self.down_proj._tp_row_parallel = True

    def forward(self, x):
        # GPU training: one autograd node whose weight-gradient GEMMs run on token-minor operands
        # written by the dual-layout gated kernels (ops/mlp.py); otherwise the module path
        return swiglu_mlp(x, self.gate_up_proj, self.down_proj)


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.self_attn = LlamaAttention(cfg)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.mlp = LlamaMLP(cfg)
        self.ckpt_mlp = cfg.activation_checkpointing and cfg.ac_policy == "mlp"

    def forward(self, x, residual, rope, position_ids=None):
        """(x, residual) -> (mlp_out, new_residual); the true hidden state is x + residual."""
        if residual is None:
            a, h = self.input_layernorm(x), x
        else:
            a, h = self.input_layernorm(x, residual)
        attn = self.self_attn(a, rope, position_ids)
        m, h2 = self.post_attention_layernorm(attn, h)
        if self.ckpt_mlp and self.training and torch.is_grad_enabled():
            return checkpoint(self.mlp, m), h2
        return self.mlp(m), h2


class LMHeadLoss(nn.Module):
    """LM head as a module (so ZeRO-3 fetch hooks see it); returns the mean CE loss when labels are
    given (labels are the input ids, shifted here: position t predicts t+1), else logits."""

    def __init__(self, cfg: LlamaConfig, weight=None):
        super().__init__()
        self.cfg = cfg
        if weight is None:
            self.weight = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden_size))
            with torch.no_grad():
                self.weight.normal_(0.0, cfg.initializer_range)
        else:
            self.weight = weight

    def forward(self, h, labels=None, ignore_index=-100, shift_labels=True):
        if labels is None:
            return F.linear(h, self.weight)
        if shift_labels:
            tgt = torch.cat([labels[:, 1:], torch.full_like(labels[:, :1], ignore_index)], dim=1)
        else:
            tgt = labels  # already shifted over the full sequence (sequence-parallel data adapter)
        spg = _sp_group() if self.cfg.sequence_parallel else None
        if spg is None:
            return fused_linear_cross_entropy(h, self.weight, tgt, ignore_index, self.cfg.loss_chunk_tokens)
        # SP: this rank's token-sum / number of valid tokens over the whole sequence (reference
        # sequence/cross_entropy.py); summed over the SP group it is the full-sequence mean
        from .. import comm as dist
        n = (tgt != ignore_index).sum().float().reshape(1)
        dist.all_reduce(n, group=spg)
        s = fused_linear_cross_entropy(h, self.weight, tgt, ignore_index, self.cfg.loss_chunk_tokens,
                                       reduction="sum")
        return s / n.clamp_min(1.0).squeeze(0)


def _ac_covers(cfg, i):
    """Layer i is under the activation-checkpoint policy (``ac_layers``: the first N layers only)."""
    return cfg.ac_layers is None or i < cfg.ac_layers


class LlamaForCausalLM(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.embed_tokens = Embedding(cfg.vocab_size, cfg.hidden_size, init_std=cfg.initializer_range)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        for i, layer in enumerate(self.layers):
            layer.ckpt_mlp = layer.ckpt_mlp and _ac_covers(cfg, i)
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.lm_head = LMHeadLoss(cfg, self.embed_tokens.weight if cfg.tie_word_embeddings else None)
        self._rope = None
        # every weight was initialised N(0, std) by its own constructor, i.e. on the whole tensor
        # before a partitioning zero.Init cut it: the model depends on the seed, not on the world size
        self._init_remaining()

    @torch.no_grad()
    def _init_remaining(self):
        """N(0, std) for Linear/Embedding modules that did not initialise themselves (e.g. MoE
        routers): on this rank's construction partition when zero.Init partitioned them."""
        std = self.cfg.initializer_range
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)) and not getattr(m, "_sxe_inited", False):
                local_shard(m.weight).normal_(0.0, std)

    @torch.no_grad()
    def reset_parameters(self):
        # element-wise i.i.d. init: under a partitioning zero.Init each rank initialises its own
        # construction partition (local_shard), which is the same distribution as the full tensor
        std = self.cfg.initializer_range
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                local_shard(m.weight).normal_(0.0, std)
        if not self.cfg.tie_word_embeddings:
            local_shard(self.lm_head.weight).normal_(0.0, std)

    def rope(self, device):
        if self._rope is None or self._rope.cos.device != device:
            self._rope = RopeCache(self.cfg.head_dim, self.cfg.max_position_embeddings, self.cfg.rope_theta, device)
        return self._rope

    def forward(self, input_ids, labels=None, position_ids=None, shift_labels=True):
        x = self.embed_tokens(input_ids)
        rope = self.rope(x.device)
        res = None
        for i, layer in enumerate(self.layers):
            if (self.cfg.activation_checkpointing and self.cfg.ac_policy == "full" and self.training
                    and torch.is_grad_enabled() and _ac_covers(self.cfg, i)):
                x, res = checkpoint(layer, x, res, rope, position_ids)
            else:
                x, res = layer(x, res, rope, position_ids)
        h = self.norm(x, res)[0] if res is not None else self.norm(x)
        return self.lm_head(h, labels, shift_labels=shift_labels)
