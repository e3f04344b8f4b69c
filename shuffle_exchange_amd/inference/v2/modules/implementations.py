"""Registered implementations (reference inference/v2/modules/implementations/: blas_fp_linear,
quantized_linear (wf6af16), dense_blocked_attention, cutlass_multi_gemm_moe, ragged_embedding,
cuda_rms_norm / cuda_pre_ln ...), each a thin object over this framework's gfx950 ops."""
from dataclasses import dataclass
from typing import Optional

import torch

from ....ops import native
from .registry import register


# ------------------------------------------------------------------------------------- configs
@dataclass
class LinearConfig:
    in_features: int
    out_features: int
    dtype: torch.dtype = torch.bfloat16
    quantization: Optional[str] = None   # None | fp8 | fp6 | wf6af16 | fp4
    device_type: str = "cuda"


@dataclass
class AttentionConfig:
    head_dim: int
    n_heads: int
    n_kv_heads: int
    dtype: torch.dtype = torch.bfloat16
    window: int = 0
    device_type: str = "cuda"


@dataclass
class MoEConfig:
    n_experts: int
    top_k: int
    device_type: str = "cuda"


@dataclass
class EmbedConfig:
    vocab: int
    hidden: int
    dtype: torch.dtype = torch.bfloat16
    device_type: str = "cuda"


@dataclass
class NormConfig:
    kind: str        # rms | layer
    hidden: int
    device_type: str = "cuda"


def _hip(cfg):
    return cfg.device_type == "cuda" and native.hip_available()


# -------------------------------------------------------------------------------------- linear
@register("linear", "quantized_weight_only", priority=10)
class QuantizedWeightLinear:
    """fp8 (W8A16), fp6 (FP6-LLM wf6af16) or fp4 weight-only: decode-sized inputs (<= 16 rows)
    stream the quantized weight through the skinny MFMA kernels; larger inputs keep the bf16
    weight on hipBLASLt (the weight is kept for them)."""

    @staticmethod
    def supports(cfg):
        return cfg.quantization is not None and cfg.in_features % (128 if cfg.quantization != "fp8" else 16) == 0

    def __init__(self, cfg, weight, bias=None):
        from ....ops.fp_quantizer import quantized_weight
        self.cfg, self.weight, self.bias = cfg, weight, bias
        self.q = quantized_weight(weight, cfg.quantization)

    def __call__(self, x):
        from ....ops.linear import linear
        if x.shape[0] <= 16:
            return linear(x, self.q, self.bias)
        return linear(x, self.weight, self.bias)


@register("linear", "blas_fp_linear", priority=0)
class BlasLinear:
    """bf16 / fp16 / fp32: ops.linear (skinny MFMA kernel for <= 16 rows, hipBLASLt otherwise)."""

    @staticmethod
    def supports(cfg):
        return cfg.quantization is None

    def __init__(self, cfg, weight, bias=None):
        self.cfg, self.weight, self.bias = cfg, weight, bias

    def __call__(self, x):
        from ....ops.linear import linear
        return linear(x, self.weight, self.bias)


# ----------------------------------------------------------------------------------- attention
@register("attention", "dense_blocked_attention_flash_prefill", priority=10)
class PagedAttentionFlashPrefill:
    """Paged decode kernel (paged_attn.hip) for decode / continuation chunks; long fresh prompts
    take the flash-attention kernel (flash_attn.hip) on the contiguous prompt."""
    flash_prefill = True
    flash_min_tokens = 256

    @staticmethod
    def supports(cfg):
        return _hip(cfg) and cfg.head_dim == 128 and cfg.dtype == torch.bfloat16 and cfg.window == 0

    def __init__(self, cfg):
        self.cfg = cfg


@register("attention", "dense_blocked_attention", priority=0)
class PagedAttention:
    """Paged attention for every token (HIP kernel for head dims 64 / 128 / 256 with optional
    sliding window; the PyTorch gather path elsewhere -- ops/paged_attention.py)."""
    flash_prefill = False
    flash_min_tokens = 1 << 30

    @staticmethod
    def supports(cfg):
        return True

    def __init__(self, cfg):
        self.cfg = cfg


# ----------------------------------------------------------------------------------------- moe
@register("moe", "hip_topk_grouped", priority=10)
class HipTopKMoE:
    """Fused softmax + top-k gating kernel (moe.hip), tokens grouped by expert, per-expert GEMMs."""
    use_hip_gating = True

    @staticmethod
    def supports(cfg):
        return _hip(cfg) and cfg.n_experts <= 512

    def __init__(self, cfg):
        self.cfg = cfg


@register("moe", "torch_topk_grouped", priority=0)
class TorchTopKMoE:
    use_hip_gating = False

    @staticmethod
    def supports(cfg):
        return True

    def __init__(self, cfg):
        self.cfg = cfg


# --------------------------------------------------------------------------------------- embed
@register("embed", "ragged_embedding", priority=0)
class RaggedEmbedding:
    """Token rows gathered by the HIP row kernel (rows.hip; PyTorch index on CPU)."""

    @staticmethod
    def supports(cfg):
        return True

    def __init__(self, cfg, weight):
        self.cfg, self.weight = cfg, weight

    def __call__(self, ids, offset=0):
        from ....ops.rows import embed
        return embed(self.weight, ids, offset)


# ---------------------------------------------------------------------------------------- norm
@register("norm", "hip_fused_norm", priority=0)
class FusedNorm:
    """RMSNorm / LayerNorm with the fused residual add (norm.hip)."""

    @staticmethod
    def supports(cfg):
        return cfg.kind in ("rms", "layer")

    def __init__(self, cfg):
        self.cfg = cfg
