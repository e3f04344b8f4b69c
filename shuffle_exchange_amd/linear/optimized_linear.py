"""OptimizedLinear: frozen (optionally sharded and/or FP8-quantized) base weight + trainable LoRA.

Parity: reference linear/optimized_linear.py -- ``OptimizedLinear`` :18 (factory),
``LoRAOptimizedLinear`` :76 (base weight sharded over ``base_weight_sharding`` ranks and gathered
per forward, LoRA A/B trainable, ``lora_alpha / lora_r`` scaling), linear/config.py
(``LoRAConfig``, ``QuantizationConfig``), linear/quantization.py (``QuantizedParameter`` /
``QuantizedLinear`` with FP8 storage).

MI355X: the frozen base weight is stored as FP8 e4m3 with per-group scales (CDNA4 converts in
hardware, quant.hip) and dequantized to bf16 right before the GEMM; with sharding each rank keeps
1/N of the (quantized) rows and one all-gather per forward rebuilds the weight over xGMI.
"""
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import comm as dist
from ..ops.linear import linear


@dataclass
class LoRAConfig:
    lora_r: int = 64
    lora_alpha: float = 16.0
    base_weight_sharding: int = 1
    offload: bool = False
    target_mods: tuple = ("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj",
                          "qkv_proj", "gate_up_proj")


@dataclass
class QuantizationConfig:
    q_bits: int = 8
    mantissa_bits: int = 3
    group_size: int = 512
    q_dtype: torch.dtype = torch.uint8


class QuantizedParameter(nn.Parameter):
    """Frozen weight kept as FP8 + scales; ``.dequantized()`` returns the bf16 tensor."""

    def __new__(cls, data, quantization_config=None, requires_grad=False):
        from ..ops.quantizer import quantize_fp8
        qc = quantization_config or QuantizationConfig()
        flat = data.detach().reshape(-1)
        pad = (-flat.numel()) % qc.group_size
        if pad:
            flat = torch.cat([flat, flat.new_zeros(pad)])
        q, s = quantize_fp8(flat, qc.group_size)
        self = super().__new__(cls, q, requires_grad=False)
        self.scales = s
        self.orig_shape = tuple(data.shape)
        self.orig_dtype = data.dtype if data.dtype != torch.float32 else torch.bfloat16
        self.qc = qc
        return self

    def dequantized(self):
        from ..ops.quantizer import dequantize_fp8
        n = 1
        for x in self.orig_shape:
            n *= x
        out = dequantize_fp8(self.data, self.scales.to(self.data.device), self.qc.group_size, dtype=self.orig_dtype)
        return out[:n].view(self.orig_shape)


class LoRAOptimizedLinear(nn.Module):
    def __init__(self, input_dim, output_dim, bias=False, lora_config: LoRAConfig = None,
                 quantization_config: QuantizationConfig = None, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.input_dim, self.output_dim = input_dim, output_dim
        self.lora_config = lora_config or LoRAConfig()
        self.quantization_config = quantization_config
        self.dtype = dtype
        self.zero_shards = max(1, self.lora_config.base_weight_sharding)
        self.group = None
        if self.zero_shards > 1:
            assert dist.is_initialized() and dist.get_world_size() % self.zero_shards == 0
            self.rank_in = dist.get_rank() % self.zero_shards
        else:
            self.rank_in = 0
        assert output_dim % self.zero_shards == 0, "output_dim must divide base_weight_sharding"
        w = torch.empty(output_dim, input_dim, dtype=dtype, device=device)
        nn.init.kaiming_uniform_(w, a=5 ** 0.5)
        self._set_base(w)
        self.bias = nn.Parameter(torch.zeros(output_dim, dtype=dtype, device=device), requires_grad=False) if bias else None
        r = self.lora_config.lora_r
        self.lora_scaling = self.lora_config.lora_alpha / r
        self.lora_weight_1 = nn.Parameter(torch.empty(r, input_dim, dtype=dtype, device=device))  # A
        self.lora_weight_2 = nn.Parameter(torch.zeros(output_dim, r, dtype=dtype, device=device))  # B
        nn.init.kaiming_uniform_(self.lora_weight_1, a=5 ** 0.5)

    def _set_base(self, w):
        rows = w.shape[0] // self.zero_shards
        local = w[self.rank_in * rows:(self.rank_in + 1) * rows].contiguous()
        if self.quantization_config is not None:
            self.base_weight = QuantizedParameter(local, self.quantization_config)
        else:
            self.base_weight = nn.Parameter(local, requires_grad=False)

    def init_lora(self):
        nn.init.kaiming_uniform_(self.lora_weight_1, a=5 ** 0.5)
        nn.init.zeros_(self.lora_weight_2)

    def load_base_weight(self, full_weight):
        """Replace the frozen base weight from a full [out, in] tensor (e.g. a pretrained checkpoint)."""
        self._set_base(full_weight.to(self.lora_weight_1.device, self.dtype))

    def full_weight(self):
        w = self.base_weight.dequantized() if isinstance(self.base_weight, QuantizedParameter) else self.base_weight
        if self.zero_shards > 1:
            parts = torch.empty(self.zero_shards * w.shape[0], w.shape[1], dtype=w.dtype, device=w.device)
            g = _shard_group(self.zero_shards)
            dist.all_gather_into_tensor(parts, w.contiguous(), group=g)
            w = parts
        return w

    @torch.no_grad()
    def fuse_lora(self):
        """Inference (hybrid-engine generation): one GEMM with W + scaling * B A instead of the base
        GEMM plus the two rank-r GEMMs. The fused weight is a separate tensor (the frozen base stays
        bit-exact for training; reference hybrid_engine.py:132 ``_fuse_lora_layer``)."""
        w = self.full_weight().detach().float().clone()
        w.add_(self.lora_weight_2.float() @ self.lora_weight_1.float(), alpha=self.lora_scaling)
        self._fused = w.to(self.dtype)

    def unfuse_lora(self):
        self._fused = None

    def forward(self, x):
        fused = self.__dict__.get("_fused")
        if fused is not None:
            return F.linear(x, fused.to(x.dtype), self.bias)
        w = self.full_weight().detach()
        y = F.linear(x, w.to(x.dtype), self.bias)
        lora = linear(linear(x, self.lora_weight_1), self.lora_weight_2)
        return y + self.lora_scaling * lora


_SHARD_GROUPS = {}


def _shard_group(n):
    if n not in _SHARD_GROUPS:
        me, W = dist.get_rank(), dist.get_world_size()
        mine = None
        for s in range(0, W, n):
            ranks = list(range(s, s + n))
            g = dist.new_group(ranks)
            if me in ranks:
                mine = g
        _SHARD_GROUPS[n] = mine
    return _SHARD_GROUPS[n]


def OptimizedLinear(input_dim, output_dim, bias=False, lora_config=None, quantization_config=None, device=None,
                    dtype=torch.bfloat16):
    """Factory (reference signature): plain Linear, LoRA linear, and/or FP8-quantized frozen base."""
    if lora_config is None and quantization_config is None:
        return nn.Linear(input_dim, output_dim, bias=bias, dtype=dtype, device=device)
    if lora_config is None:
        lora_config = LoRAConfig(lora_r=1, lora_alpha=0.0)
    return LoRAOptimizedLinear(input_dim, output_dim, bias, lora_config, quantization_config, device, dtype)
