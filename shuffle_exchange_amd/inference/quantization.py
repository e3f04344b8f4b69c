"""Post-training group-wise weight quantization for inference (int8 / int4).

Parity: reference inference/quantization/quantization.py:20 ``_init_group_wise_weight_quantization``
(config ``weight_quantization.post_init_quant`` = {module-name substring: {num_bits, group_size,
group_dim, symmetric}}), layers.py:47 ``QuantizedLinear`` / :75 ``QuantizedEmbedding``,
utils.py:43 ``Quantizer`` / :96 ``DeQuantizer`` (asymmetric min/scale, int4 packed two per byte).

MI355X path: symmetric groups use the gfx950 quantize/dequantize kernels (ops/quantizer.py,
quant.hip: 16-byte vector loads, one group per lane-group); the weight is dequantized into a
bf16 scratch just before its GEMM, so HBM holds 1 (int8) or 0.5 (int4) bytes per weight and the
GEMM stays a full-rate hipBLASLt bf16 call. Asymmetric groups (the reference's only mode) use the
same storage with a per-group minimum, dequantized by fused PyTorch elementwise ops.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.quantizer import dequantize, quantize


class _QuantizedWeight:
    def __init__(self, w, num_bits=8, group_size=64, group_dim=1, symmetric=False):
        assert num_bits in (4, 8), "int4 / int8 only"
        self.shape, self.dtype = tuple(w.shape), w.dtype
        self.bits, self.group, self.dim, self.sym = num_bits, int(group_size), int(group_dim), bool(symmetric)
        x = w.detach().movedim(self.dim, -1).contiguous()  # groups along the last dim
        self.moved_shape = tuple(x.shape)
        assert x.shape[-1] % self.group == 0, f"dim {self.dim} ({x.shape[-1]}) not divisible by group {self.group}"
        if self.sym:
            self.q, self.scale = quantize(x, self.group, self.bits)
            self.min = None
        else:
            g = x.float().reshape(-1, self.group)
            mn, mx = g.amin(1, keepdim=True), g.amax(1, keepdim=True)
            levels = 2 ** self.bits - 1
            scale = ((mx - mn) / levels).clamp_min(1e-8)
            q = torch.clamp(torch.round((g - mn) / scale), 0, levels).to(torch.uint8).reshape(-1)
            if self.bits == 4:
                q = (q[0::2] | (q[1::2] << 4)).contiguous()
            self.q, self.scale, self.min = q, scale.reshape(-1), mn.reshape(-1)

    def nbytes(self):
        return self.q.numel() * self.q.element_size() + self.scale.numel() * 4 + (self.min.numel() * 4 if self.min
                                                                                   is not None else 0)

    def dequantize(self):
        n = 1
        for s in self.moved_shape:
            n *= s
        if self.sym:
            flat = dequantize(self.q, self.scale, self.group, self.bits, numel=n, dtype=self.dtype)
        else:
            q = self.q
            if self.bits == 4:
                q = torch.stack([q & 0xF, q >> 4], 1).reshape(-1)
            flat = (q.float().reshape(-1, self.group) * self.scale[:, None] + self.min[:, None]).to(self.dtype)
        return flat.reshape(self.moved_shape).movedim(-1, self.dim)

    def to(self, device):
        self.q, self.scale = self.q.to(device), self.scale.to(device)
        if self.min is not None:
            self.min = self.min.to(device)
        return self


class QuantizedLinear(nn.Module):
    def __init__(self, config, pre_quant_layer: nn.Linear):
        super().__init__()
        self.in_features, self.out_features = pre_quant_layer.in_features, pre_quant_layer.out_features
        self.qweight = _QuantizedWeight(pre_quant_layer.weight, **config)
        self.bias = pre_quant_layer.bias

    @property
    def weight(self):
        return self.qweight.dequantize()

    def forward(self, x):
        return F.linear(x, self.qweight.dequantize().to(x.dtype), self.bias)

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        probe = fn(torch.empty(0, device=self.qweight.q.device))
        self.qweight.to(probe.device)
        return self


class QuantizedEmbedding(nn.Module):
    def __init__(self, config, pre_quant_layer: nn.Embedding):
        super().__init__()
        self.num_embeddings, self.embedding_dim = pre_quant_layer.num_embeddings, pre_quant_layer.embedding_dim
        self.padding_idx = pre_quant_layer.padding_idx
        self.qweight = _QuantizedWeight(pre_quant_layer.weight, **config)

    @property
    def weight(self):
        return self.qweight.dequantize()

    def forward(self, ids):
        return F.embedding(ids, self.qweight.dequantize(), self.padding_idx)

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        probe = fn(torch.empty(0, device=self.qweight.q.device))
        self.qweight.to(probe.device)
        return self


_LAYERS = {nn.Linear: QuantizedLinear, nn.Embedding: QuantizedEmbedding}


def _init_group_wise_weight_quantization(model, ds_config):
    """Replace every Linear / Embedding whose qualified name contains a configured key."""
    cfg = ds_config["weight_quantization"]["post_init_quant"]
    replaced = 0
    for name, mod in list(model.named_modules()):
        cls = None
        for base, q in _LAYERS.items():
            if isinstance(mod, base):
                cls = q
        if cls is None:
            continue
        key = next((k for k in cfg if k in name), None)
        if key is None:
            continue
        c = dict(cfg[key])
        c.setdefault("group_dim", 1 if cls is QuantizedLinear else 1)
        c.setdefault("symmetric", False)
        c.setdefault("group_size", 64)
        c.setdefault("num_bits", 8)
        parent = model.get_submodule(name.rsplit(".", 1)[0]) if "." in name else model
        setattr(parent, name.rsplit(".", 1)[-1], cls(c, mod))
        replaced += 1
    model._sxe_quantized_modules = replaced
    return model


def quantize_model(model, post_init_quant):
    """Convenience: ``quantize_model(model, {"fc": {"num_bits": 4, "group_size": 64}})``."""
    return _init_group_wise_weight_quantization(model, {"weight_quantization": {"post_init_quant": post_init_quant}})
