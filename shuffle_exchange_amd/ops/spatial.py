"""Spatial (diffusers UNet / VAE) inference ops (reference ops/transformer/inference/bias_add.py
``nhwc_bias_add`` over the SpatialInferenceBuilder kernels, not in the snapshot).

Channels-last activations are a [pixels, C] matrix, so the per-channel bias add is the bias-act
kernel of act.hip with the identity activation (16-byte vector lanes, one pass); the residual
variants add the second operand (and its bias) in the same expression."""
from typing import Optional

import torch

from .activation import bias_act


def _as_rows(t):
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1]), True
    return t.reshape(-1, t.shape[-1]), False


def _restore(rows, like, cl):
    if cl:
        n, c, h, w = like.shape
        return rows.view(n, h, w, c).permute(0, 3, 1, 2)
    return rows.view(like.shape)


def nhwc_bias_add(activation: torch.Tensor, bias: torch.Tensor, other: Optional[torch.Tensor] = None,
                  other_bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """activation + bias (+ other (+ other_bias)); bias broadcasts over the channel dimension, which
    is the last dimension in memory (NHWC, or NCHW tensors in channels_last format)."""
    rows, cl = _as_rows(activation)
    out = bias_act(rows.contiguous(), bias.to(rows.dtype), "identity")
    if other is not None:
        orow, _ = _as_rows(other)
        out = out + (orow if other_bias is None else orow + other_bias.to(orow.dtype))
    return _restore(out, activation, cl)
