"""Generic (diffusers-style) injection: fused attention for UNet / VAE / transformer-block attention.

Parity: reference module_inject/replace_module.py ``generic_injection`` (:88) with the
containers/unet.py ``UNetPolicy`` and containers/vae.py ``VAEPolicy``: every diffusers attention
module (``Attention`` / legacy ``CrossAttention``: ``to_q``, ``to_k``, ``to_v``, ``to_out[0]``,
``heads``) is replaced by a fused attention module -- ONE packed [q | k | v] projection GEMM for
self-attention, q plus ONE packed [k | v] GEMM over the encoder states for cross-attention --
and UNet / VAE models get whole-forward HIP-graph replay (the reference's ``DSUNet`` / ``DSVAE``
CUDA-graph wrappers), here through the v1 engine's graph capture (``InferenceEngine``
``enable_cuda_graph``).

MI355X-first: attention runs the gfx950 flash kernel (``ops.attention``; non-causal, head dims up
to 128 on padded copies -- SD UNet heads are 40/64/80/160 wide, head dims above 128 such as the
single 512-wide VAE head run SDPA), the optional GroupNorm runs before the projections exactly as
diffusers' ``AttnProcessor2_0`` does, and the residual / ``rescale_output_factor`` epilogue is
applied in place. Anything the fused path does not cover (attention masks, spatial norm, cross
norm, added KV projections, a non-default processor) is delegated to the original module.
diffusers itself is not installed here: tests drive the policy with a module that mirrors
diffusers' ``Attention`` + ``AttnProcessor2_0`` semantics (parity unpinned against diffusers).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.linear import linear
from .replace_module import _Fused, _attend

ATTENTION_CLASSES = ("Attention", "CrossAttention")


def _is_diffusers_attention(m):
    return (type(m).__name__ in ATTENTION_CLASSES and all(hasattr(m, a) for a in ("to_q", "to_k", "to_v", "to_out"))
            and hasattr(m, "heads") and isinstance(m.to_q, nn.Linear))


class FusedDiffusersAttention(_Fused):
    """Fused replacement of one diffusers attention module (see the module docstring)."""

    def __init__(self, attn):
        super().__init__(attn)
        self.heads = int(attn.heads)
        self.inner = attn.to_q.weight.shape[0]
        self.hd = self.inner // self.heads
        self.scale = float(getattr(attn, "scale", self.hd ** -0.5))
        self.cross_dim = attn.to_k.weight.shape[1]
        self.self_only = self.cross_dim == attn.to_q.weight.shape[1]
        qb = attn.to_q.bias
        has_b = qb is not None
        if self.self_only:  # one packed [q | k | v] weight; q / [k | v] row slices serve cross calls
            self.w_qkv = self._p(torch.cat([attn.to_q.weight, attn.to_k.weight, attn.to_v.weight]))
            self.b_qkv = self._p(torch.cat([qb, attn.to_k.bias, attn.to_v.bias])) if has_b else None
        else:  # cross-attention: q over the latents, ONE packed [k | v] GEMM over the encoder states
            self.w_q = self._p(attn.to_q.weight)
            self.b_q = self._p(qb) if has_b else None
            self.w_kv = self._p(torch.cat([attn.to_k.weight, attn.to_v.weight]))
            self.b_kv = self._p(torch.cat([attn.to_k.bias, attn.to_v.bias])) if has_b else None
        out = attn.to_out[0]
        self.w_o = self._p(out.weight)
        self.b_o = self._p(out.bias) if out.bias is not None else None
        self.residual = bool(getattr(attn, "residual_connection", False))
        self.rescale = float(getattr(attn, "rescale_output_factor", 1.0))
        self._link()

    def _links(self):
        a, n = self.orig, self.inner
        out = [(a.to_out[0].weight, self.w_o)]
        if self.b_o is not None:
            out.append((a.to_out[0].bias, self.b_o))
        if self.self_only:
            ws, bs = [self.w_qkv[i * n:(i + 1) * n] for i in range(3)], None
            if self.b_qkv is not None:
                bs = [self.b_qkv[i * n:(i + 1) * n] for i in range(3)]
        else:
            ws = [self.w_q, self.w_kv[:n], self.w_kv[n:]]
            bs = None if self.b_q is None else [self.b_q, self.b_kv[:n], self.b_kv[n:]]
        for i, lin in enumerate((a.to_q, a.to_k, a.to_v)):
            out.append((lin.weight, ws[i]))
            if bs is not None:
                out.append((lin.bias, bs[i]))
        return out

    def _q_kv(self):
        """(w_q, b_q, w_kv, b_kv) for a call with separate query / context inputs."""
        if not self.self_only:
            return self.w_q, self.b_q, self.w_kv, self.b_kv
        n, b = self.inner, self.b_qkv
        return self.w_qkv[:n], None if b is None else b[:n], self.w_qkv[n:], None if b is None else b[n:]

    def _covered(self, attention_mask, kwargs):
        a = self.orig
        proc = getattr(a, "processor", None)
        default_proc = proc is None or type(proc).__name__ in ("AttnProcessor2_0", "AttnProcessor")
        return (attention_mask is None and not kwargs and default_proc and getattr(a, "spatial_norm", None) is None
                and getattr(a, "norm_cross", None) is None and getattr(a, "add_k_proj", None) is None
                and getattr(a, "norm_q", None) is None and getattr(a, "norm_k", None) is None)

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None, **kwargs):
        if not self._covered(attention_mask, kwargs):
            return self._delegate(hidden_states, encoder_hidden_states=encoder_hidden_states,
                                  attention_mask=attention_mask, **kwargs)
        a = self.orig
        x = hidden_states
        residual = x
        nd = x.dim()
        if nd == 4:  # [B, C, H, W] (VAE mid-block attention) -> [B, HW, C]
            B, C, Hh, Ww = x.shape
            x = x.view(B, C, Hh * Ww).transpose(1, 2)
        if getattr(a, "group_norm", None) is not None:
            x = a.group_norm(x.transpose(1, 2)).transpose(1, 2)
        B, S, _ = x.shape
        if encoder_hidden_states is None and self.self_only:
            qkv = linear(x, self.w_qkv, self.b_qkv).view(B, S, 3, self.heads, self.hd)
            q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        else:
            ctx = x if encoder_hidden_states is None else encoder_hidden_states
            w_q, b_q, w_kv, b_kv = self._q_kv()
            q = linear(x, w_q, b_q).view(B, S, self.heads, self.hd)
            kv = linear(ctx, w_kv, b_kv).view(B, ctx.shape[1], 2, self.heads, self.hd)
            k, v = kv[:, :, 0], kv[:, :, 1]
        if q.shape[1] == k.shape[1]:
            o = _attend(q, k, v, None, False, self.scale)
        else:  # cross-attention with another sequence length: SDPA on [B, H, S, D]
            o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                               scale=self.scale).transpose(1, 2)
        y = linear(o.reshape(B, S, self.inner), self.w_o, self.b_o)
        if nd == 4:
            y = y.transpose(1, 2).reshape(B, C, Hh, Ww)
        if self.residual:
            y = y + residual
        if self.rescale != 1.0:
            y = y / self.rescale
        return y


def generic_injection(module, dtype=None, enable_cuda_graph=False):
    """Replace every diffusers-style attention module under ``module`` by the fused module; returns
    the number replaced. ``dtype`` casts the model first (the reference requires fp16; bf16 and
    fp16 both run the gfx950 kernels here). ``enable_cuda_graph`` is honoured by the inference
    engine's HIP-graph capture of the whole forward (``sxe.init_inference(..., enable_cuda_graph=
    True)``), not here."""
    if dtype is not None:
        module.to(dtype)
    n = 0
    for parent in list(module.modules()):
        for name, child in list(parent.named_children()):
            if isinstance(child, FusedDiffusersAttention):
                continue
            if _is_diffusers_attention(child):
                setattr(parent, name, FusedDiffusersAttention(child))
                n += 1
    return n
