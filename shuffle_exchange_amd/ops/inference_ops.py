"""Functional inference-v1 ops (reference ops/transformer/inference/op_binding/*.py, whose
``InferenceBuilder`` native module is not in the snapshot -- SURVEY 2.5).

The reference wraps each CUDA entry point in an ``*Op`` class configured by
``DeepSpeedInferenceConfig``; here every op is a plain function on this framework's gfx950 kernels
(norms with fused residual: norm.hip; bias + activation, gated activations: act.hip; GEMMs:
hipBLASLt / the MFMA skinny GEMM through ``ops.linear``; attention: flash / paged kernels), with the
configuration passed as arguments. Semantics follow the reference's kernels:

  layer_norm / rms_norm / pre_rms_norm(x, residual) -> (y, x + residual)
  bias_add, bias_gelu, bias_relu, bias_residual(out, residual, bias) = out + residual + bias
  vector_add(a, b, gamma) = a + gamma * b
  gated_activation(x, bias, act): x + bias split in halves [gate | up] -> act(gate) * up
  qkv_gemm(x, W, b, gamma, beta) -> (norm(x) @ W (+ b), norm(x))   (W stored [in, out] like the
                                      reference's transposed_mode=False, or [out, in] if transposed)
  mlp_gemm(x, residual, W1, W2, ...) -> (act(norm(x + residual + input_bias) @ W1 + b1) @ W2, new residual)
  vector_matmul(x, W) -> x @ W;   linear(x, W, b) -> x @ W + b
  softmax(scores, mask, triangular, ...) -> softmax over the last dim with additive / causal masks
  softmax_context(qkv, ...) -> attention of the new tokens over a per-layer KV workspace
  moe_res_matmul(residual, coef, out) = residual * coef[..., 0] + out * coef[..., 1]
  einsum_sec_sm_ecm(Q, W) = einsum('sec,sm->ecm')
  pad_transform(q, k, v, heads) -> [B, H, S, D] views (head dim padded to a multiple of 32)
  Workspace: allocate_workspace / reset_cache / release_workspace bookkeeping for softmax_context.
"""
import math

import torch
import torch.nn.functional as F

from . import native
from .activation import ACT, bias_act, gated_act
from .linear import linear as _linear
from .norm import layer_norm as _layer_norm
from .norm import rms_norm as _rms_norm

ActivationFuncType = {"UNKNOWN": 0, "GELU": 1, "ReLU": 2, "GATED_GELU": 3, "GATED_SILU": 4}


def layer_norm(x, gamma, beta, epsilon):
    return _layer_norm(x, gamma.to(x.dtype), beta.to(x.dtype) if beta is not None else None, epsilon)


def rms_norm(x, gamma, epsilon):
    return _rms_norm(x, gamma.to(x.dtype), epsilon)


def pre_rms_norm(x, residual, gamma, epsilon):
    """Returns (rms_norm(x + residual), x + residual)."""
    return _rms_norm(x, gamma.to(x.dtype), epsilon, residual=residual)


def bias_add(x, bias):
    return bias_act(x, bias.to(x.dtype), ACT["identity"])


def bias_gelu(x, bias):
    return bias_act(x, bias.to(x.dtype), ACT["gelu"])


def bias_relu(x, bias):
    return bias_act(x, bias.to(x.dtype), ACT["relu"])


def bias_residual(output, residual, bias):
    return bias_add(output, bias) + residual


def vector_add(a, b, gamma):
    return a + gamma * b


def gated_activation(activation, bias, activation_func_type):
    """act(x_gate + b_gate) * (x_up + b_up) with [gate | up] halves of the last dim."""
    x = activation + bias.to(activation.dtype) if bias is not None else activation
    kind = activation_func_type if isinstance(activation_func_type, str) else \
        {3: "GATED_GELU", 4: "GATED_SILU"}.get(int(activation_func_type), "GATED_SILU")
    return gated_act(x.contiguous(), "gelu" if "GELU" in str(kind).upper() else "silu")


def _mm(x, w, b=None, transposed_mode=False):
    """x @ W with W stored [in, out] (reference default) or [out, in] (transposed_mode)."""
    wt = w if transposed_mode else w.t()
    return _linear(x, wt.contiguous() if not wt.is_contiguous() else wt, b)


def vector_matmul(input, weight, async_op=False, transposed_mode=False):
    return _mm(input, weight, None, transposed_mode)


def linear(input, weight, bias=None, transposed_mode=False):
    return _mm(input, weight, bias, transposed_mode)


def qkv_gemm(input, weight, bias, gamma, beta, epsilon=1e-5, norm_type="layernorm", transposed_mode=False):
    norm = layer_norm(input, gamma, beta, epsilon) if norm_type == "layernorm" else rms_norm(input, gamma, epsilon)
    return _mm(norm, weight, bias, transposed_mode), norm


def mlp_gemm(input, residual, weight_interm, weight_out, input_bias=None, bias=None, gamma=None, beta=None,
             epsilon=1e-5, pre_layer_norm=True, mlp_after_attn=True, act="gelu", norm_type="layernorm",
             transposed_mode=False):
    """Reference semantics (pre-LN, mlp_after_attn): residual_add = input + residual (+ input_bias);
    out = act(norm(residual_add) @ W1 + b1) @ W2. Returns (out, residual_add)."""
    h = input + residual if mlp_after_attn else input
    if input_bias is not None:
        h = h + input_bias.to(h.dtype)
    if norm_type == "layernorm":
        n = layer_norm(h, gamma, beta, epsilon) if pre_layer_norm else h
    else:
        n = rms_norm(h, gamma, epsilon)
    inter = _mm(n, weight_interm, None, transposed_mode)
    if act in ("gated_silu", "gated_gelu"):
        inter = gated_activation(inter, bias, act.upper())
    else:
        inter = bias_act(inter, bias.to(inter.dtype) if bias is not None else None, ACT[act])
    return _mm(inter, weight_out, None, transposed_mode), h


def softmax(attn_scores, attn_mask=None, alibi=None, triangular=False, recompute=False, local_attention=False,
            window_size=1, async_op=False, layer_scale=1.0, head_offset=0, mp_size=1):
    """scores [B, H, q, k] (already scaled) -> probabilities; additive/boolean mask, alibi bias,
    causal (triangular) and local-window masking. GPU: one HIP kernel (csrc/kernels/softmax.hip)
    reading broadcast masks / ALiBi in place."""
    if (attn_scores.is_cuda and attn_scores.dim() == 4 and native.use_hip(attn_scores)
            and attn_scores.dtype in (torch.float32, torch.bfloat16, torch.float16)):
        m = attn_mask
        if m is not None:
            m = m if m.dtype == torch.bool else m.float()
            while m.dim() < 4:
                m = m.unsqueeze(0)
        a = alibi.float() if alibi is not None else None
        while a is not None and a.dim() < 4:
            a = a.unsqueeze(0)
        return torch.ops.sxe.masked_softmax(attn_scores.contiguous(), float(layer_scale), m, a, bool(triangular),
                                            int(window_size) if local_attention else 0)
    s = attn_scores.float() * layer_scale
    if alibi is not None:
        s = s + alibi.float()
    q, k = s.shape[-2], s.shape[-1]
    if triangular or local_attention:
        qpos = torch.arange(k - q, k, device=s.device)[:, None]
        kpos = torch.arange(k, device=s.device)[None, :]
        bad = kpos > qpos if triangular else torch.zeros(q, k, dtype=torch.bool, device=s.device)
        if local_attention:
            bad = bad | (kpos <= qpos - window_size)
        s = s.masked_fill(bad, float("-inf"))
    if attn_mask is not None:
        s = s.masked_fill(~attn_mask, float("-inf")) if attn_mask.dtype == torch.bool else s + attn_mask.float()
    return torch.softmax(s, dim=-1).to(attn_scores.dtype)


class Workspace:
    """Per-layer KV cache of the v1 incremental decoding path (reference ``allocate_workspace_*``
    / ``reset_cache`` / ``release_workspace``)."""

    def __init__(self):
        self.kv = {}

    def allocate_workspace(self, *args, **kwargs):
        self.kv.clear()

    def reset_cache(self):
        self.kv.clear()

    def release_workspace(self):
        self.kv.clear()

    def append(self, layer_id, k, v):
        if layer_id in self.kv:
            pk, pv = self.kv[layer_id]
            k, v = torch.cat([pk, k], dim=1), torch.cat([pv, v], dim=1)
        self.kv[layer_id] = (k, v)
        return k, v


_WORKSPACE = Workspace()


def softmax_context(query_key_value, attn_mask, heads, num_kv, norm_factor, layer_id, rotary_dim=0,
                    rotate_half=True, triangular_masking=True, rope_theta=10000.0, workspace=None):
    """qkv [B, q, (heads + 2 num_kv) * D] of the NEW tokens -> context [B, q, heads * D]; appends
    K/V to the layer's workspace cache and attends over everything cached (GQA, causal, optional
    rotary on the first ``rotary_dim`` dims, rotate-half convention)."""
    ws = workspace or _WORKSPACE
    B, q, _ = query_key_value.shape
    D = query_key_value.shape[-1] // (heads + 2 * num_kv)
    x = query_key_value.view(B, q, heads + 2 * num_kv, D)
    qh, kh, vh = x[:, :, :heads], x[:, :, heads:heads + num_kv], x[:, :, heads + num_kv:]
    past = ws.kv[layer_id][0].shape[1] if layer_id in ws.kv else 0
    if rotary_dim:
        pos = torch.arange(past, past + q, device=x.device, dtype=torch.float32)
        inv = 1.0 / (rope_theta ** (torch.arange(0, rotary_dim, 2, device=x.device, dtype=torch.float32) / rotary_dim))
        f = pos[:, None] * inv[None, :]
        cos, sin = f.cos()[None, :, None, :], f.sin()[None, :, None, :]

        def rot(t):
            r = t[..., :rotary_dim].float()
            if rotate_half:
                a, b = r[..., :rotary_dim // 2], r[..., rotary_dim // 2:]
                out = torch.cat([a * cos - b * sin, b * cos + a * sin], dim=-1)
            else:
                a, b = r[..., 0::2], r[..., 1::2]
                out = torch.stack([a * cos - b * sin, b * cos + a * sin], dim=-1).flatten(-2)
            return torch.cat([out.to(t.dtype), t[..., rotary_dim:]], dim=-1)
        qh, kh = rot(qh), rot(kh)
    k, v = ws.append(layer_id, kh.contiguous(), vh.contiguous())
    G = heads // num_kv
    kk = k.repeat_interleave(G, dim=2).transpose(1, 2)
    vv = v.repeat_interleave(G, dim=2).transpose(1, 2)
    scores = torch.matmul(qh.transpose(1, 2).float(), kk.float().transpose(-1, -2)) / norm_factor
    probs = softmax(scores, attn_mask, triangular=triangular_masking)
    ctx = torch.matmul(probs.float(), vv.float()).to(query_key_value.dtype)
    return ctx.transpose(1, 2).reshape(B, q, heads * D), k, v


def moe_res_matmul(residual, coef, output):
    return residual * coef[..., 0:1] + output * coef[..., 1:2]


def einsum_sec_sm_ecm(Q, W):
    return torch.einsum("sec,sm->ecm", Q.to(W.dtype), W)


def pad_transform(query, key, value, heads, do_flash_attn=False):
    """[B, S, H*D] x3 -> [B, H, S, Dp] x3 with D padded to a multiple of 32 (zeros)."""
    B, S, HD = query.shape
    D = HD // heads
    Dp = int(math.ceil(D / 32) * 32)

    def t(x):
        x = x.view(B, x.shape[1], heads, D).transpose(1, 2)
        return F.pad(x, (0, Dp - D)) if Dp != D else x
    return t(query), t(key), t(value)
