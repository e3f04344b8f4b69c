"""Kernel-injection policies for Megatron-LM GPT (dense and MoE) and InternLM, checked against mirror
modules with the same attribute structure and forward semantics (the libraries are not installed
here: reference module_inject/containers/megatron_gpt.py, megatron_gpt_moe.py, internlm.py; parity
with the real modules is unpinned beyond these mirrors)."""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from shuffle_exchange_amd.module_inject.replace_module import (FusedInternLMLayer, FusedMegatronLayer,
                                                               replace_transformer_layer)

H, NH, S, B = 64, 4, 12, 2
HD = H // NH


class _MegAttn(nn.Module):
    def __init__(self):
        super().__init__()
        self.query_key_value = nn.Linear(H, 3 * H)
        self.dense = nn.Linear(H, H)
        self.num_attention_heads = NH


class _MegMLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.dense_h_to_4h = nn.Linear(H, 4 * H)
        self.dense_4h_to_h = nn.Linear(4 * H, H)

    def forward(self, x):
        return self.dense_4h_to_h(F.gelu(self.dense_h_to_4h(x)))


class _MoEMLP(nn.Module):
    """A DeepSpeed-MoE-shaped mlp: returns (out, l_aux, exp_counts)."""

    def __init__(self):
        super().__init__()
        self.e = nn.Linear(H, H)

    def forward(self, x):
        return torch.tanh(self.e(x)), torch.zeros(()), torch.zeros(2)


class ParallelTransformerLayer(nn.Module):  # Megatron-LM v2 mirror ([S, B, H], per-head QKV layout)
    def __init__(self, moe=False, post_ln_residual=False):
        super().__init__()
        self.input_layernorm = nn.LayerNorm(H)
        self.self_attention = _MegAttn()
        self.post_attention_layernorm = nn.LayerNorm(H)
        self.mlp = _MoEMLP() if moe else _MegMLP()
        self.apply_residual_connection_post_layernorm = post_ln_residual

    def forward(self, hidden_states, attention_mask=None, encoder_output=None, enc_dec_attn_mask=None,
                layer_past=None, get_key_value=False):
        ln1 = self.input_layernorm(hidden_states)
        mixed = self.self_attention.query_key_value(ln1).view(S, B, NH, 3 * HD)
        q, k, v = torch.split(mixed, HD, dim=-1)  # [S, B, nh, hd] each
        q, k, v = (t.permute(1, 2, 0, 3) for t in (q, k, v))
        sc = q @ k.transpose(-1, -2) / math.sqrt(HD)
        sc = sc.masked_fill(attention_mask, float("-inf"))
        ctx = (sc.softmax(-1) @ v).permute(2, 0, 1, 3).reshape(S, B, H)
        a = self.self_attention.dense(ctx)
        res = ln1 if self.apply_residual_connection_post_layernorm else hidden_states
        h = res + a
        ln2 = self.post_attention_layernorm(h)
        m = self.mlp(ln2)
        m = m[0] if isinstance(m, tuple) else m
        return (ln2 if self.apply_residual_connection_post_layernorm else h) + m


def _causal_bool():
    return torch.ones(S, S, dtype=torch.bool).triu(1).view(1, 1, S, S)


def test_megatron_gpt_policy_dense_moe_and_post_ln():
    torch.manual_seed(0)
    for moe, post in [(False, False), (True, False), (False, True)]:
        m = nn.Sequential(ParallelTransformerLayer(moe, post))
        x = torch.randn(S, B, H)
        ref = m[0](x, _causal_bool())
        assert replace_transformer_layer(m) == 1 and isinstance(m[0], FusedMegatronLayer)
        out = m[0](x, _causal_bool())
        torch.testing.assert_close(out, ref, atol=2e-5, rtol=1e-4)
        # a non-causal mask is delegated to the original layer
        mask = torch.zeros(1, 1, S, S, dtype=torch.bool)
        torch.testing.assert_close(m[0](x, mask), m[0].orig(x, mask))


class _Rotary(nn.Module):  # old-HF style: cos/sin [1, 1, seq, dim]
    def __init__(self, dim, base=10000):
        super().__init__()
        self.inv = 1.0 / (base ** (torch.arange(0, dim, 2).float() / dim))

    def forward(self, x, seq_len=None):
        t = torch.arange(seq_len).float()
        f = torch.outer(t, self.inv)
        emb = torch.cat([f, f], -1)
        return emb.cos()[None, None].to(x.dtype), emb.sin()[None, None].to(x.dtype)


class _RMS(nn.Module):
    def __init__(self):
        super().__init__()
        self.weight = nn.Parameter(torch.rand(H) + 0.5)
        self.variance_epsilon = 1e-6

    def forward(self, x):
        return self.weight * x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + self.variance_epsilon)


class _ILMAttn(nn.Module):
    def __init__(self):
        super().__init__()
        self.q_proj, self.k_proj, self.v_proj, self.o_proj = (nn.Linear(H, H, bias=True) for _ in range(4))
        self.num_heads = NH
        self.rotary_emb = _Rotary(HD)


class _ILMMLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.gate_proj, self.up_proj = nn.Linear(H, 96, bias=False), nn.Linear(H, 96, bias=False)
        self.down_proj = nn.Linear(96, H, bias=False)


def _rot(x):
    d = x.shape[-1] // 2
    return torch.cat([-x[..., d:], x[..., :d]], -1)


class InternLMDecoderLayer(nn.Module):  # InternLM v1 mirror
    def __init__(self):
        super().__init__()
        self.self_attn, self.mlp = _ILMAttn(), _ILMMLP()
        self.input_layernorm, self.post_attention_layernorm = _RMS(), _RMS()

    def forward(self, hidden_states, attention_mask=None, position_ids=None, past_key_value=None,
                output_attentions=False, use_cache=False):
        x = hidden_states
        Bq, Sq, _ = x.shape
        a = self.self_attn
        h = self.input_layernorm(x)
        q, k, v = (p(h).view(Bq, Sq, NH, HD).transpose(1, 2) for p in (a.q_proj, a.k_proj, a.v_proj))
        past = past_key_value[0].shape[-2] if past_key_value is not None else 0
        cos, sin = a.rotary_emb(v, seq_len=past + Sq)
        cos, sin = cos[0, 0][position_ids].unsqueeze(1), sin[0, 0][position_ids].unsqueeze(1)
        q, k = q * cos + _rot(q) * sin, k * cos + _rot(k) * sin
        if past_key_value is not None:
            k, v = torch.cat([past_key_value[0], k], 2), torch.cat([past_key_value[1], v], 2)
        sc = q @ k.transpose(-1, -2) / math.sqrt(HD) + attention_mask
        o = (sc.softmax(-1) @ v).transpose(1, 2).reshape(Bq, Sq, H)
        x = x + a.o_proj(o)
        m = self.mlp
        y = self.post_attention_layernorm(x)
        x = x + m.down_proj(F.silu(m.gate_proj(y)) * m.up_proj(y))
        return (x,) + (((k, v),) if use_cache else ())


def _additive(Sq, Sk, pad=0):
    m = torch.full((B, 1, Sq, Sk), float("-inf")).triu(Sk - Sq + 1)
    m = torch.where(torch.isinf(m), m, torch.zeros(()))
    if pad:
        m[0, :, :, :pad] = float("-inf")
    return m


def test_internlm_policy_prefill_padding_and_decode():
    torch.manual_seed(1)
    mdl = nn.Sequential(InternLMDecoderLayer())
    x = torch.randn(B, S, H)
    pos = torch.arange(S).expand(B, S)
    ref, ref_kv = mdl[0](x, _additive(S, S), pos, use_cache=True)
    ref_pad = mdl[0](x, _additive(S, S, pad=3), pos)[0]
    assert replace_transformer_layer(mdl) == 1 and isinstance(mdl[0], FusedInternLMLayer)
    out, kv = mdl[0](x, _additive(S, S), pos, use_cache=True)
    torch.testing.assert_close(out, ref, atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(kv[0], ref_kv[0], atol=2e-5, rtol=1e-4)
    got_pad = mdl[0](x, _additive(S, S, pad=3), pos)[0]
    torch.testing.assert_close(got_pad[1:], ref_pad[1:], atol=2e-5, rtol=1e-4)
    # padded sequence: the masked-key path (queries that see at least one key)
    torch.testing.assert_close(got_pad[0, 3:], ref_pad[0, 3:], atol=2e-5, rtol=1e-4)
    # one decode step on the cache
    x1 = torch.randn(B, 1, H)
    p1 = torch.full((B, 1), S)
    want = mdl[0].orig(x1, _additive(1, S + 1), p1, past_key_value=ref_kv)[0]
    got = mdl[0](x1, _additive(1, S + 1), p1, past_key_value=kv)[0]
    torch.testing.assert_close(got, want, atol=2e-5, rtol=1e-4)
