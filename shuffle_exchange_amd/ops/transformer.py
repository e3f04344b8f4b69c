"""Fused BERT-style transformer layer for training (reference ops/transformer/transformer.py:
``DeepSpeedTransformerConfig`` :34, ``DeepSpeedTransformerLayer`` :296, whose CUDA kernels
``create_transformer_layer_fp{16,32}`` / ``forward_*`` / ``backward_*`` are not in the snapshot).

Same parameters (``attn_qkvw/attn_qkvb/attn_ow/attn_ob/attn_nw/attn_nb/inter_w/inter_b/output_w/
output_b/norm_w/norm_b``), same Pre-LN / Post-LN semantics and forward signature, built from this
framework's gfx950 pieces instead of one monolithic CUDA layer:

* LayerNorm with the residual add fused in (norm.hip), bias + GELU in one pass (act.hip), GEMMs on
  hipBLASLt through ``ops.linear`` (ZeRO writes weight gradients straight into its buffers);
* attention: the MFMA flash kernel (flash_attn.hip) when there is no padding mask and the head dim
  is 128; otherwise PyTorch SDPA with the additive mask (BERT heads are usually 64 wide);
* ``gelu_checkpoint`` / ``attn_dropout_checkpoint`` / ``normalize_invertible`` trade memory for
  recompute through activation checkpointing of the corresponding sub-blocks (the reference's
  flags); ``stochastic_mode`` is accepted (the kernels here are deterministic).

GELU is the exact (erf) form, matching HF ``BertLayer``; set ``config.gelu_approximate = True`` for
the tanh form the reference CUDA kernel used.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

from . import native
from .activation import ACT, bias_act
from .linear import linear
from .norm import layer_norm


class TransformerConfig:
    def __init__(self, batch_size, hidden_size, intermediate_size, heads, attn_dropout_ratio, hidden_dropout_ratio,
                 num_hidden_layers, initializer_range):
        self.layer_id = -1
        self.batch_size = batch_size
        self.hidden_size = hidden_size
        self.intermediate_size = intermediate_size
        self.heads = heads
        self.attn_dropout_ratio = attn_dropout_ratio
        self.hidden_dropout_ratio = hidden_dropout_ratio
        self.num_hidden_layers = num_hidden_layers
        self.initializer_range = initializer_range


class DeepSpeedTransformerConfig(TransformerConfig):
    def __init__(self, batch_size=-1, hidden_size=-1, intermediate_size=-1, heads=-1, attn_dropout_ratio=-1,
                 hidden_dropout_ratio=-1, num_hidden_layers=-1, initializer_range=-1, layer_norm_eps=1e-12,
                 local_rank=-1, seed=-1, fp16=False, pre_layer_norm=True, normalize_invertible=False,
                 gelu_checkpoint=False, adjust_init_range=True, attn_dropout_checkpoint=False, stochastic_mode=False,
                 return_tuple=False, training=True):
        super().__init__(batch_size, hidden_size, intermediate_size if intermediate_size > 0 else 4 * hidden_size,
                         heads, attn_dropout_ratio, hidden_dropout_ratio, num_hidden_layers, initializer_range)
        self.fp16 = fp16
        self.pre_layer_norm = pre_layer_norm
        self.local_rank = local_rank
        self.seed = seed
        self.normalize_invertible = normalize_invertible
        self.gelu_checkpoint = gelu_checkpoint
        self.adjust_init_range = adjust_init_range
        self.test_gemm = False
        self.layer_norm_eps = layer_norm_eps
        self.training = training
        self.is_grad_enabled = True
        self.attn_dropout_checkpoint = attn_dropout_checkpoint
        self.stochastic_mode = stochastic_mode
        self.return_tuple = return_tuple
        self.gelu_approximate = False

    @classmethod
    def from_dict(cls, json_object):
        config = cls()
        for k, v in json_object.items():
            config.__dict__[k] = v
        return config

    @classmethod
    def from_json_file(cls, json_file):
        import json
        with open(json_file, "r", encoding="utf-16") as f:
            return cls.from_dict(json.loads(f.read()))


class DeepSpeedTransformerLayer(nn.Module):
    layer_id = 0

    def __init__(self, config, initial_weights=None, initial_biases=None):
        super().__init__()
        self.config = config
        self.config.layer_id = DeepSpeedTransformerLayer.layer_id
        DeepSpeedTransformerLayer.layer_id += 1
        if config.local_rank >= 0 and torch.cuda.is_available():
            torch.cuda.set_device(config.local_rank)
        H, I = config.hidden_size, config.intermediate_size
        P = lambda *shape: nn.Parameter(torch.empty(*shape))  # noqa: E731
        if initial_weights is None and initial_biases is None:
            self.attn_qkvw, self.attn_qkvb = P(3 * H, H), P(3 * H)
            self.attn_ow, self.attn_ob = P(H, H), P(H)
            self.attn_nw, self.attn_nb = P(H), P(H)
            self.inter_w, self.inter_b = P(I, H), P(I)
            self.output_w, self.output_b = P(H, I), P(H)
            self.norm_w, self.norm_b = P(H), P(H)
            self.init_transformer_weights(config.adjust_init_range)
        else:  # unit-test path of the reference: [q, k, v, attn_out, attn_norm, inter, output, norm]
            w, b = initial_weights, initial_biases
            self.attn_qkvw = nn.Parameter(torch.cat([w[0].data, w[1].data, w[2].data]))
            self.attn_qkvb = nn.Parameter(torch.cat([b[0].data, b[1].data, b[2].data])
                                          if b[0] is not None else torch.zeros(3 * H))
            self.attn_ow, self.attn_ob = w[3], b[3]
            self.attn_nw, self.attn_nb = w[4], b[4]
            self.inter_w, self.inter_b = w[5], b[5]
            self.output_w, self.output_b = w[6], b[6]
            self.norm_w, self.norm_b = w[7], b[7]

    def init_transformer_weights(self, adjust_init_range=False):
        c = self.config
        out_std = c.initializer_range / math.sqrt(2.0 * c.num_hidden_layers) if adjust_init_range else \
            c.initializer_range
        for p, std in ((self.attn_qkvw, c.initializer_range), (self.attn_ow, out_std),
                       (self.inter_w, c.initializer_range), (self.output_w, out_std)):
            p.data.normal_(mean=0.0, std=std)
        for p in (self.attn_qkvb, self.attn_ob, self.attn_nb, self.inter_b, self.output_b, self.norm_b):
            p.data.zero_()
        self.attn_nw.data.fill_(1.0)
        self.norm_w.data.fill_(1.0)

    # ------------------------------------------------------------------------------- sub-blocks
    def _ln(self, x, w, b, residual=None):
        return layer_norm(x, w.to(x.dtype), b.to(x.dtype), self.config.layer_norm_eps, residual=residual)

    def _attention(self, x, mask):
        c = self.config
        B, S, H = x.shape
        nh = c.heads
        d = H // nh
        qkv = linear(x, self.attn_qkvw, self.attn_qkvb).view(B, S, 3, nh, d)
        p = c.attn_dropout_ratio if self.training and c.attn_dropout_ratio > 0 else 0.0
        if (mask is None and p == 0.0 and d == 128 and x.dtype == torch.bfloat16 and native.use_hip(x)
                and S % 128 == 0):
            from .attention import attention
            ctx = attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], causal=False)
        else:
            q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
            am = mask.to(q.dtype) if mask is not None else None
            ctx = F.scaled_dot_product_attention(q, k, v, attn_mask=am, dropout_p=p).transpose(1, 2)
        return linear(ctx.reshape(B, S, H), self.attn_ow, self.attn_ob)

    def _ffn(self, x):
        act = "gelu" if getattr(self.config, "gelu_approximate", False) else "gelu_exact"
        inter = bias_act(linear(x, self.inter_w), self.inter_b.to(x.dtype), ACT[act])
        return linear(inter, self.output_w, self.output_b)

    def _drop(self, x):
        p = self.config.hidden_dropout_ratio
        return F.dropout(x, p, self.training) if p > 0 else x

    def _maybe_ckpt(self, flag, fn, *args):
        if flag and self.training and torch.is_grad_enabled():
            return checkpoint(fn, *args, use_reentrant=False)
        return fn(*args)

    def forward(self, hidden_states, attention_mask=None, head_mask=None, layer_head_mask=None,
                encoder_hidden_states=None, encoder_attention_mask=None, past_key_value=None,
                output_attentions=False, grad_enabled=False):
        assert encoder_hidden_states is None and past_key_value is None, "self-attention encoder layer only"
        assert not output_attentions, "output_attentions is not supported by the fused layer"
        c = self.config
        x = hidden_states
        mask = attention_mask
        if mask is not None and mask.dim() == 2:  # [B, S] 1/0 padding mask -> additive [B, 1, 1, S]
            mask = (1.0 - mask[:, None, None, :].to(x.dtype)) * torch.finfo(x.dtype).min
        ckpt_attn = c.attn_dropout_checkpoint or c.normalize_invertible
        if c.pre_layer_norm:
            a = self._ln(x, self.attn_nw, self.attn_nb)
            h = x + self._drop(self._maybe_ckpt(ckpt_attn, self._attention, a, mask))
            m = self._ln(h, self.norm_w, self.norm_b)
            out = h + self._drop(self._maybe_ckpt(c.gelu_checkpoint, self._ffn, m))
        else:
            attn = self._drop(self._maybe_ckpt(ckpt_attn, self._attention, x, mask))
            h, _ = self._ln(attn, self.attn_nw, self.attn_nb, residual=x)
            ffn = self._drop(self._maybe_ckpt(c.gelu_checkpoint, self._ffn, h))
            out, _ = self._ln(ffn, self.norm_w, self.norm_b, residual=h)
        return (out,) if c.return_tuple else out
