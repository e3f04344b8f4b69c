"""v1 kernel injection: swap Hugging Face transformer layers for fused gfx950 layers in place.

Parity: reference module_inject/replace_module.py (``replace_transformer_layer`` /
``replace_with_policy``: walk the model, match each layer class against the injection policies,
build the fused inference layer from the policy's weights) and the per-architecture containers
module_inject/containers/{bert.py, gpt2.py, distil_bert.py} (``HFBertLayerPolicy``,
``HFGPT2LayerPolicy``: HF parameter names -> qkv / attn-out / mlp / norm tensors).

MI355X-first layer: the policy packs q/k/v into ONE [3H, H] weight (one hipBLASLt GEMM instead of
three), keeps every projection in the ``y = x W^T`` layout ``ops.linear`` dispatches (hipBLASLt, or
the skinny-M gfx950 kernel for decode-sized inputs), runs bias+GELU as one elementwise kernel
(``ops.activation.bias_act``) and folds every residual add into the following LayerNorm kernel
(``ops.norm.layer_norm(..., residual=)``). Attention is the HIP flash kernel where it applies
(bf16, head dim 128, no padding mask) and SDPA otherwise. Decoder blocks keep Hugging Face's
``Cache`` protocol (``past_key_values.update``), so ``model.generate`` works on injected models.
Anything a fused layer does not cover (cross-attention, head masks, attention-probability outputs)
is delegated to the original module, which the fused layer keeps without re-registering its
parameters. The original module holds no weight memory of its own: its parameters are re-pointed
at views of the fused tensors (row slices of the packed QKV, transposed views for GPT-2's
Conv1D), and re-pointed again after every ``.to()`` / ``.half()`` of the fused layer; a layout that
has no view (NeoX's head-interleaved QKV) is rebuilt only for the duration of a delegated call.
Encoder layers configured as decoders (BERT/RoBERTa ``is_decoder``: causal self-attention, a KV
cache, optional cross-attention) are not injected.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.activation import bias_act
from ..ops.attention import attention, hip_paddable, hip_supported
from ..ops.linear import linear
from ..ops.norm import layer_norm


def _act_name(hf_act):
    # Hugging Face "gelu" is the exact (erf) GELU; the framework's "gelu" is the tanh form
    return {"gelu": "gelu_exact"}.get(hf_act, hf_act) if isinstance(hf_act, str) else "gelu_exact"


def _attend(q, k, v, mask, causal, scale):
    """q [B, Sq, H, D], k/v [B, Sk, H, D] -> [B, Sq, H, D]."""
    if mask is None and q.shape[1] == k.shape[1] and (hip_supported(q, k, v) or hip_paddable(q, k, v)):
        return attention(q, k, v, causal=causal, softmax_scale=scale)
    qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    if causal and mask is None and qt.shape[2] != kt.shape[2]:
        # new tokens after a cached prefix: bottom-right aligned causal mask
        sq, sk = qt.shape[2], kt.shape[2]
        mask = torch.ones(sq, sk, dtype=torch.bool, device=q.device).tril(sk - sq)
        causal = False
    if mask is not None and mask.dtype != torch.bool:
        mask = mask.to(q.dtype)
    o = F.scaled_dot_product_attention(qt, kt, vt, attn_mask=mask, is_causal=causal and mask is None,
                                       scale=scale)
    return o.transpose(1, 2)


class _Fused(nn.Module):
    def __init__(self, orig):
        super().__init__()
        self.__dict__["orig"] = orig  # not a submodule: its parameters stay out of this layer's state

    @staticmethod
    def _p(t):
        """Fused parameter from an HF tensor: shares its storage when already contiguous."""
        t = t.detach()
        return nn.Parameter(t if t.is_contiguous() else t.contiguous(), requires_grad=False)

    def _links(self):
        """(orig parameter, view of a fused tensor) pairs; see the module docstring."""
        return []

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        for q in self.__dict__.get("_qweights", {}).values():  # int8 / int4 weights (quantize_fused_layer)
            q.to(fn(torch.empty(0, device=q.q.device)).device)
        self._link()
        return out

    def _delegate(self, *args, **kwargs):
        if self.__dict__.get("_unlinked"):
            raise NotImplementedError(f"{type(self).__name__}: this call needs the original Hugging Face layer, which "
                                      f"was released when the fused layer was tensor-parallel sharded or quantized")
        return self.orig(*args, **kwargs)

    # ---------------------------------------------------------------- tensor parallelism
    _tp = None  # (rank, size, group) once shard_fused_layer ran

    def _row(self, x, w, b=None):
        """Row-parallel projection: the rank's partial product, summed over the TP group (the
        bias is held by TP rank 0 only, so the sum adds it once)."""
        y = linear(x, w, b)
        if self._tp is not None:
            from .. import comm as dist
            dist.inference_all_reduce(y, group=self._tp[2])
        return y

    def _alibi_heads(self, alibi, B):
        """This rank's heads of an ALiBi bias built for every head ([B * heads, 1, kv])."""
        if self._tp is None:
            return alibi.view(B, self.nh, 1, -1).float()
        r, n, _ = self._tp
        return alibi.view(B, self.nh * n, 1, -1)[:, r * self.nh:(r + 1) * self.nh].float()

    def _unlink_orig(self):
        """Free the original layer's parameters (their views no longer match the sharded / quantized
        fused tensors) and stop re-linking them."""
        orig = self.__dict__.get("orig")
        if orig is not None:
            for p in orig.parameters():
                p.data = p.data.new_empty(0)
        self.__dict__["_unlinked"] = True

    def _link(self):
        if self.__dict__.get("orig") is None or self.__dict__.get("_unlinked"):
            return
        for param, view in self._links():
            param.data = view


class FusedEncoderLayer(_Fused):
    """Post-LayerNorm encoder layer (BERT / RoBERTa): self-attention, out-proj + residual LN,
    bias-GELU MLP + residual LN."""

    def __init__(self, layer, config):
        super().__init__(layer)
        sa, ao = layer.attention.self, layer.attention.output
        self.nh = sa.num_attention_heads
        self.hd = sa.attention_head_size
        self.w_qkv = self._p(torch.cat([sa.query.weight, sa.key.weight, sa.value.weight]))
        self.b_qkv = self._p(torch.cat([sa.query.bias, sa.key.bias, sa.value.bias]))
        self.w_o, self.b_o = self._p(ao.dense.weight), self._p(ao.dense.bias)
        self.ln1_w, self.ln1_b, self.eps1 = self._p(ao.LayerNorm.weight), self._p(ao.LayerNorm.bias), ao.LayerNorm.eps
        self.w_fc, self.b_fc = self._p(layer.intermediate.dense.weight), self._p(layer.intermediate.dense.bias)
        self.w_out, self.b_out = self._p(layer.output.dense.weight), self._p(layer.output.dense.bias)
        ln2 = layer.output.LayerNorm
        self.ln2_w, self.ln2_b, self.eps2 = self._p(ln2.weight), self._p(ln2.bias), ln2.eps
        self.act = _act_name(getattr(config, "hidden_act", "gelu"))
        self._link()

    def _links(self):
        L, H = self.orig, self.nh * self.hd
        sa, ao = L.attention.self, L.attention.output
        out = []
        for i, lin in enumerate((sa.query, sa.key, sa.value)):
            out += [(lin.weight, self.w_qkv[i * H:(i + 1) * H]), (lin.bias, self.b_qkv[i * H:(i + 1) * H])]
        out += [(ao.dense.weight, self.w_o), (ao.dense.bias, self.b_o), (ao.LayerNorm.weight, self.ln1_w),
                (ao.LayerNorm.bias, self.ln1_b), (L.intermediate.dense.weight, self.w_fc),
                (L.intermediate.dense.bias, self.b_fc), (L.output.dense.weight, self.w_out),
                (L.output.dense.bias, self.b_out), (L.output.LayerNorm.weight, self.ln2_w),
                (L.output.LayerNorm.bias, self.ln2_b)]
        return out

    def forward(self, hidden_states, attention_mask=None, encoder_hidden_states=None, *args, **kwargs):
        if encoder_hidden_states is not None or kwargs.get("output_attentions"):
            return self._delegate(hidden_states, attention_mask, encoder_hidden_states, *args, **kwargs)
        x = hidden_states
        B, S, H = x.shape
        qkv = linear(x, self.w_qkv, self.b_qkv).view(B, S, 3, self.nh, self.hd)
        o = _attend(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], attention_mask, False, 1.0 / math.sqrt(self.hd))
        a = self._row(o.reshape(B, S, -1), self.w_o, self.b_o)
        h, _ = layer_norm(a, self.ln1_w, self.ln1_b, self.eps1, residual=x)
        m = self._row(bias_act(linear(h, self.w_fc), self.b_fc, self.act), self.w_out, self.b_out)
        y, _ = layer_norm(m, self.ln2_w, self.ln2_b, self.eps2, residual=h)
        return y


class FusedGPT2Block(_Fused):
    """Pre-LayerNorm decoder block (GPT-2): LN -> fused QKV -> causal attention (KV cache through
    the HF Cache protocol) -> out-proj; residual folded into LN2; bias-GELU MLP."""

    def __init__(self, block, config):
        super().__init__(block)
        at = block.attn
        self.nh, self.hd = at.num_heads, at.head_dim
        self.layer_idx = at.layer_idx
        t = lambda conv: conv.weight.t()  # HF Conv1D stores [in, out]
        self.w_qkv, self.b_qkv = self._p(t(at.c_attn)), self._p(at.c_attn.bias)
        self.w_o, self.b_o = self._p(t(at.c_proj)), self._p(at.c_proj.bias)
        self.ln1_w, self.ln1_b, self.eps1 = self._p(block.ln_1.weight), self._p(block.ln_1.bias), block.ln_1.eps
        self.ln2_w, self.ln2_b, self.eps2 = self._p(block.ln_2.weight), self._p(block.ln_2.bias), block.ln_2.eps
        self.w_fc, self.b_fc = self._p(t(block.mlp.c_fc)), self._p(block.mlp.c_fc.bias)
        self.w_out, self.b_out = self._p(t(block.mlp.c_proj)), self._p(block.mlp.c_proj.bias)
        self.act = _act_name(getattr(config, "activation_function", "gelu_new"))
        scale = 1.0 / math.sqrt(self.hd) if getattr(at, "scale_attn_weights", True) else 1.0
        if getattr(at, "scale_attn_by_inverse_layer_idx", False):
            scale /= float(self.layer_idx + 1)
        self.scale = scale
        self.cross = getattr(block, "crossattention", None) is not None
        self._link()

    def _links(self):
        b = self.orig
        return [(b.attn.c_attn.weight, self.w_qkv.t()), (b.attn.c_attn.bias, self.b_qkv),
                (b.attn.c_proj.weight, self.w_o.t()), (b.attn.c_proj.bias, self.b_o),
                (b.ln_1.weight, self.ln1_w), (b.ln_1.bias, self.ln1_b), (b.ln_2.weight, self.ln2_w),
                (b.ln_2.bias, self.ln2_b), (b.mlp.c_fc.weight, self.w_fc.t()), (b.mlp.c_fc.bias, self.b_fc),
                (b.mlp.c_proj.weight, self.w_out.t()), (b.mlp.c_proj.bias, self.b_out)]

    def forward(self, hidden_states, past_key_values=None, attention_mask=None, encoder_hidden_states=None,
                *args, **kwargs):
        if self.cross or encoder_hidden_states is not None or kwargs.get("output_attentions"):
            return self._delegate(hidden_states, past_key_values, attention_mask, encoder_hidden_states, *args,
                                  **kwargs)
        x = hidden_states
        B, S, H = x.shape
        y = layer_norm(x, self.ln1_w, self.ln1_b, self.eps1)
        qkv = linear(y, self.w_qkv, self.b_qkv).view(B, S, 3, self.nh, self.hd)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        if past_key_values is not None:
            kt, vt = past_key_values.update(k.transpose(1, 2), v.transpose(1, 2), self.layer_idx)
            k, v = kt.transpose(1, 2), vt.transpose(1, 2)
        o = _attend(q, k, v, attention_mask, attention_mask is None, self.scale)
        a = self._row(o.reshape(B, S, -1), self.w_o, self.b_o)
        h2, h = layer_norm(a, self.ln2_w, self.ln2_b, self.eps2, residual=x)
        m = self._row(bias_act(linear(h2, self.w_fc), self.b_fc, self.act), self.w_out, self.b_out)
        return h + m


def _rope_partial(x, cos, sin):
    """NeoX-style (rotate-half) rotary on the first cos.shape[-1] dims of x [B, S, H, D]; cos/sin
    [B, S, rot] as the HF model's rotary embedding hands them to its layers."""
    cos, sin = cos.unsqueeze(2).to(x.dtype), sin.unsqueeze(2).to(x.dtype)
    rot = cos.shape[-1]
    xr, xp = x[..., :rot], x[..., rot:]
    rotated = torch.cat([-xr[..., rot // 2:], xr[..., :rot // 2]], -1)
    return torch.cat([xr * cos + rotated * sin, xp], -1)


class FusedGPTNeoXLayer(_Fused):
    """GPT-NeoX / Pythia layer (reference containers/gptneox.py): pre-LN, per-head interleaved QKV
    re-packed to [3, heads, D] rows at injection, partial rotary, parallel (or sequential) residual
    with the residual add folded into the post-attention LayerNorm in the sequential form."""

    def __init__(self, layer, config):
        super().__init__(layer)
        at = layer.attention
        self.nh, self.hd = at.num_attention_heads if hasattr(at, "num_attention_heads") else config.num_attention_heads, \
            at.head_size
        self.layer_idx, self.scale = at.layer_idx, float(at.scaling)
        H = at.query_key_value.weight.shape[1]
        w = at.query_key_value.weight.view(self.nh, 3, self.hd, H).transpose(0, 1).reshape(-1, H)
        b = at.query_key_value.bias.view(self.nh, 3, self.hd).transpose(0, 1).reshape(-1)
        self.w_qkv, self.b_qkv = self._p(w), self._p(b)
        self.w_o, self.b_o = self._p(at.dense.weight), self._p(at.dense.bias)
        li, lp = layer.input_layernorm, layer.post_attention_layernorm
        self.ln1_w, self.ln1_b, self.eps1 = self._p(li.weight), self._p(li.bias), li.eps
        self.ln2_w, self.ln2_b, self.eps2 = self._p(lp.weight), self._p(lp.bias), lp.eps
        self.w_fc, self.b_fc = self._p(layer.mlp.dense_h_to_4h.weight), self._p(layer.mlp.dense_h_to_4h.bias)
        self.w_out, self.b_out = self._p(layer.mlp.dense_4h_to_h.weight), self._p(layer.mlp.dense_4h_to_h.bias)
        self.act = _act_name(getattr(config, "hidden_act", "gelu"))
        self.parallel = bool(layer.use_parallel_residual)
        self._link()

    def _links(self):
        L = self.orig
        at = L.attention
        empty = self.w_qkv.new_empty(0)  # head-interleaved QKV has no view: rebuilt per delegated call
        return [(at.query_key_value.weight, empty), (at.query_key_value.bias, self.b_qkv.new_empty(0)),
                (at.dense.weight, self.w_o), (at.dense.bias, self.b_o), (L.input_layernorm.weight, self.ln1_w),
                (L.input_layernorm.bias, self.ln1_b), (L.post_attention_layernorm.weight, self.ln2_w),
                (L.post_attention_layernorm.bias, self.ln2_b), (L.mlp.dense_h_to_4h.weight, self.w_fc),
                (L.mlp.dense_h_to_4h.bias, self.b_fc), (L.mlp.dense_4h_to_h.weight, self.w_out),
                (L.mlp.dense_4h_to_h.bias, self.b_out)]

    def _delegate(self, *args, **kwargs):
        at = self.orig.attention
        H = self.w_qkv.shape[1]
        at.query_key_value.weight.data = self.w_qkv.view(3, self.nh, self.hd, H).transpose(0, 1).reshape(-1, H)
        at.query_key_value.bias.data = self.b_qkv.view(3, self.nh, self.hd).transpose(0, 1).reshape(-1)
        try:
            return self.orig(*args, **kwargs)
        finally:
            self._link()

    def _mlp(self, y):
        return self._row(bias_act(linear(y, self.w_fc), self.b_fc, self.act), self.w_out, self.b_out)

    def forward(self, hidden_states, attention_mask=None, position_ids=None, use_cache=False, layer_past=None,
                position_embeddings=None, **kwargs):
        if position_embeddings is None or kwargs.get("output_attentions"):
            return self._delegate(hidden_states, attention_mask=attention_mask, position_ids=position_ids,
                                  use_cache=use_cache, layer_past=layer_past, position_embeddings=position_embeddings,
                                  **kwargs)
        x = hidden_states
        B, S, H = x.shape
        qkv = linear(layer_norm(x, self.ln1_w, self.ln1_b, self.eps1), self.w_qkv, self.b_qkv)
        qkv = qkv.view(B, S, 3, self.nh, self.hd)
        cos, sin = position_embeddings
        q, k, v = _rope_partial(qkv[:, :, 0], cos, sin), _rope_partial(qkv[:, :, 1], cos, sin), qkv[:, :, 2]
        if layer_past is not None:
            kt, vt = layer_past.update(k.transpose(1, 2), v.transpose(1, 2), self.layer_idx)
            k, v = kt.transpose(1, 2), vt.transpose(1, 2)
        o = _attend(q, k, v, attention_mask, attention_mask is None, self.scale)
        a = self._row(o.reshape(B, S, -1), self.w_o, self.b_o)
        if self.parallel:
            return self._mlp(layer_norm(x, self.ln2_w, self.ln2_b, self.eps2)) + a + x
        y2, h = layer_norm(a, self.ln2_w, self.ln2_b, self.eps2, residual=x)
        return self._mlp(y2) + h


def _rope_half(x, cos, sin):
    """HF Llama-style rotate-half rotary on x [B, S, H, D] with cos/sin [B, S, D]."""
    cos, sin = cos.unsqueeze(2).to(x.dtype), sin.unsqueeze(2).to(x.dtype)
    d = x.shape[-1] // 2
    return x * cos + torch.cat([-x[..., d:], x[..., :d]], -1) * sin


def _attend_gqa(q, k, v, mask, causal, scale):
    """_attend for grouped-query heads (q heads a multiple of kv heads)."""
    if q.shape[2] != k.shape[2] and (mask is not None or q.shape[1] != k.shape[1]
                                     or not (hip_supported(q, k, v) or hip_paddable(q, k, v))):
        rep = q.shape[2] // k.shape[2]
        k, v = k.repeat_interleave(rep, dim=2), v.repeat_interleave(rep, dim=2)
    return _attend(q, k, v, mask, causal, scale)


class FusedLlamaLayer(_Fused):
    """Llama / Mistral / Qwen2 decoder layer (reference containers/llama.py, llama2.py): RMSNorm ->
    one packed [q | k | v] GEMM (GQA, optional biases) -> rotate-half RoPE from the model's
    ``position_embeddings`` -> causal attention with the HF Cache -> o_proj; the residual add is
    folded into the post-attention RMSNorm; gate|up as ONE GEMM -> SwiGLU kernel -> down."""

    def __init__(self, layer, config):
        super().__init__(layer)
        at, mlp = layer.self_attn, layer.mlp
        self.hd = at.head_dim
        self.nq = at.q_proj.weight.shape[0] // self.hd
        self.nkv = at.k_proj.weight.shape[0] // self.hd
        self.layer_idx, self.scale = at.layer_idx, float(at.scaling)
        self.w_qkv = self._p(torch.cat([at.q_proj.weight, at.k_proj.weight, at.v_proj.weight]))
        self.b_qkv = (self._p(torch.cat([at.q_proj.bias, at.k_proj.bias, at.v_proj.bias]))
                      if at.q_proj.bias is not None else None)
        self.w_o = self._p(at.o_proj.weight)
        self.w_gu = self._p(torch.cat([mlp.gate_proj.weight, mlp.up_proj.weight]))
        self.w_down = self._p(mlp.down_proj.weight)
        li, lp = layer.input_layernorm, layer.post_attention_layernorm
        self.ln1_w, self.eps1 = self._p(li.weight), float(getattr(li, "variance_epsilon", getattr(li, "eps", 1e-6)))
        self.ln2_w, self.eps2 = self._p(lp.weight), float(getattr(lp, "variance_epsilon", getattr(lp, "eps", 1e-6)))
        act = getattr(config, "hidden_act", "silu")
        self.swiglu = act in ("silu", "swish")
        self.act = act
        self._link()

    def _links(self):
        L, D = self.orig, self.hd
        at, mlp = L.self_attn, L.mlp
        q, kv = self.nq * D, self.nkv * D
        out = [(at.q_proj.weight, self.w_qkv[:q]), (at.k_proj.weight, self.w_qkv[q:q + kv]),
               (at.v_proj.weight, self.w_qkv[q + kv:]), (at.o_proj.weight, self.w_o),
               (mlp.gate_proj.weight, self.w_gu[:self.w_gu.shape[0] // 2]),
               (mlp.up_proj.weight, self.w_gu[self.w_gu.shape[0] // 2:]), (mlp.down_proj.weight, self.w_down),
               (L.input_layernorm.weight, self.ln1_w), (L.post_attention_layernorm.weight, self.ln2_w)]
        if self.b_qkv is not None:
            out += [(at.q_proj.bias, self.b_qkv[:q]), (at.k_proj.bias, self.b_qkv[q:q + kv]),
                    (at.v_proj.bias, self.b_qkv[q + kv:])]
        return out

    def forward(self, hidden_states, attention_mask=None, position_ids=None, past_key_values=None, use_cache=False,
                position_embeddings=None, **kwargs):
        if position_embeddings is None or kwargs.get("output_attentions") or not self.swiglu:
            return self._delegate(hidden_states, attention_mask=attention_mask, position_ids=position_ids,
                                  past_key_values=past_key_values, use_cache=use_cache,
                                  position_embeddings=position_embeddings, **kwargs)
        from ..ops.activation import swiglu
        from ..ops.norm import rms_norm
        x = hidden_states
        B, S, H = x.shape
        qkv = linear(rms_norm(x, self.ln1_w, self.eps1), self.w_qkv, self.b_qkv)
        qkv = qkv.view(B, S, self.nq + 2 * self.nkv, self.hd)
        cos, sin = position_embeddings
        q = _rope_half(qkv[:, :, :self.nq], cos, sin)
        k = _rope_half(qkv[:, :, self.nq:self.nq + self.nkv], cos, sin)
        v = qkv[:, :, self.nq + self.nkv:]
        if past_key_values is not None:
            kt, vt = past_key_values.update(k.transpose(1, 2), v.transpose(1, 2), self.layer_idx)
            k, v = kt.transpose(1, 2), vt.transpose(1, 2)
        o = _attend_gqa(q, k, v, attention_mask, attention_mask is None, self.scale)
        a = self._row(o.reshape(B, S, self.nq * self.hd), self.w_o)
        y2, h = rms_norm(a, self.ln2_w, self.eps2, residual=x)
        return h + self._row(swiglu(linear(y2, self.w_gu)), self.w_down)


class FusedOPTLayer(_Fused):
    """OPT decoder layer (reference containers/opt.py): packed biased QKV (q pre-scaled by
    head_dim^-0.5 as HF does), causal attention with the HF Cache, out-proj with the residual folded
    into the final LayerNorm (pre-LN models), bias + ReLU MLP."""

    def __init__(self, layer, config):
        super().__init__(layer)
        at = layer.self_attn
        self.nh, self.hd = at.num_heads, at.head_dim
        self.layer_idx, self.scaling = at.layer_idx, float(at.scaling)
        self.w_qkv = self._p(torch.cat([at.q_proj.weight, at.k_proj.weight, at.v_proj.weight]))
        self.b_qkv = self._p(torch.cat([at.q_proj.bias, at.k_proj.bias, at.v_proj.bias]))
        self.w_o, self.b_o = self._p(at.out_proj.weight), self._p(at.out_proj.bias)
        l1, l2 = layer.self_attn_layer_norm, layer.final_layer_norm
        self.ln1_w, self.ln1_b, self.eps1 = self._p(l1.weight), self._p(l1.bias), l1.eps
        self.ln2_w, self.ln2_b, self.eps2 = self._p(l2.weight), self._p(l2.bias), l2.eps
        self.w_fc1, self.b_fc1 = self._p(layer.fc1.weight), self._p(layer.fc1.bias)
        self.w_fc2, self.b_fc2 = self._p(layer.fc2.weight), self._p(layer.fc2.bias)
        self.pre_ln = bool(layer.do_layer_norm_before)
        self.act = getattr(config, "activation_function", "relu")
        self._link()

    def _links(self):
        L, H = self.orig, self.nh * self.hd
        at = L.self_attn
        out = []
        for i, lin in enumerate((at.q_proj, at.k_proj, at.v_proj)):
            out += [(lin.weight, self.w_qkv[i * H:(i + 1) * H]), (lin.bias, self.b_qkv[i * H:(i + 1) * H])]
        return out + [(at.out_proj.weight, self.w_o), (at.out_proj.bias, self.b_o),
                      (L.self_attn_layer_norm.weight, self.ln1_w), (L.self_attn_layer_norm.bias, self.ln1_b),
                      (L.final_layer_norm.weight, self.ln2_w), (L.final_layer_norm.bias, self.ln2_b),
                      (L.fc1.weight, self.w_fc1), (L.fc1.bias, self.b_fc1), (L.fc2.weight, self.w_fc2),
                      (L.fc2.bias, self.b_fc2)]

    def forward(self, hidden_states, attention_mask=None, past_key_values=None, use_cache=False, position_ids=None,
                **kwargs):
        if kwargs.get("output_attentions") or not self.pre_ln or self.act not in ("relu", "gelu", "gelu_new"):
            return self._delegate(hidden_states, attention_mask=attention_mask, past_key_values=past_key_values,
                                  use_cache=use_cache, position_ids=position_ids, **kwargs)
        x = hidden_states
        B, S, H = x.shape
        qkv = linear(layer_norm(x, self.ln1_w, self.ln1_b, self.eps1), self.w_qkv, self.b_qkv).view(
            B, S, 3, self.nh, self.hd)
        q, k, v = qkv[:, :, 0] * self.scaling, qkv[:, :, 1], qkv[:, :, 2]
        if past_key_values is not None:
            kt, vt = past_key_values.update(k.transpose(1, 2), v.transpose(1, 2), self.layer_idx)
            k, v = kt.transpose(1, 2), vt.transpose(1, 2)
        o = _attend(q, k, v, attention_mask, attention_mask is None, 1.0)
        a = self._row(o.reshape(B, S, -1), self.w_o, self.b_o)
        y2, h = layer_norm(a, self.ln2_w, self.ln2_b, self.eps2, residual=x)
        return h + self._row(bias_act(linear(y2, self.w_fc1), self.b_fc1, _act_name(self.act)), self.w_fc2, self.b_fc2)


class FusedGPTJBlock(_Fused):
    """GPT-J block (reference containers/gptj.py): one LayerNorm feeding attention and MLP in
    parallel; packed bias-free QKV; interleaved (rotate-every-two) rotary on the first
    ``rotary_dim`` dims from the model's sinusoid table; attention + MLP + residual summed."""

    def __init__(self, block, config):
        super().__init__(block)
        at = block.attn
        self.nh, self.hd = at.num_attention_heads, at.head_dim
        self.layer_idx, self.rot = at.layer_idx, at.rotary_dim
        self.w_qkv = self._p(torch.cat([at.q_proj.weight, at.k_proj.weight, at.v_proj.weight]))
        self.w_o = self._p(at.out_proj.weight)
        self.ln_w, self.ln_b, self.eps = self._p(block.ln_1.weight), self._p(block.ln_1.bias), block.ln_1.eps
        self.w_in, self.b_in = self._p(block.mlp.fc_in.weight), self._p(block.mlp.fc_in.bias)
        self.w_out, self.b_out = self._p(block.mlp.fc_out.weight), self._p(block.mlp.fc_out.bias)
        self.act = getattr(config, "activation_function", "gelu_new")
        self.register_buffer("embed_positions", at.embed_positions.detach().clone(), persistent=False)  # sin | cos
        self._link()

    def _links(self):
        b, H = self.orig, self.nh * self.hd
        at = b.attn
        return [(at.q_proj.weight, self.w_qkv[:H]), (at.k_proj.weight, self.w_qkv[H:2 * H]),
                (at.v_proj.weight, self.w_qkv[2 * H:]), (at.out_proj.weight, self.w_o), (b.ln_1.weight, self.ln_w),
                (b.ln_1.bias, self.ln_b), (b.mlp.fc_in.weight, self.w_in), (b.mlp.fc_in.bias, self.b_in),
                (b.mlp.fc_out.weight, self.w_out), (b.mlp.fc_out.bias, self.b_out)]

    def _rotary(self, x, sin, cos):
        r = self.rot or x.shape[-1]
        xr, xp = x[..., :r], x[..., r:]
        sin = sin.repeat_interleave(2, -1).unsqueeze(2).to(x.dtype)
        cos = cos.repeat_interleave(2, -1).unsqueeze(2).to(x.dtype)
        rot = torch.stack((-xr[..., 1::2], xr[..., ::2]), dim=-1).flatten(-2)
        return torch.cat([xr * cos + rot * sin, xp], -1)

    def forward(self, hidden_states, layer_past=None, attention_mask=None, position_ids=None, use_cache=False,
                output_attentions=False, **kwargs):
        if output_attentions or position_ids is None:
            return self._delegate(hidden_states, layer_past=layer_past, attention_mask=attention_mask,
                                  position_ids=position_ids, use_cache=use_cache, output_attentions=output_attentions,
                                  **kwargs)
        x = hidden_states
        B, S, H = x.shape
        y = layer_norm(x, self.ln_w, self.ln_b, self.eps)
        qkv = linear(y, self.w_qkv).view(B, S, 3, self.nh, self.hd)
        sincos = self.embed_positions[position_ids].to(x.dtype)  # [B, S, rot]
        sin, cos = torch.split(sincos, sincos.shape[-1] // 2, dim=-1)
        q, k, v = self._rotary(qkv[:, :, 0], sin, cos), self._rotary(qkv[:, :, 1], sin, cos), qkv[:, :, 2]
        if layer_past is not None:
            kt, vt = layer_past.update(k.transpose(1, 2), v.transpose(1, 2), self.layer_idx)
            k, v = kt.transpose(1, 2), vt.transpose(1, 2)
        o = _attend(q.float(), k.float(), v.float(), attention_mask, attention_mask is None,
                    1.0 / math.sqrt(self.hd)).to(x.dtype)  # GPT-J attends in fp32
        a = self._row(o.reshape(B, S, -1), self.w_o)
        m = self._row(bias_act(linear(y, self.w_in), self.b_in, _act_name(self.act)), self.w_out, self.b_out)
        return a + m + x, None


class FusedDistilBertBlock(_Fused):
    """DistilBERT encoder block (reference containers/distil_bert.py): packed biased QKV,
    bidirectional attention, residual-fused post-LayerNorms, bias-GELU FFN."""

    def __init__(self, block, config):
        super().__init__(block)
        at = block.attention
        self.nh = at.n_heads
        self.hd = at.dim // at.n_heads
        self.w_qkv = self._p(torch.cat([at.q_lin.weight, at.k_lin.weight, at.v_lin.weight]))
        self.b_qkv = self._p(torch.cat([at.q_lin.bias, at.k_lin.bias, at.v_lin.bias]))
        self.w_o, self.b_o = self._p(at.out_lin.weight), self._p(at.out_lin.bias)
        l1, l2 = block.sa_layer_norm, block.output_layer_norm
        self.ln1_w, self.ln1_b, self.eps1 = self._p(l1.weight), self._p(l1.bias), l1.eps
        self.ln2_w, self.ln2_b, self.eps2 = self._p(l2.weight), self._p(l2.bias), l2.eps
        self.w1, self.b1 = self._p(block.ffn.lin1.weight), self._p(block.ffn.lin1.bias)
        self.w2, self.b2 = self._p(block.ffn.lin2.weight), self._p(block.ffn.lin2.bias)
        self.act = _act_name(getattr(config, "activation", "gelu"))
        self._link()

    def _links(self):
        b, H = self.orig, self.nh * self.hd
        at = b.attention
        out = []
        for i, lin in enumerate((at.q_lin, at.k_lin, at.v_lin)):
            out += [(lin.weight, self.w_qkv[i * H:(i + 1) * H]), (lin.bias, self.b_qkv[i * H:(i + 1) * H])]
        return out + [(at.out_lin.weight, self.w_o), (at.out_lin.bias, self.b_o), (b.sa_layer_norm.weight, self.ln1_w),
                      (b.sa_layer_norm.bias, self.ln1_b), (b.output_layer_norm.weight, self.ln2_w),
                      (b.output_layer_norm.bias, self.ln2_b), (b.ffn.lin1.weight, self.w1), (b.ffn.lin1.bias, self.b1),
                      (b.ffn.lin2.weight, self.w2), (b.ffn.lin2.bias, self.b2)]

    def forward(self, hidden_states, attention_mask=None, **kwargs):
        if kwargs.get("output_attentions"):
            return self._delegate(hidden_states, attention_mask=attention_mask, **kwargs)
        x = hidden_states
        B, S, H = x.shape
        qkv = linear(x, self.w_qkv, self.b_qkv).view(B, S, 3, self.nh, self.hd)
        o = _attend(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], attention_mask, False, 1.0 / math.sqrt(self.hd))
        a = self._row(o.reshape(B, S, -1), self.w_o, self.b_o)
        h, _ = layer_norm(a, self.ln1_w, self.ln1_b, self.eps1, residual=x)
        f = self._row(bias_act(linear(h, self.w1), self.b1, self.act), self.w2, self.b2)
        y, _ = layer_norm(f, self.ln2_w, self.ln2_b, self.eps2, residual=h)
        return y


def _probs_context(scores, v, mask, alibi, causal, window, scale):
    """softmax(scale * scores + alibi + mask) @ v through the HIP masked softmax (softmax.hip):
    scores [B, H, q, k] fp32, v [B, H, k, D]; a bool mask keeps True, a float mask is additive."""
    from ..ops.inference_ops import softmax
    if mask is not None and mask.dim() == 2:
        mask = mask[:, None, None, :]
    p = softmax(scores, attn_mask=mask, alibi=alibi, triangular=causal, local_attention=window > 0,
                window_size=max(window, 1), layer_scale=scale)
    return torch.matmul(p.to(v.dtype), v)


class FusedBloomBlock(_Fused):
    """BLOOM block (reference containers/bloom.py ``BLOOMLayerPolicy``): LN -> head-interleaved packed
    QKV GEMM (kept in Bloom's [head][q|k|v][d] layout, so no repacking) -> scores -> ONE HIP masked
    softmax kernel applying the ALiBi bias, the additive / causal mask and the 1/sqrt(d) scale ->
    context GEMM -> dense + residual -> LN -> bias-GELU MLP + residual."""

    def __init__(self, block, config):
        super().__init__(block)
        at = block.self_attention
        self.nh, self.hd = at.num_heads, at.head_dim
        self.layer_idx = at.layer_idx
        self.inv_norm = float(at.inv_norm_factor)
        self.post_ln_residual = bool(block.apply_residual_connection_post_layernorm)
        self.w_qkv, self.b_qkv = self._p(at.query_key_value.weight), self._p(at.query_key_value.bias)
        self.w_o, self.b_o = self._p(at.dense.weight), self._p(at.dense.bias)
        l1, l2 = block.input_layernorm, block.post_attention_layernorm
        self.ln1_w, self.ln1_b, self.eps1 = self._p(l1.weight), self._p(l1.bias), l1.eps
        self.ln2_w, self.ln2_b, self.eps2 = self._p(l2.weight), self._p(l2.bias), l2.eps
        mlp = block.mlp
        self.w_fc, self.b_fc = self._p(mlp.dense_h_to_4h.weight), self._p(mlp.dense_h_to_4h.bias)
        self.w_out, self.b_out = self._p(mlp.dense_4h_to_h.weight), self._p(mlp.dense_4h_to_h.bias)
        self._link()

    def _links(self):
        b = self.orig
        at, mlp = b.self_attention, b.mlp
        return [(at.query_key_value.weight, self.w_qkv), (at.query_key_value.bias, self.b_qkv),
                (at.dense.weight, self.w_o), (at.dense.bias, self.b_o),
                (b.input_layernorm.weight, self.ln1_w), (b.input_layernorm.bias, self.ln1_b),
                (b.post_attention_layernorm.weight, self.ln2_w), (b.post_attention_layernorm.bias, self.ln2_b),
                (mlp.dense_h_to_4h.weight, self.w_fc), (mlp.dense_h_to_4h.bias, self.b_fc),
                (mlp.dense_4h_to_h.weight, self.w_out), (mlp.dense_4h_to_h.bias, self.b_out)]

    def forward(self, hidden_states, alibi=None, attention_mask=None, layer_past=None, use_cache=False,
                output_attentions=False, **kwargs):
        if output_attentions or alibi is None:
            return self._delegate(hidden_states, alibi, attention_mask, layer_past=layer_past, use_cache=use_cache,
                                  output_attentions=output_attentions, **kwargs)
        x = hidden_states
        B, S, H = x.shape
        y = layer_norm(x, self.ln1_w, self.ln1_b, self.eps1)
        qkv = linear(y, self.w_qkv, self.b_qkv).view(B, S, self.nh, 3, self.hd)
        q, k, v = (qkv[..., i, :].transpose(1, 2) for i in range(3))  # [B, nh, S, hd]
        if layer_past is not None:
            k, v = layer_past.update(k, v, self.layer_idx)
        scores = torch.matmul(q, k.transpose(-1, -2)).float()
        ab = self._alibi_heads(alibi, B)  # HF builds [B*nh, 1, kv]
        o = _probs_context(scores, v, attention_mask, ab, attention_mask is None, 0, self.inv_norm)
        res = y if self.post_ln_residual else x
        a = self._row(o.transpose(1, 2).reshape(B, S, -1), self.w_o, self.b_o)
        h2, h = layer_norm(a, self.ln2_w, self.ln2_b, self.eps2, residual=res)
        res2 = h2 if self.post_ln_residual else h
        m = self._row(bias_act(linear(h2, self.w_fc), self.b_fc, "gelu"), self.w_out, self.b_out)
        return res2 + m, None


class FusedGPTNeoBlock(_Fused):
    """GPT-Neo block (reference containers/gptneo.py ``HFGPTNEOLayerPolicy``): LN -> q|k|v packed
    into one GEMM -> unscaled fp32 scores (GPT-Neo applies no 1/sqrt(d)) -> ONE HIP masked softmax
    with the causal and, on "local" layers, the sliding-window mask -> out-proj + residual folded
    into LN2 -> bias-GELU MLP + residual."""

    def __init__(self, block, config):
        super().__init__(block)
        at = block.attn.attention
        self.nh, self.hd = at.num_heads, at.head_dim
        self.layer_idx = at.layer_id
        self.window = int(config.window_size) if at.attention_type == "local" else 0
        self.w_qkv = self._p(torch.cat([at.q_proj.weight, at.k_proj.weight, at.v_proj.weight]))
        self.w_o, self.b_o = self._p(at.out_proj.weight), self._p(at.out_proj.bias)
        self.ln1_w, self.ln1_b, self.eps1 = self._p(block.ln_1.weight), self._p(block.ln_1.bias), block.ln_1.eps
        self.ln2_w, self.ln2_b, self.eps2 = self._p(block.ln_2.weight), self._p(block.ln_2.bias), block.ln_2.eps
        self.w_fc, self.b_fc = self._p(block.mlp.c_fc.weight), self._p(block.mlp.c_fc.bias)
        self.w_out, self.b_out = self._p(block.mlp.c_proj.weight), self._p(block.mlp.c_proj.bias)
        self.act = _act_name(getattr(config, "activation_function", "gelu_new"))
        self._link()

    def _links(self):
        b = self.orig
        at = b.attn.attention
        H = self.nh * self.hd
        return [(at.q_proj.weight, self.w_qkv[:H]), (at.k_proj.weight, self.w_qkv[H:2 * H]),
                (at.v_proj.weight, self.w_qkv[2 * H:]), (at.out_proj.weight, self.w_o), (at.out_proj.bias, self.b_o),
                (b.ln_1.weight, self.ln1_w), (b.ln_1.bias, self.ln1_b), (b.ln_2.weight, self.ln2_w),
                (b.ln_2.bias, self.ln2_b), (b.mlp.c_fc.weight, self.w_fc), (b.mlp.c_fc.bias, self.b_fc),
                (b.mlp.c_proj.weight, self.w_out), (b.mlp.c_proj.bias, self.b_out)]

    def forward(self, hidden_states, layer_past=None, attention_mask=None, use_cache=False, output_attentions=False,
                **kwargs):
        if output_attentions:
            return self._delegate(hidden_states, layer_past=layer_past, attention_mask=attention_mask,
                                  use_cache=use_cache, output_attentions=output_attentions, **kwargs)
        x = hidden_states
        B, S, H = x.shape
        y = layer_norm(x, self.ln1_w, self.ln1_b, self.eps1)
        qkv = linear(y, self.w_qkv).view(B, S, 3, self.nh, self.hd)
        q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
        if layer_past is not None:
            k, v = layer_past.update(k, v, self.layer_idx)
        scores = torch.matmul(q.float(), k.float().transpose(-1, -2))
        o = _probs_context(scores, v, attention_mask, None, True, self.window, 1.0)
        a = self._row(o.transpose(1, 2).reshape(B, S, -1), self.w_o, self.b_o)
        h2, h = layer_norm(a, self.ln2_w, self.ln2_b, self.eps2, residual=x)
        m = self._row(bias_act(linear(h2, self.w_fc), self.b_fc, self.act), self.w_out, self.b_out)
        return h + m, None


class FusedCLIPEncoderLayer(_Fused):
    """CLIP text / vision encoder layer (reference containers/clip.py ``HFCLIPLayerPolicy``): pre-LN,
    packed biased QKV GEMM, flash attention (causal for the text tower, through ``is_causal`` or
    its 4-D mask), out-proj + residual folded into LN2, bias + quick-GELU MLP (HIP kernel)."""

    def __init__(self, layer, config):
        super().__init__(layer)
        at = layer.self_attn
        self.nh, self.hd = at.num_heads, at.head_dim
        self.scale = float(at.scale)
        self.w_qkv = self._p(torch.cat([at.q_proj.weight, at.k_proj.weight, at.v_proj.weight]))
        self.b_qkv = self._p(torch.cat([at.q_proj.bias, at.k_proj.bias, at.v_proj.bias]))
        self.w_o, self.b_o = self._p(at.out_proj.weight), self._p(at.out_proj.bias)
        l1, l2 = layer.layer_norm1, layer.layer_norm2
        self.ln1_w, self.ln1_b, self.eps1 = self._p(l1.weight), self._p(l1.bias), l1.eps
        self.ln2_w, self.ln2_b, self.eps2 = self._p(l2.weight), self._p(l2.bias), l2.eps
        self.w_fc, self.b_fc = self._p(layer.mlp.fc1.weight), self._p(layer.mlp.fc1.bias)
        self.w_out, self.b_out = self._p(layer.mlp.fc2.weight), self._p(layer.mlp.fc2.bias)
        self.act = _act_name(getattr(getattr(layer.mlp, "config", config), "hidden_act", "quick_gelu"))
        self._link()

    def _links(self):
        L = self.orig
        at, H = L.self_attn, self.nh * self.hd
        out = []
        for i, lin in enumerate((at.q_proj, at.k_proj, at.v_proj)):
            out += [(lin.weight, self.w_qkv[i * H:(i + 1) * H]), (lin.bias, self.b_qkv[i * H:(i + 1) * H])]
        return out + [(at.out_proj.weight, self.w_o), (at.out_proj.bias, self.b_o),
                      (L.layer_norm1.weight, self.ln1_w), (L.layer_norm1.bias, self.ln1_b),
                      (L.layer_norm2.weight, self.ln2_w), (L.layer_norm2.bias, self.ln2_b),
                      (L.mlp.fc1.weight, self.w_fc), (L.mlp.fc1.bias, self.b_fc),
                      (L.mlp.fc2.weight, self.w_out), (L.mlp.fc2.bias, self.b_out)]

    def forward(self, hidden_states, attention_mask=None, *args, **kwargs):
        if kwargs.get("output_attentions") or args:
            return self._delegate(hidden_states, attention_mask, *args, **kwargs)
        x = hidden_states
        B, S, H = x.shape
        y = layer_norm(x, self.ln1_w, self.ln1_b, self.eps1)
        qkv = linear(y, self.w_qkv, self.b_qkv).view(B, S, 3, self.nh, self.hd)
        causal = bool(kwargs.get("is_causal", False)) and attention_mask is None
        o = _attend(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], attention_mask, causal, self.scale)
        a = self._row(o.reshape(B, S, -1), self.w_o, self.b_o)
        h2, h = layer_norm(a, self.ln2_w, self.ln2_b, self.eps2, residual=x)
        m = self._row(bias_act(linear(h2, self.w_fc), self.b_fc, self.act), self.w_out, self.b_out)
        return h + m


class FusedMegatronLayer(_Fused):
    """Megatron-LM GPT ``ParallelTransformerLayer`` (reference containers/megatron_gpt.py
    ``MegatronLayerPolicy`` + features/megatron.py, and megatron_gpt_moe.py for its MoE form):
    sequence-first hidden states [S, B, H], pre-LayerNorm, ONE packed QKV GEMM -- Megatron v2
    stores query_key_value per head as [q_h | k_h | v_h] row blocks; the policy re-packs them to
    [q | k | v] once (``_align_qkv_transposed``) --, causal flash attention, dense + residual folded
    into the post-attention LayerNorm, bias-GELU MLP (or the layer's own MoE / expert module, whose
    first output is kept), residual. ``attention`` (v1) and ``self_attention`` (v2) are both
    recognised; ``apply_residual_connection_post_layernorm`` is honoured. KV-cache, cross-attention
    and non-causal masks go to the original layer."""

    def __init__(self, layer, config):
        super().__init__(layer)
        at = getattr(layer, "self_attention", None) or layer.attention
        self.v2 = hasattr(layer, "self_attention")
        qkv = at.query_key_value
        H = qkv.weight.shape[1]
        self.nh = int(getattr(at, "num_attention_heads", getattr(at, "num_attention_heads_per_partition", 0)) or
                      getattr(config, "num_attention_heads"))
        self.hd = qkv.weight.shape[0] // (3 * self.nh)
        w, b = qkv.weight, qkv.bias
        if self.v2:  # [nh, 3, hd, H] -> [3, nh, hd, H]
            w = w.view(self.nh, 3, self.hd, H).transpose(0, 1).reshape(3 * self.nh * self.hd, H)
            b = b.view(self.nh, 3, self.hd).transpose(0, 1).reshape(-1) if b is not None else None
        self.w_qkv = self._p(w)
        self.b_qkv = self._p(b) if b is not None else None
        self.w_o = self._p(at.dense.weight)
        self.b_o = self._p(at.dense.bias) if at.dense.bias is not None else None
        li, lp = layer.input_layernorm, layer.post_attention_layernorm
        self.ln1_w, self.ln1_b, self.eps1 = self._p(li.weight), self._p(li.bias), float(getattr(li, "eps", 1e-5))
        self.ln2_w, self.ln2_b, self.eps2 = self._p(lp.weight), self._p(lp.bias), float(getattr(lp, "eps", 1e-5))
        self.post_ln_residual = bool(getattr(layer, "apply_residual_connection_post_layernorm", False))
        mlp = layer.mlp
        self.dense_mlp = hasattr(mlp, "dense_h_to_4h")
        if self.dense_mlp:
            self.w_fc, self.b_fc = self._p(mlp.dense_h_to_4h.weight), self._p(mlp.dense_h_to_4h.bias)
            self.w_out, self.b_out = self._p(mlp.dense_4h_to_h.weight), self._p(mlp.dense_4h_to_h.bias)
        else:
            self.mlp = mlp  # MoE (megatron_gpt_moe): the expert layer runs as is
        self.act = _act_name(getattr(config, "hidden_act", "gelu")) if config is not None else "gelu_exact"
        self._link()

    def _links(self):
        if self.v2:
            return []  # the per-head interleaved QKV has no view of the re-packed weight
        at = self.orig.attention
        out = [(at.query_key_value.weight, self.w_qkv), (at.dense.weight, self.w_o)]
        if self.b_qkv is not None:
            out.append((at.query_key_value.bias, self.b_qkv))
        return out

    @staticmethod
    def _is_causal_mask(mask, S):
        if mask is None:
            return True
        if mask.dtype != torch.bool or mask.shape[-1] != S or mask.shape[-2] != S:
            return False
        m = mask.reshape(-1, S, S)
        ref = torch.ones(S, S, dtype=torch.bool, device=mask.device).triu(1)  # True = masked (Megatron)
        return bool((m == ref).all())

    def forward(self, hidden_states, attention_mask=None, encoder_output=None, enc_dec_attn_mask=None,
                layer_past=None, get_key_value=False, **kwargs):
        S, B, H = hidden_states.shape
        if (encoder_output is not None or layer_past is not None or get_key_value
                or not self._is_causal_mask(attention_mask, S)):
            return self._delegate(hidden_states, attention_mask, encoder_output=encoder_output,
                                  enc_dec_attn_mask=enc_dec_attn_mask, layer_past=layer_past,
                                  get_key_value=get_key_value, **kwargs)
        x = hidden_states.transpose(0, 1)  # [B, S, H]
        ln1 = layer_norm(x, self.ln1_w, self.ln1_b, self.eps1)
        qkv = linear(ln1, self.w_qkv, self.b_qkv).view(B, S, 3, self.nh, self.hd)
        o = _attend(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], None, True, 1.0 / math.sqrt(self.hd))
        a = self._row(o.reshape(B, S, self.nh * self.hd), self.w_o, self.b_o)
        ln2, h = layer_norm(a, self.ln2_w, self.ln2_b, self.eps2, residual=ln1 if self.post_ln_residual else x)
        if self.dense_mlp:
            m = self._row(bias_act(linear(ln2, self.w_fc), self.b_fc, self.act), self.w_out, self.b_out)
        else:
            m = self.mlp(ln2)
            m = m[0] if isinstance(m, tuple) else m
        y = (ln2 if self.post_ln_residual else h) + m
        return y.transpose(0, 1).contiguous()


def _is_causal_additive(mask, Sq, Sk):
    """An HF additive mask [B, 1, Sq, Sk] that is exactly the bottom-right causal pattern (no padding):
    the fused causal kernel can replace it."""
    if mask is None:
        return True
    if mask.dim() != 4 or mask.shape[-2] != Sq or mask.shape[-1] != Sk:
        return False
    vis = torch.ones(Sq, Sk, dtype=torch.bool, device=mask.device).tril(Sk - Sq)
    m = mask.reshape(-1, Sq, Sk)
    return bool(((m == 0) == vis).all())


class FusedInternLMLayer(_Fused):
    """InternLM (v1) ``InternLMDecoderLayer`` (reference containers/internlm.py
    ``InternLMLayerPolicy``): the Llama structure with biased q/k/v/o projections and the rotary
    table inside the attention module (``rotary_emb(x, seq_len)`` -> cos/sin indexed by
    ``position_ids``). RMSNorm -> one packed biased QKV GEMM -> rotate-half RoPE -> causal attention
    (legacy tuple KV cache) -> o_proj -> residual folded into the post-attention RMSNorm -> gate|up
    GEMM -> SwiGLU -> down. Returns the HF-v4 tuple ``(hidden, [attn_weights], [present])``."""

    def __init__(self, layer, config):
        super().__init__(layer)
        at, mlp = layer.self_attn, layer.mlp
        self.nh = int(getattr(at, "num_heads", getattr(config, "num_attention_heads", 0)))
        self.hd = at.q_proj.weight.shape[0] // self.nh
        self.w_qkv = self._p(torch.cat([at.q_proj.weight, at.k_proj.weight, at.v_proj.weight]))
        self.b_qkv = (self._p(torch.cat([at.q_proj.bias, at.k_proj.bias, at.v_proj.bias]))
                      if at.q_proj.bias is not None else None)
        self.w_o = self._p(at.o_proj.weight)
        self.b_o = self._p(at.o_proj.bias) if at.o_proj.bias is not None else None
        self.w_gu = self._p(torch.cat([mlp.gate_proj.weight, mlp.up_proj.weight]))
        self.w_down = self._p(mlp.down_proj.weight)
        li, lp = layer.input_layernorm, layer.post_attention_layernorm
        self.ln1_w, self.eps1 = self._p(li.weight), float(getattr(li, "variance_epsilon", 1e-6))
        self.ln2_w, self.eps2 = self._p(lp.weight), float(getattr(lp, "variance_epsilon", 1e-6))
        self._link()

    def _links(self):
        L, q = self.orig, self.nh * self.hd
        at, mlp = L.self_attn, L.mlp
        out = [(at.q_proj.weight, self.w_qkv[:q]), (at.k_proj.weight, self.w_qkv[q:2 * q]),
               (at.v_proj.weight, self.w_qkv[2 * q:]), (at.o_proj.weight, self.w_o),
               (mlp.gate_proj.weight, self.w_gu[:self.w_gu.shape[0] // 2]),
               (mlp.up_proj.weight, self.w_gu[self.w_gu.shape[0] // 2:]), (mlp.down_proj.weight, self.w_down),
               (L.input_layernorm.weight, self.ln1_w), (L.post_attention_layernorm.weight, self.ln2_w)]
        if self.b_qkv is not None:
            out += [(at.q_proj.bias, self.b_qkv[:q]), (at.k_proj.bias, self.b_qkv[q:2 * q]),
                    (at.v_proj.bias, self.b_qkv[2 * q:])]
        if self.b_o is not None:
            out.append((at.o_proj.bias, self.b_o))
        return out

    def forward(self, hidden_states, attention_mask=None, position_ids=None, past_key_value=None,
                output_attentions=False, use_cache=False, **kwargs):
        if output_attentions:
            return self._delegate(hidden_states, attention_mask=attention_mask, position_ids=position_ids,
                                  past_key_value=past_key_value, output_attentions=output_attentions,
                                  use_cache=use_cache, **kwargs)
        from ..ops.activation import swiglu
        from ..ops.norm import rms_norm
        x = hidden_states
        B, S, H = x.shape
        past = past_key_value[0].shape[-2] if past_key_value is not None else 0
        if position_ids is None:
            position_ids = torch.arange(past, past + S, device=x.device).unsqueeze(0).expand(B, S)
        qkv = linear(rms_norm(x, self.ln1_w, self.eps1), self.w_qkv, self.b_qkv).view(B, S, 3, self.nh, self.hd)
        cos, sin = self.orig.self_attn.rotary_emb(qkv, seq_len=past + S)
        cos, sin = cos.reshape(-1, self.hd)[position_ids], sin.reshape(-1, self.hd)[position_ids]  # [B, S, D]
        q, k, v = _rope_half(qkv[:, :, 0], cos, sin), _rope_half(qkv[:, :, 1], cos, sin), qkv[:, :, 2]
        present = None
        if past_key_value is not None:  # legacy ([B, H, S, D], [B, H, S, D]) cache
            k = torch.cat([past_key_value[0].transpose(1, 2), k], 1)
            v = torch.cat([past_key_value[1].transpose(1, 2), v], 1)
        if use_cache:
            present = (k.transpose(1, 2), v.transpose(1, 2))
        causal_only = _is_causal_additive(attention_mask, S, k.shape[1])
        o = _attend(q, k, v, None if causal_only else attention_mask, causal_only, 1.0 / math.sqrt(self.hd))
        a = self._row(o.reshape(B, S, -1), self.w_o, self.b_o)
        y2, h = rms_norm(a, self.ln2_w, self.eps2, residual=x)
        out = (h + self._row(swiglu(linear(y2, self.w_gu)), self.w_down),)
        return out + ((present,) if use_cache else ())


# layer class name -> fused layer constructor (reference containers/__init__.py policy list)
POLICIES = {
    "BertLayer": FusedEncoderLayer,
    "RobertaLayer": FusedEncoderLayer,
    "GPT2Block": FusedGPT2Block,
    "GPTNeoXLayer": FusedGPTNeoXLayer,
    "LlamaDecoderLayer": FusedLlamaLayer,
    "MistralDecoderLayer": FusedLlamaLayer,
    "Qwen2DecoderLayer": FusedLlamaLayer,
    "OPTDecoderLayer": FusedOPTLayer,
    "GPTJBlock": FusedGPTJBlock,
    "TransformerBlock": FusedDistilBertBlock,  # DistilBERT
    "BloomBlock": FusedBloomBlock,
    "GPTNeoBlock": FusedGPTNeoBlock,
    "CLIPEncoderLayer": FusedCLIPEncoderLayer,
    "ParallelTransformerLayer": FusedMegatronLayer,  # Megatron-LM GPT (dense and MoE)
    "InternLMDecoderLayer": FusedInternLMLayer,
}


def _is_decoder_layer(layer, config):
    sa = getattr(getattr(layer, "attention", None), "self", None)
    return bool(getattr(config, "is_decoder", False) or getattr(layer, "is_decoder", False)
                or getattr(sa, "is_causal", False) or getattr(sa, "is_decoder", False)
                or getattr(layer, "add_cross_attention", False))


def replace_transformer_layer(model, config=None):
    """Replace every layer with an injection policy by its fused counterpart; returns the number of
    replaced layers (0 = the model's layers have no policy, e.g. this framework's own models,
    which already run the gfx950 kernels)."""
    config = config if config is not None else getattr(model, "config", None)
    n = 0
    for parent in list(model.modules()):
        for name, child in list(parent.named_children()):
            ctor = POLICIES.get(type(child).__name__)
            if ctor is FusedDistilBertBlock and not hasattr(child, "sa_layer_norm"):
                continue  # another library's "TransformerBlock"
            if ctor is FusedEncoderLayer and _is_decoder_layer(child, config):
                continue  # causal self-attention + KV cache: the encoder fusion does not apply
            if ctor is not None:
                setattr(parent, name, ctor(child, config))
                n += 1
    return n


# ------------------------------------------------------------------------------------------------
# Tensor parallelism of injected layers (reference replace_module.py:207-231: the containers' qkv /
# mlp tensors are sliced per rank by ReplaceWithTensorSlicing and the attention-out / MLP-out
# GEMMs all-reduce). Per fused class: the head counts divided by the TP degree, the packed QKV
# layout ("3": [q|k|v] x heads x hd rows, "h3": Bloom's [head][q|k|v][hd], "gqa": [nq | nkv | nkv]
# heads), the column-parallel (output-row) projections, the packed gate|up projections and the
# row-parallel (input-column) projections whose products ``_row`` sums over the TP group.
_ENC = dict(heads=("nh",), qkv=("w_qkv", "b_qkv", "3"), col=[("w_fc", "b_fc")], gu=[],
            row=[("w_o", "b_o"), ("w_out", "b_out")])
TP_SPECS = {
    FusedEncoderLayer: _ENC, FusedGPT2Block: _ENC, FusedGPTNeoXLayer: _ENC, FusedCLIPEncoderLayer: _ENC,
    FusedMegatronLayer: _ENC,
    FusedLlamaLayer: dict(heads=("nq", "nkv"), qkv=("w_qkv", "b_qkv", "gqa"), col=[], gu=["w_gu"],
                          row=[("w_o", None), ("w_down", None)]),
    FusedInternLMLayer: dict(heads=("nh",), qkv=("w_qkv", "b_qkv", "3"), col=[], gu=["w_gu"],
                             row=[("w_o", "b_o"), ("w_down", None)]),
    FusedOPTLayer: dict(heads=("nh",), qkv=("w_qkv", "b_qkv", "3"), col=[("w_fc1", "b_fc1")], gu=[],
                        row=[("w_o", "b_o"), ("w_fc2", "b_fc2")]),
    FusedGPTJBlock: dict(heads=("nh",), qkv=("w_qkv", None, "3"), col=[("w_in", "b_in")], gu=[],
                         row=[("w_o", None), ("w_out", "b_out")]),
    FusedDistilBertBlock: dict(heads=("nh",), qkv=("w_qkv", "b_qkv", "3"), col=[("w1", "b1")], gu=[],
                               row=[("w_o", "b_o"), ("w2", "b2")]),
    FusedBloomBlock: dict(heads=("nh",), qkv=("w_qkv", "b_qkv", "h3"), col=[("w_fc", "b_fc")], gu=[],
                          row=[("w_o", "b_o"), ("w_out", "b_out")]),
    FusedGPTNeoBlock: dict(heads=("nh",), qkv=("w_qkv", None, "3"), col=[("w_fc", "b_fc")], gu=[],
                           row=[("w_o", "b_o"), ("w_out", "b_out")]),
}


def _rows(t, r, n):
    k = t.shape[0] // n
    return t[r * k:(r + 1) * k]


def _cut_qkv(t, kind, heads, hd, r, n):
    tail = tuple(t.shape[1:])
    if kind == "3":
        nh = heads[0]
        return t.reshape(3, nh, hd, *tail)[:, r * nh // n:(r + 1) * nh // n].reshape(-1, *tail)
    if kind == "h3":
        nh = heads[0]
        return t.reshape(nh, 3 * hd, *tail)[r * nh // n:(r + 1) * nh // n].reshape(-1, *tail)
    nq, nkv = heads
    q = t[:nq * hd].reshape(nq, hd, *tail)[r * nq // n:(r + 1) * nq // n]
    k = t[nq * hd:(nq + nkv) * hd].reshape(nkv, hd, *tail)[r * nkv // n:(r + 1) * nkv // n]
    v = t[(nq + nkv) * hd:].reshape(nkv, hd, *tail)[r * nkv // n:(r + 1) * nkv // n]
    return torch.cat([q.reshape(-1, *tail), k.reshape(-1, *tail), v.reshape(-1, *tail)])


def shard_fused_layer(layer, rank, size, group):
    """Slice one injected layer to TP rank ``rank`` of ``size`` (in place)."""
    spec = TP_SPECS.get(type(layer))
    if spec is None:
        raise NotImplementedError(f"no tensor-parallel layout for {type(layer).__name__}")
    if isinstance(layer, FusedMegatronLayer) and not layer.dense_mlp:
        raise NotImplementedError("Megatron MoE layers under tensor parallelism: shard the experts with expert "
                                  "parallelism instead")
    heads = [int(getattr(layer, h)) for h in spec["heads"]]
    if any(h % size for h in heads):
        raise ValueError(f"{type(layer).__name__}: {dict(zip(spec['heads'], heads))} heads are not divisible by "
                         f"tp_size={size}")

    def put(name, t):
        setattr(layer, name, nn.Parameter(t.contiguous().clone(), requires_grad=False))

    wq, bq, kind = spec["qkv"]
    put(wq, _cut_qkv(getattr(layer, wq), kind, heads, layer.hd, rank, size))
    if bq is not None and getattr(layer, bq, None) is not None:
        put(bq, _cut_qkv(getattr(layer, bq), kind, heads, layer.hd, rank, size))
    for w, b in spec["col"]:
        put(w, _rows(getattr(layer, w), rank, size))
        if b is not None and getattr(layer, b, None) is not None:
            put(b, _rows(getattr(layer, b), rank, size))
    for w in spec["gu"]:
        t = getattr(layer, w)
        half = t.shape[0] // 2
        put(w, torch.cat([_rows(t[:half], rank, size), _rows(t[half:], rank, size)]))
    for w, b in spec["row"]:
        t = getattr(layer, w)
        k = t.shape[1] // size
        put(w, t[:, rank * k:(rank + 1) * k])
        if b is not None and getattr(layer, b, None) is not None and rank != 0:
            put(b, torch.zeros_like(getattr(layer, b)))  # added once: by TP rank 0
    for h, v in zip(spec["heads"], heads):
        setattr(layer, h, v // size)
    layer._unlink_orig()
    layer._tp = (rank, size, group)
    return layer


def shard_fused_layers(model, rank, size, group):
    """Slice every injected layer of ``model`` for TP rank ``rank``; the rest of the model (embeddings,
    final norm, LM head) stays replicated. Returns the number of sharded layers."""
    n = 0
    for m in model.modules():
        if isinstance(m, _Fused):
            shard_fused_layer(m, rank, size, group)
            n += 1
    return n


class _FusedQWeight:
    """A quantized GEMM weight of an injected layer: ``ops.linear`` calls ``.linear(x, bias)`` for
    non-tensor weights; int8 / int4 groups are dequantized right before the GEMM
    (inference/quantization.py)."""

    def __init__(self, w, cfg):
        from ..inference.quantization import _QuantizedWeight
        self.qw = _QuantizedWeight(w.detach(), **cfg)
        self.shape, self.dtype = tuple(w.shape), w.dtype

    @property
    def q(self):
        return self.qw.q

    def to(self, device):
        self.qw.to(device)
        return self

    def linear(self, x, bias=None):
        return F.linear(x, self.qw.dequantize().to(x.dtype), bias)

    def nbytes(self):
        return self.qw.nbytes()


def quantize_fused_layer(layer, cfg):
    """Store every GEMM weight of an injected layer group-quantized (``cfg``: num_bits, group_size,
    group_dim, symmetric -- the weight_quantization.post_init_quant entry). Returns the count."""
    spec = TP_SPECS.get(type(layer))
    if spec is None:
        return 0
    names = [spec["qkv"][0]] + [w for w, _ in spec["col"]] + list(spec["gu"]) + [w for w, _ in spec["row"]]
    c = dict(cfg)
    c.setdefault("num_bits", 8)
    c.setdefault("group_size", 64)
    c.setdefault("group_dim", 1)
    c.setdefault("symmetric", False)
    qs = layer.__dict__.setdefault("_qweights", {})
    n = 0
    for name in names:
        w = layer._parameters.get(name)
        if w is None or w.shape[c["group_dim"]] % int(c["group_size"]):
            continue
        q = _FusedQWeight(w, c)
        del layer._parameters[name]
        layer.__dict__[name] = q
        qs[name] = q.qw
        n += 1
    if n:
        layer._unlink_orig()
    return n
