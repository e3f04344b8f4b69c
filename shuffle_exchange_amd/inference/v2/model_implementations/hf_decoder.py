"""Ragged decoder for Hugging Face checkpoints of the families the reference's FastGen serves.

Parity: reference inference/v2/model_implementations/{llama_v2, mistral, mixtral, opt, falcon, phi,
phi3, qwen, qwen_v2, qwen_v2_moe}/ (``container.py`` = checkpoint-name -> parameter mapping,
``model.py`` = ``_forward_embed`` / ``_forward_transformer_layer`` / ``_forward_unembed``) and
engine_factory.py:69-133 (``build_hf_engine``: pick the implementation from ``config.model_type``).

MI355X-first structure: ONE decoder whose per-family differences are data (``DecoderSpec``), not
ten model classes. Every family is converted at load time into the same packed layout the gfx950
kernels want:
  * q/k/v (whatever the checkpoint's layout: separate, fused, Falcon's per-group interleave) ->
    one [(nq + 2 nkv) * D, H] QKV weight, so the projection is one hipBLASLt GEMM and RoPE +
    KV-cache append read the head-packed output in place;
  * gate/up (separate or fused) -> one [2 I, H] weight consumed by the gated-activation kernel;
  * MoE experts (per-expert tensors or stacked) -> [E, 2I, H] / [E, H, I] stacks; routing is
    dropless (argsort grouping, one GEMM pair per expert with rows);
  * residual adds are fused into the next norm (pre-RMS / pre-LN kernels with residual).
Layout families: sequential pre-norm (Llama, Mistral, Qwen2, Qwen2-MoE, Mixtral, Phi-3, OPT) and
parallel attention+MLP residual (Phi, Falcon; Falcon-40B style with two input norms).
Partial rotary (Phi), learned positions (OPT), sliding windows (Mistral/Qwen2), QKV biases (Qwen2,
Phi, OPT, Falcon), shared experts (Qwen2-MoE) and Llama-3.1 rope scaling are supported.
"""
import glob
import json
import math
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F

from ....ops import native
from ....ops.activation import ACT, bias_act, gated_act
from ....ops.linear import linear
from ....ops.norm import layer_norm, rms_norm
from ....ops.paged_attention import kv_cache_append, paged_attention
from ....ops.rope import RopeCache, apply_rope_tokens_
from ....ops.rows import embed, gather_last

FLASH_PREFILL_MIN = 128


@dataclass
class DecoderSpec:
    family: str
    vocab_size: int
    hidden: int
    n_layers: int
    nq: int
    nkv: int
    head_dim: int
    intermediate: int
    norm: str = "rms"               # rms | ln
    norm_eps: float = 1e-6
    act: str = "silu"
    gated: bool = True
    parallel_residual: bool = False
    two_norms: bool = False         # parallel residual with separate attention / MLP input norms
    rope_theta: float = 10000.0
    rotary_dim: int = 0             # 0: no RoPE (learned positions)
    rope_scaling: Optional[dict] = None
    learned_pos: bool = False
    pos_offset: int = 0
    max_positions: int = 8192
    sliding_window: Optional[int] = None
    tie_embeddings: bool = False
    num_experts: int = 0
    top_k: int = 0
    norm_topk: bool = True
    moe_intermediate: int = 0
    shared_intermediate: int = 0
    dense_layers: tuple = ()        # Qwen2-MoE mlp_only_layers / decoder_sparse_step


# ------------------------------------------------------------------------------------- config
def _rope_params(c):
    rp = dict(c.get("rope_parameters") or {})
    if "rope_theta" not in rp:
        rp["rope_theta"] = c.get("rope_theta", 10000.0)
    rs = c.get("rope_scaling") or {}
    for k, v in rs.items():
        rp.setdefault(k, v)
    if "type" in rp and "rope_type" not in rp:
        rp["rope_type"] = rp["type"]
    if "partial_rotary_factor" not in rp and c.get("partial_rotary_factor") is not None:
        rp["partial_rotary_factor"] = c["partial_rotary_factor"]
    return rp


def spec_from_hf_config(c):
    """HF ``config.json`` dict -> DecoderSpec (reference engine_factory.py:69-133 dispatch)."""
    mt = c["model_type"]
    rp = _rope_params(c)
    theta = float(rp.get("rope_theta", 10000.0))
    rtype = rp.get("rope_type", "default")
    scaling = None if rtype in (None, "default") else rp
    nq = c.get("num_attention_heads")
    H = c.get("hidden_size")
    common = dict(vocab_size=c["vocab_size"], hidden=H, n_layers=c["num_hidden_layers"], nq=nq,
                  max_positions=c.get("max_position_embeddings", 8192), rope_theta=theta, rope_scaling=scaling,
                  tie_embeddings=bool(c.get("tie_word_embeddings", False)))
    if mt in ("llama", "mistral", "qwen2", "mixtral", "qwen2_moe", "phi3"):
        nkv = c.get("num_key_value_heads") or nq
        D = c.get("head_dim") or H // nq
        sw = c.get("sliding_window")
        if mt == "qwen2" or mt == "qwen2_moe":
            sw = sw if c.get("use_sliding_window") else None
        s = DecoderSpec(family=mt, nkv=nkv, head_dim=D, intermediate=c.get("intermediate_size", 0),
                        norm="rms", norm_eps=c.get("rms_norm_eps", 1e-6), act=c.get("hidden_act", "silu"),
                        gated=True, rotary_dim=int(D * rp.get("partial_rotary_factor", 1.0)),
                        sliding_window=sw or None, **common)
        if mt == "phi3" and rtype not in (None, "default"):
            raise NotImplementedError(f"phi3 rope_type={rtype} (longrope/su) is not supported")
        if mt == "mixtral":
            s.num_experts, s.top_k, s.norm_topk = c["num_local_experts"], c["num_experts_per_tok"], True
            s.moe_intermediate = c["intermediate_size"]
        if mt == "qwen2_moe":
            s.num_experts, s.top_k = c["num_experts"], c["num_experts_per_tok"]
            s.norm_topk = bool(c.get("norm_topk_prob", False))
            s.moe_intermediate = c["moe_intermediate_size"]
            s.shared_intermediate = c.get("shared_expert_intermediate_size", 0) or 0
            step = c.get("decoder_sparse_step", 1) or 1
            only = set(c.get("mlp_only_layers", []) or [])
            s.dense_layers = tuple(i for i in range(s.n_layers) if i in only or (i + 1) % step != 0)
        return s
    if mt == "phi":
        D = H // nq
        if c.get("qk_layernorm"):
            raise NotImplementedError("phi qk_layernorm is not supported")
        return DecoderSpec(family=mt, nkv=c.get("num_key_value_heads") or nq, head_dim=D,
                           intermediate=c["intermediate_size"], norm="ln", norm_eps=c.get("layer_norm_eps", 1e-5),
                           act=c.get("hidden_act", "gelu_new"), gated=False, parallel_residual=True,
                           rotary_dim=int(D * rp.get("partial_rotary_factor", 0.5)), **common)
    if mt == "falcon":
        if c.get("alibi"):
            raise NotImplementedError("falcon alibi is not supported")
        new = bool(c.get("new_decoder_architecture", False))
        mq = bool(c.get("multi_query", True))
        nkv = c.get("num_kv_heads") if new else (1 if mq else nq)
        D = H // nq
        n_ln = c.get("num_ln_in_parallel_attn") or (2 if new else 1)
        parallel = bool(c.get("parallel_attn", True)) or new
        common["tie_embeddings"] = bool(c.get("tie_word_embeddings", True))
        return DecoderSpec(family=mt, nkv=nkv, head_dim=D, intermediate=c.get("ffn_hidden_size") or 4 * H,
                           norm="ln", norm_eps=c.get("layer_norm_epsilon", 1e-5), act="gelu_exact", gated=False,
                           parallel_residual=parallel, two_norms=parallel and n_ln == 2, rotary_dim=D, **common)
    if mt == "opt":
        if not c.get("do_layer_norm_before", True):
            raise NotImplementedError("OPT post-LN variant (opt-350m) is not supported")
        if c.get("word_embed_proj_dim", H) != H:
            raise NotImplementedError("OPT word_embed_proj_dim != hidden_size is not supported")
        common["tie_embeddings"] = bool(c.get("tie_word_embeddings", True))
        return DecoderSpec(family=mt, nkv=nq, head_dim=H // nq, intermediate=c["ffn_dim"], norm="ln", norm_eps=1e-5,
                           act=c.get("activation_function", "relu"), gated=False, rotary_dim=0, learned_pos=True,
                           pos_offset=2, **common)
    raise NotImplementedError(f"no ragged implementation for model_type={mt!r}")


def _llama3_scaling(rp):
    factor = rp.get("factor", 8.0)
    lo, hi = rp.get("low_freq_factor", 1.0), rp.get("high_freq_factor", 4.0)
    old = rp.get("original_max_position_embeddings", 8192)

    def f(inv):
        wl = 2 * math.pi / inv
        lo_wl, hi_wl = old / lo, old / hi
        out = torch.where(wl > lo_wl, inv / factor, inv)
        smooth = (old / wl - lo) / (hi - lo)
        sm = (1 - smooth) * out / factor + smooth * out
        med = ~(wl < hi_wl) & ~(wl > lo_wl)
        return torch.where(med, sm, out)
    return f


def _rope_cache(spec, device):
    sc = spec.rope_scaling
    fn = None
    if sc:
        t = sc.get("rope_type")
        if t == "llama3":
            fn = _llama3_scaling(sc)
        elif t == "linear":
            fn = (lambda inv, k=float(sc["factor"]): inv / k)
        else:
            raise NotImplementedError(f"rope_type={t!r}")
    return RopeCache(spec.rotary_dim, spec.max_positions, spec.rope_theta, device, scaling=fn)


# ------------------------------------------------------------------------------------ weights
def _load_state_dict(path):
    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    sd = {}
    if files:
        from safetensors.torch import load_file
        for f in files:
            sd.update(load_file(f))
        return sd
    for f in sorted(glob.glob(os.path.join(path, "pytorch_model*.bin"))):
        sd.update(torch.load(f, map_location="cpu", weights_only=True))
    if not sd:
        raise FileNotFoundError(f"no *.safetensors / pytorch_model*.bin under {path}")
    return sd


class _SD:
    """State-dict accessor with prefix fallbacks."""

    def __init__(self, sd):
        self.sd = sd

    def get(self, *names, required=True):
        for n in names:
            if n in self.sd:
                return self.sd[n]
        if required:
            raise KeyError(f"missing checkpoint tensor: one of {names}")
        return None


def _falcon_qkv(w, spec, new_arch):
    """Falcon fused QKV rows -> [all q | all k | all v] rows."""
    nq, nkv, D = spec.nq, spec.nkv, spec.head_dim
    if new_arch:
        G = nq // nkv
        x = w.view(nkv, G + 2, D, *w.shape[1:])
        q = x[:, :G].reshape(nq * D, *w.shape[1:])
        k = x[:, G].reshape(nkv * D, *w.shape[1:])
        v = x[:, G + 1].reshape(nkv * D, *w.shape[1:])
        return torch.cat([q, k, v])
    if nkv == 1:
        return w  # multi-query: already [nq q heads | k | v]
    x = w.view(nq, 3, D, *w.shape[1:])
    return torch.cat([x[:, 0].reshape(nq * D, *w.shape[1:]), x[:, 1].reshape(nq * D, *w.shape[1:]),
                      x[:, 2].reshape(nq * D, *w.shape[1:])])


def convert_hf_weights(spec, sd, hf_cfg=None):
    """Checkpoint tensors -> packed per-layer dicts (reference container.py mappings)."""
    S = _SD(sd)
    fam = spec.family
    W = {"layers": []}
    if fam == "falcon":
        lp = "transformer.h.{}."
        W["embed"] = S.get("transformer.word_embeddings.weight")
        W["final_w"], W["final_b"] = S.get("transformer.ln_f.weight"), S.get("transformer.ln_f.bias")
    elif fam == "opt":
        lp = "model.decoder.layers.{}."
        W["embed"] = S.get("model.decoder.embed_tokens.weight", "decoder.embed_tokens.weight")
        W["pos_embed"] = S.get("model.decoder.embed_positions.weight", "decoder.embed_positions.weight")
        W["final_w"] = S.get("model.decoder.final_layer_norm.weight", "decoder.final_layer_norm.weight")
        W["final_b"] = S.get("model.decoder.final_layer_norm.bias", "decoder.final_layer_norm.bias")
    else:
        lp = "model.layers.{}."
        W["embed"] = S.get("model.embed_tokens.weight")
        if fam == "phi":
            W["final_w"], W["final_b"] = S.get("model.final_layernorm.weight"), S.get("model.final_layernorm.bias")
        else:
            W["final_w"] = S.get("model.norm.weight")
    lm = S.get("lm_head.weight", required=False)
    W["lm_head"] = lm if lm is not None else W["embed"]
    W["lm_head_b"] = S.get("lm_head.bias", required=False)
    new_falcon = bool((hf_cfg or {}).get("new_decoder_architecture", False))
    for i in range(spec.n_layers):
        p = lp.format(i)
        L = {}
        g = (lambda *n, required=True: S.get(*[p + x for x in n], required=required))
        # ---- norms
        if fam == "falcon":
            if spec.two_norms:
                L["ln1_w"], L["ln1_b"] = g("ln_attn.weight"), g("ln_attn.bias")
                L["ln2_w"], L["ln2_b"] = g("ln_mlp.weight"), g("ln_mlp.bias")
            else:
                L["ln1_w"], L["ln1_b"] = g("input_layernorm.weight"), g("input_layernorm.bias")
                if not spec.parallel_residual:
                    L["ln2_w"], L["ln2_b"] = g("post_attention_layernorm.weight"), g("post_attention_layernorm.bias")
        elif fam == "opt":
            L["ln1_w"], L["ln1_b"] = g("self_attn_layer_norm.weight"), g("self_attn_layer_norm.bias")
            L["ln2_w"], L["ln2_b"] = g("final_layer_norm.weight"), g("final_layer_norm.bias")
        elif fam == "phi":
            L["ln1_w"], L["ln1_b"] = g("input_layernorm.weight"), g("input_layernorm.bias")
        else:
            L["ln1_w"], L["ln2_w"] = g("input_layernorm.weight"), g("post_attention_layernorm.weight")
        # ---- attention
        if fam == "falcon":
            L["qkv_w"] = _falcon_qkv(g("self_attention.query_key_value.weight"), spec, new_falcon)
            b = g("self_attention.query_key_value.bias", required=False)
            L["qkv_b"] = _falcon_qkv(b, spec, new_falcon) if b is not None else None
            L["o_w"], L["o_b"] = g("self_attention.dense.weight"), g("self_attention.dense.bias", required=False)
        elif fam == "phi3":
            L["qkv_w"] = g("self_attn.qkv_proj.weight")
            L["qkv_b"] = None
            L["o_w"], L["o_b"] = g("self_attn.o_proj.weight"), None
        else:
            L["qkv_w"] = torch.cat([g("self_attn.q_proj.weight"), g("self_attn.k_proj.weight"),
                                    g("self_attn.v_proj.weight")])
            qb = g("self_attn.q_proj.bias", required=False)
            L["qkv_b"] = torch.cat([qb, g("self_attn.k_proj.bias"), g("self_attn.v_proj.bias")]) if qb is not None else None
            o = "self_attn.dense" if fam == "phi" else ("self_attn.out_proj" if fam == "opt" else "self_attn.o_proj")
            L["o_w"], L["o_b"] = g(o + ".weight"), g(o + ".bias", required=False)
        # ---- MLP / MoE
        moe_layer = spec.num_experts > 0 and i not in spec.dense_layers
        if moe_layer:
            m = "mlp." if g("mlp.gate.weight", required=False) is not None else "block_sparse_moe."
            L["router"] = g(m + "gate.weight")
            gu = g(m + "experts.gate_up_proj", required=False)
            if gu is not None:
                L["e_gu"], L["e_down"] = gu, g(m + "experts.down_proj")
            else:
                gus, downs = [], []
                for e in range(spec.num_experts):
                    ep = m + f"experts.{e}."
                    if g(ep + "w1.weight", required=False) is not None:  # Mixtral: w1 gate, w3 up, w2 down
                        gus.append(torch.cat([g(ep + "w1.weight"), g(ep + "w3.weight")]))
                        downs.append(g(ep + "w2.weight"))
                    else:
                        gus.append(torch.cat([g(ep + "gate_proj.weight"), g(ep + "up_proj.weight")]))
                        downs.append(g(ep + "down_proj.weight"))
                L["e_gu"], L["e_down"] = torch.stack(gus), torch.stack(downs)
            if spec.shared_intermediate:
                L["sh_gu"] = torch.cat([g(m + "shared_expert.gate_proj.weight"), g(m + "shared_expert.up_proj.weight")])
                L["sh_down"] = g(m + "shared_expert.down_proj.weight")
                L["sh_gate"] = g(m + "shared_expert_gate.weight")
        elif spec.gated:
            fused = g("mlp.gate_up_proj.weight", required=False)
            L["gu_w"] = fused if fused is not None else torch.cat([g("mlp.gate_proj.weight"), g("mlp.up_proj.weight")])
            L["down_w"] = g("mlp.down_proj.weight")
        else:
            if fam == "falcon":
                n1, n2 = "mlp.dense_h_to_4h", "mlp.dense_4h_to_h"
            elif fam == "opt":
                n1, n2 = "fc1", "fc2"
            else:
                n1, n2 = "mlp.fc1", "mlp.fc2"
            L["fc1_w"], L["fc1_b"] = g(n1 + ".weight"), g(n1 + ".bias", required=False)
            L["fc2_w"], L["fc2_b"] = g(n2 + ".weight"), g(n2 + ".bias", required=False)
        W["layers"].append(L)
    return W


# ---------------------------------------------------------------------------- shared attention
def ragged_attention(qkv, kv_layer, batch, nq, nkv, D, scale, window=None):
    """Attention of a ragged batch's new tokens over their paged KV: pure prefills of >= 128 tokens
    run the training flash kernel (MFMA, causal), the rest the paged-attention kernel."""
    q = qkv[:, :nq]
    use_flash = (native.use_hip(qkv) and D == 128 and qkv.dtype == torch.bfloat16 and
                 (window is None or batch.max_kv_len <= window))
    flash_ids = [i for i in range(batch.num_seqs)
                 if use_flash and batch.host_seen[i] == 0 and batch.host_q_len[i] >= FLASH_PREFILL_MIN] \
        if use_flash else []
    if not flash_ids:
        return paged_attention(q, kv_layer, batch.block_table, batch.q_start, batch.q_len, batch.kv_len, scale,
                               batch.max_kv_len, window=window)
    out = torch.empty(qkv.shape[0], nq, D, dtype=qkv.dtype, device=qkv.device)
    fset = set(flash_ids)
    rest = [i for i in range(batch.num_seqs) if i not in fset]
    for i in flash_ids:
        s, n = batch.host_q_start[i], batch.host_q_len[i]
        pad = (-n) % 128
        x = qkv[s:s + n]
        if pad:
            x = torch.cat([x, x.new_zeros(pad, *x.shape[1:])])
        x = x.unsqueeze(0)
        o, _ = torch.ops.sxe.flash_attn_fwd(x[:, :, :nq], x[:, :, nq:nq + nkv], x[:, :, nq + nkv:], True, float(scale))
        out[s:s + n] = o[0, :n]
    if rest:
        idx = torch.tensor(rest, device=qkv.device)
        o = paged_attention(q, kv_layer, batch.block_table.index_select(0, idx).contiguous(),
                            batch.q_start.index_select(0, idx).contiguous(),
                            batch.q_len.index_select(0, idx).contiguous(),
                            batch.kv_len.index_select(0, idx).contiguous(), scale,
                            max(batch.host_kv_len[i] for i in rest), window=window)
        for i in rest:
            s, n = batch.host_q_start[i], batch.host_q_len[i]
            out[s:s + n] = o[s:s + n]
    return out


# Measured on MI355X (tools/grouped_gemm_bench.py, profiles/grouped_gemm_bench.log): the grouped
# kernel wins with many experts / few rows each (Qwen-MoE 60 experts x 273 rows: 0.47 vs 1.33 ms;
# Mixtral decode 16 rows/expert: 0.39 vs 0.50 ms) and loses to per-expert hipBLASLt at 1024 rows
# per expert (Mixtral prefill gate_up: 3.99 vs 1.77 ms).
GROUPED_MAX_ROWS_PER_EXPERT = 512


def dropless_moe(x, router_w, e_gu, e_down, top_k, norm_topk, act="silu"):
    """Exact top-k routing (no capacity): group rows by expert with one argsort, one GEMM pair per
    expert that received rows, weighted scatter-add back (reference ragged_ops top_k_gating +
    moe_scatter + moe_gather)."""
    probs = torch.softmax(F.linear(x.float(), router_w.float()), dim=-1)
    topw, topi = probs.topk(top_k, dim=-1)
    if norm_topk:
        topw = topw / topw.sum(-1, keepdim=True)
    flat = topi.reshape(-1)
    order = torch.argsort(flat, stable=True)
    tok = order // top_k
    from ....ops.moe import QuantizedExperts, expert_offsets, grouped_gemm, grouped_gemm_ok, grouped_gemm_q
    E = e_gu.shape[0]
    if isinstance(e_gu, QuantizedExperts):
        # int8 / int4 experts (weight_quant='int8' | 'int4'): the mixed-precision grouped kernel
        # streams the codes and widens them per staged K block (reference mixed_moe_gemm)
        offs = expert_offsets(flat, E)
        xs = x.index_select(0, tok)
        ws = topw.reshape(-1).index_select(0, order).float()
        h = gated_act(grouped_gemm_q(xs, e_gu, offs), act)
        return torch.zeros_like(x).index_add_(0, tok, grouped_gemm_q(h, e_down, offs, ws).to(x.dtype))
    if (grouped_gemm_ok(x, e_gu) and grouped_gemm_ok(x, e_down.transpose(1, 2))
            and flat.numel() <= GROUPED_MAX_ROWS_PER_EXPERT * E):
        # one ragged grouped-GEMM launch per projection (grouped_gemm.hip), routing weight fused
        # into the down projection's epilogue, offsets kept on the device: no host sync. Large
        # per-expert row counts keep hipBLASLt's per-expert GEMMs (faster there; see below).
        offs = expert_offsets(flat, E)
        xs = x.index_select(0, tok)
        ws = topw.reshape(-1).index_select(0, order).float()
        h = gated_act(grouped_gemm(xs, e_gu, offs), act)
        return torch.zeros_like(x).index_add_(0, tok, grouped_gemm(h, e_down, offs, ws))
    counts = torch.bincount(flat, minlength=e_gu.shape[0]).tolist()
    xs = x.index_select(0, tok)
    ws = topw.reshape(-1).index_select(0, order).to(x.dtype).unsqueeze(1)
    out = torch.zeros_like(x)
    o = 0
    for e, c in enumerate(counts):
        if c == 0:
            continue
        h = gated_act(linear(xs[o:o + c], e_gu[e]), act)
        out.index_add_(0, tok[o:o + c], linear(h, e_down[e]) * ws[o:o + c])
        o += c
    return out


# ------------------------------------------------------------------------ tensor parallelism
def shard_decoder_weights(spec, W, t, r):
    """This TP rank's share of converted weights (reference inference/v2/model_implementations/
    sharding/{qkv,attn_out,mlp,moe,unembed}.py): q heads and their kv heads (kv heads replicated
    when t exceeds their count), o_proj / down / fc2 input columns (row-parallel: partial sums,
    biases added once after the all-reduce), gate|up / fc1 output rows, every expert's FFN
    columns (expert TP: routing stays replicated), vocab rows of the LM head (padded to an equal
    split; logits are all-gathered). Returns (weights, local q heads, local kv heads)."""
    nq, nkv, D = spec.nq, spec.nkv, spec.head_dim
    assert nq % t == 0, f"query heads ({nq}) must divide by tp_size ({t})"
    assert nkv % t == 0 or t % nkv == 0, f"kv heads ({nkv}) and tp_size ({t}) must divide one another"
    lq, q0 = nq // t, r * (nq // t)
    if nkv % t == 0:
        lkv, kv0 = nkv // t, r * (nkv // t)
    else:  # fewer kv heads than ranks: each rank keeps the kv head its q heads attend to
        lkv, kv0 = 1, q0 // (nq // nkv)

    def qkv(w):
        return torch.cat([w[q0 * D:(q0 + lq) * D], w[(nq + kv0) * D:(nq + kv0 + lkv) * D],
                          w[(nq + nkv + kv0) * D:(nq + nkv + kv0 + lkv) * D]]).contiguous()

    def part(n):
        assert n % t == 0, f"FFN width {n} must divide by tp_size {t}"
        return r * (n // t), n // t

    def gate_up(w, dim):  # [gate | up] halves along `dim`: this rank's slice of each
        n = w.shape[dim] // 2
        a, c = part(n)
        return torch.cat([w.narrow(dim, a, c), w.narrow(dim, n + a, c)], dim).contiguous()

    out = {k: v for k, v in W.items() if k != "layers"}
    out["layers"] = []
    for L in W["layers"]:
        M = dict(L)
        M["qkv_w"] = qkv(L["qkv_w"])
        if L.get("qkv_b") is not None:
            M["qkv_b"] = qkv(L["qkv_b"])
        M["o_w"] = L["o_w"][:, q0 * D:(q0 + lq) * D].contiguous()
        if "gu_w" in L:
            M["gu_w"] = gate_up(L["gu_w"], 0)
            a, c = part(L["down_w"].shape[1])
            M["down_w"] = L["down_w"][:, a:a + c].contiguous()
        if "fc1_w" in L:
            a, c = part(L["fc1_w"].shape[0])
            M["fc1_w"] = L["fc1_w"][a:a + c].contiguous()
            if L.get("fc1_b") is not None:
                M["fc1_b"] = L["fc1_b"][a:a + c].contiguous()
            M["fc2_w"] = L["fc2_w"][:, a:a + c].contiguous()
        if "e_gu" in L:
            M["e_gu"] = gate_up(L["e_gu"], 1)
            a, c = part(L["e_down"].shape[2])
            M["e_down"] = L["e_down"][:, :, a:a + c].contiguous()
        if "sh_gu" in L:
            M["sh_gu"] = gate_up(L["sh_gu"], 0)
            a, c = part(L["sh_down"].shape[1])
            M["sh_down"] = L["sh_down"][:, a:a + c].contiguous()
        out["layers"].append(M)
    V = W["lm_head"].shape[0]
    vs = -(-V // t)
    lo, hi = min(r * vs, V), min((r + 1) * vs, V)

    def vrows(w):
        w = w[lo:hi]
        if hi - lo < vs:  # pad the last shard: every rank gathers the same size
            w = torch.cat([w, w.new_zeros(vs - (hi - lo), *w.shape[1:])])
        return w.contiguous()
    out["lm_head"] = vrows(W["lm_head"])
    if W.get("lm_head_b") is not None:
        out["lm_head_b"] = vrows(W["lm_head_b"])
    return out, lq, lkv


# --------------------------------------------------------------------------------- the decoder
class RaggedDecoder:
    """Engine-facing model (InferenceEngineV2 protocol: num_layers / nkv / head_dim / dtype /
    device / vocab_size / forward(batch, kv_cache) -> last-token fp32 logits)."""

    QUANT_KEYS = ("qkv_w", "o_w", "gu_w", "down_w", "fc1_w", "fc2_w", "sh_gu", "sh_down")

    def __init__(self, spec: DecoderSpec, weights, dtype=torch.bfloat16, device=None, weight_quant=None,
                 tp_group=None, tp_size=1):
        self.spec = spec
        device = torch.device(device) if device is not None else torch.device("cpu")
        from .... import comm as dist
        self.tp, self.tp_group = int(tp_size), tp_group  # tp_group None with tp_size > 1: the world
        self.tp_rank = dist.get_rank(tp_group) if self.tp > 1 else 0
        self.nq, self.nkv = spec.nq, spec.nkv
        if self.tp > 1:
            assert dist.get_world_size(tp_group) == self.tp, "tp_group size != tp_size"
            weights, self.nq, self.nkv = shard_decoder_weights(spec, weights, self.tp, self.tp_rank)

        def mv(t):
            return t.to(device=device, dtype=dtype).contiguous() if torch.is_tensor(t) else t
        self.w = {k: mv(v) for k, v in weights.items() if k != "layers"}
        self.w["layers"] = [{k: mv(v) for k, v in L.items()} for L in weights["layers"]]
        if weight_quant:
            # weight-only FP8 (row-scaled e4m3) projections and LM head: decode GEMMs stream half
            # the bytes through the skinny MFMA kernel (reference: FP6-LLM QuantizedWf6Af16Linear)
            from ....ops.fp_quantizer import quantized_weight
            for L in self.w["layers"]:
                for k in self.QUANT_KEYS:
                    if torch.is_tensor(L.get(k)) and L[k].dim() == 2:
                        L[k] = quantized_weight(L[k], weight_quant)
            self.w["lm_head"] = quantized_weight(self.w["lm_head"], weight_quant)
            if weight_quant in ("int8", "int4"):
                from ....ops.moe import QuantizedExperts
                for L in self.w["layers"]:
                    for k in ("e_gu", "e_down"):
                        if torch.is_tensor(L.get(k)):
                            L[k] = QuantizedExperts(L[k], 8 if weight_quant == "int8" else 4)
        self.weight_quant = weight_quant
        self.num_layers, self.head_dim = spec.n_layers, spec.head_dim
        self.vocab_size = spec.vocab_size
        self._dtype, self._device = dtype, device
        self.rope = _rope_cache(spec, device) if spec.rotary_dim else None
        self.scale = spec.head_dim ** -0.5
        self.model = self  # InferenceEngineV2.serialize() reads .model.state_dict()

    @property
    def device(self):
        return self._device

    @property
    def dtype(self):
        return self._dtype

    def state_dict(self):
        sd = {k: v for k, v in self.w.items() if torch.is_tensor(v)}
        for i, L in enumerate(self.w["layers"]):
            sd.update({f"layers.{i}.{k}": v for k, v in L.items() if torch.is_tensor(v)})
        return sd

    # -- blocks
    def _norm(self, x, w, b, residual=None):
        if self.spec.norm == "rms":
            return rms_norm(x, w, self.spec.norm_eps, residual=residual)
        return layer_norm(x, w, b, self.spec.norm_eps, residual=residual)

    def _reduce(self, y, *biases):
        """Row-parallel epilogue: sum the TP ranks' partial products over xGMI, then add the
        (replicated) output biases once."""
        if self.tp > 1:
            from .... import comm as dist
            y = y.contiguous()
            dist.all_reduce(y, group=self.tp_group)
        for b in biases:
            if b is not None:
                y = y + b
        return y

    def _attn(self, a, L, li, batch, kv_cache, reduce=True):
        s, T = self.spec, a.shape[0]
        nq, nkv, D = self.nq, self.nkv, s.head_dim
        qkv = linear(a, L["qkv_w"], L.get("qkv_b")).view(T, nq + 2 * nkv, D)
        if self.rope is not None:
            apply_rope_tokens_(qkv, self.rope, nq + nkv, batch.positions, rot_dim=s.rotary_dim)
        kv_layer = kv_cache.layer(li)
        kv_cache_append(qkv, kv_layer, batch.slots, nq, nkv)
        o = ragged_attention(qkv, kv_layer, batch, nq, nkv, D, self.scale, s.sliding_window)
        if self.tp == 1:
            return linear(o.reshape(T, nq * D), L["o_w"], L.get("o_b"))
        y = linear(o.reshape(T, nq * D), L["o_w"])
        return self._reduce(y, L.get("o_b")) if reduce else y

    def _mlp(self, m, L, reduce=True):
        if self.tp > 1:  # partial sums of this rank's FFN / expert columns
            y = self._mlp_partial(m, L)
            return self._reduce(y, L.get("fc2_b")) if reduce else y
        return self._mlp_partial(m, L, L.get("fc2_b"))

    def _mlp_partial(self, m, L, fc2_b=None):
        s = self.spec
        if "router" in L:
            out = dropless_moe(m, L["router"], L["e_gu"], L["e_down"], s.top_k, s.norm_topk, s.act)
            if "sh_gu" in L:
                sh = linear(gated_act(linear(m, L["sh_gu"]), s.act), L["sh_down"])
                out = out + torch.sigmoid(linear(m, L["sh_gate"])) * sh
            return out
        if "gu_w" in L:
            return linear(gated_act(linear(m, L["gu_w"]), s.act), L["down_w"])
        h = bias_act(linear(m, L["fc1_w"]), L.get("fc1_b"), ACT[s.act])
        return linear(h, L["fc2_w"], fc2_b)

    @torch.no_grad()
    def forward(self, batch, kv_cache):
        s, W = self.spec, self.w
        if self.rope is not None and batch.max_kv_len > self.rope.max_pos:  # HIP RoPE indexes the table unchecked
            raise ValueError(f"sequence length {batch.max_kv_len} exceeds the RoPE table ({self.rope.max_pos} positions)")
        x = embed(W["embed"], batch.input_ids)
        if s.learned_pos:
            x = x + embed(W["pos_embed"], batch.positions, -s.pos_offset)
        res = None  # pending residual: the true hidden state is x + res
        for li, L in enumerate(W["layers"]):
            if s.parallel_residual:
                h = x if res is None else x + res
                a = self._norm(h, L["ln1_w"], L.get("ln1_b"))
                m = self._norm(h, L["ln2_w"], L.get("ln2_b")) if s.two_norms else a
                if self.tp > 1:  # attention and MLP partials share ONE all-reduce
                    y = self._attn(a, L, li, batch, kv_cache, reduce=False) + self._mlp(m, L, reduce=False)
                    x, res = self._reduce(y, L.get("o_b"), L.get("fc2_b")), h
                else:
                    x, res = self._attn(a, L, li, batch, kv_cache) + self._mlp(m, L), h
            else:
                a, h = (self._norm(x, L["ln1_w"], L.get("ln1_b")), x) if res is None else \
                    self._norm(x, L["ln1_w"], L.get("ln1_b"), residual=res)
                attn = self._attn(a, L, li, batch, kv_cache)
                m, h2 = self._norm(attn, L["ln2_w"], L.get("ln2_b"), residual=h)
                x, res = self._mlp(m, L), h2
        last = batch.last_idx
        h = gather_last(x, last, res)  # one HIP gather with the residual add fused
        h = self._norm(h, W["final_w"], W.get("final_b"))
        logits = linear(h, W["lm_head"], W.get("lm_head_b")).float()
        if self.tp > 1:  # vocab-parallel head: gather every rank's logit columns
            from .... import comm as dist
            full = torch.empty(self.tp * logits.shape[0], logits.shape[1], dtype=logits.dtype, device=logits.device)
            dist.all_gather_into_tensor(full, logits.contiguous(), group=self.tp_group)
            logits = full.view(self.tp, -1, logits.shape[1]).permute(1, 0, 2).reshape(logits.shape[0], -1)
            logits = logits[:, :self.vocab_size]
        return logits


def load_hf_decoder(model_or_path, dtype=torch.bfloat16, device=None, weight_quant=None, tp_group=None, tp_size=1):
    """A transformers model instance or a local checkpoint directory (config.json + safetensors /
    pytorch_model*.bin, loaded without executing pickled code) -> RaggedDecoder (this rank's
    tensor-parallel shard when ``tp_size > 1``)."""
    if isinstance(model_or_path, (str, os.PathLike)):
        with open(os.path.join(model_or_path, "config.json")) as f:
            cfg = json.load(f)
        sd = _load_state_dict(model_or_path)
    else:
        cfg = model_or_path.config.to_dict()
        sd = {k: v.detach() for k, v in model_or_path.state_dict().items()}
    spec = spec_from_hf_config(cfg)
    return RaggedDecoder(spec, convert_hf_weights(spec, sd, cfg), dtype=dtype, device=device, weight_quant=weight_quant,
                         tp_group=tp_group, tp_size=tp_size)
