"""Ragged (continuous-batching) forward for the Llama / Mixtral families over a paged KV cache.

Parity: reference inference/v2/model_implementations/llama_v2/model.py and mixtral/model.py
(``_forward_embed`` / ``_forward_transformer_layer`` / ``_forward_unembed``), with the module
choices the reference makes through its registry (blocked KV rotary, blocked flash, pre-RMS norm,
BLAS linear, cutlass MoE GEMM) replaced by this framework's gfx950 kernels:

  * RMSNorm with fused residual add (norm.hip), projections through hipBLASLt,
  * RoPE in place on the packed QKV (rope.hip), KV scatter into the blocked cache and paged
    attention (paged_attn.hip); sequences in pure prefill (no history, >= 128 new tokens) run the
    training flash-attention kernel instead (MFMA, causal; their padding rows are discarded),
  * SwiGLU (act.hip); Mixtral experts via the grouped MoE path of moe/,
  * only the last token of every sequence goes through the final norm + LM head.
The weights are the training modules' own parameters (no copy): a trained LlamaForCausalLM /
MixtralForCausalLM serves directly.

Tensor parallelism (``tp_group`` of size t; reference llama_v2/model.py:156 all-reduce after the
attention output and MLP down projections, :191 all-gather of the vocab-parallel logits): each rank
holds q heads / kv heads / FFN columns / vocab rows of its 1/t share (kv heads replicated when t
exceeds their count), its KV cache holds only its kv heads, and per layer exactly two all-reduces
(o_proj, down_proj) plus one logits all-gather per forward cross xGMI. The embedding and norms stay
replicated. MoE layers shard every expert's FFN columns (routing replicated, one all-reduce after
the experts); ``weight_quant`` quantizes each rank's slices.
"""
import os

import torch
import torch.nn.functional as F

from ....ops import native
from ....ops.activation import swiglu
from ....ops.linear import linear
from ....ops.paged_attention import paged_attention, paged_attention_parts, rope_kv_cache_append
from ....ops.rows import embed, gather_rows

FLASH_PREFILL_MIN = 128


class _TPShards:
    """This rank's slices of every projection (copied once; the full weights can then be freed)."""

    def __init__(self, model, t, r, nq, nkv, D):
        assert nq % t == 0, f"query heads ({nq}) must divide by tp_size ({t})"
        assert nkv % t == 0 or t % nkv == 0, f"kv heads ({nkv}) and tp_size ({t}) must divide one another"
        self.nq = nq // t
        if nkv % t == 0:
            self.nkv, kv0 = nkv // t, r * (nkv // t)
        else:  # fewer kv heads than ranks: each rank keeps the kv head its q heads attend to
            self.nkv, kv0 = 1, (r * nq // t) // (nq // nkv)
        q0 = r * self.nq
        self.layers = []
        for layer in model.layers:
            a = layer.self_attn
            w = a.qkv_proj.weight
            q = w[q0 * D:(q0 + self.nq) * D]
            k = w[(nq + kv0) * D:(nq + kv0 + self.nkv) * D]
            v = w[(nq + nkv + kv0) * D:(nq + nkv + kv0 + self.nkv) * D]
            d = {"qkv": torch.cat([q, k, v]).contiguous(),
                 "o": a.o_proj.weight[:, q0 * D:(q0 + self.nq) * D].contiguous()}
            if hasattr(layer, "mlp"):
                mlp = layer.mlp
                inter = mlp.gate_up_proj.weight.shape[0] // 2
                assert inter % t == 0, f"intermediate size ({inter}) must divide by tp_size ({t})"
                c = inter // t
                gu = mlp.gate_up_proj.weight
                d["gu"] = torch.cat([gu[r * c:(r + 1) * c], gu[inter + r * c:inter + (r + 1) * c]]).contiguous()
                d["down"] = mlp.down_proj.weight[:, r * c:(r + 1) * c].contiguous()
            else:  # MoE: every expert's FFN columns (reference sharding/moe.py); routing replicated
                moe = (layer.block_sparse_moe if hasattr(layer, "block_sparse_moe") else layer.moe).deepspeed_moe
                ex = moe.experts
                inter = ex.w_down.shape[1]
                assert inter % t == 0, f"expert intermediate size ({inter}) must divide by tp_size ({t})"
                c = inter // t
                w = ex.w_gate_up  # [E, H, 2I]: x @ w
                d["e_gu"] = torch.cat([w[..., r * c:(r + 1) * c], w[..., inter + r * c:inter + (r + 1) * c]], -1).contiguous()
                d["e_down"] = ex.w_down[:, r * c:(r + 1) * c].contiguous()
            self.layers.append(d)
        V = model.lm_head.weight.shape[0]
        self.vshard = -(-V // t)
        self.vocab = V
        lo, hi = min(r * self.vshard, V), min((r + 1) * self.vshard, V)
        head = model.lm_head.weight[lo:hi]
        if hi - lo < self.vshard:  # pad the last shard so every rank gathers the same size
            head = torch.cat([head, head.new_zeros(self.vshard - (hi - lo), head.shape[1])])
        self.head = head.contiguous()


class RaggedLlama:
    def __init__(self, model, weight_quant=None, tp_group=None, tp_size=1, pins=None):
        from ..modules import heuristics as H
        self.model = model
        self.qw = None
        from .... import comm as dist
        self.tp_group = tp_group  # None with tp_size > 1: the world group
        self.tp = int(tp_size)
        if self.tp > 1:
            assert dist.get_world_size(tp_group) == self.tp, "tp_group size != tp_size"
        self.tp_rank = dist.get_rank(tp_group) if self.tp > 1 else 0
        p0 = next(model.parameters())
        dev = p0.device.type
        self._weight_quant, self._pins = weight_quant, pins
        if weight_quant and self.tp == 1:
            # linear implementations from the registry (modules/heuristics.py): quantized
            # weight-only GEMMs for decode-sized inputs, the bf16 weight on hipBLASLt otherwise
            self.qw = []
            for layer in model.layers:
                d = {"qkv": self._lin(layer.self_attn.qkv_proj.weight), "o": self._lin(layer.self_attn.o_proj.weight)}
                if hasattr(layer, "mlp"):
                    d["gu"] = self._lin(layer.mlp.gate_up_proj.weight)
                    d["down"] = self._lin(layer.mlp.down_proj.weight)
                self.qw.append(d)
            self.qhead = self._lin(model.lm_head.weight)
        self.cfg = model.cfg
        self.is_moe = hasattr(model.layers[0], "block_sparse_moe") or hasattr(model.layers[0], "moe")
        a0 = model.layers[0].self_attn
        self.nq, self.nkv, self.head_dim = a0.nq, a0.nkv, a0.d
        self.attn_impl = H.instantiate_attention(H.AttentionConfig(self.head_dim, self.nq, self.nkv, p0.dtype, 0, dev),
                                                 pins)
        emb = getattr(model.embed_tokens, "weight", None)
        self.embed_impl = H.instantiate_embed(H.EmbedConfig(emb.shape[0], emb.shape[1], emb.dtype, dev), emb, pins) \
            if emb is not None else None
        self.moe_impl = None
        if self.is_moe:
            l0 = model.layers[0]
            moe = (l0.block_sparse_moe if hasattr(l0, "block_sparse_moe") else l0.moe).deepspeed_moe
            self.moe_impl = H.instantiate_moe(H.MoEConfig(moe.gate.wg.weight.shape[0], moe.gate.k, dev), pins)
        self.implementations = {"attention": self.attn_impl.impl_name,
                                "embed": self.embed_impl.impl_name if self.embed_impl else "module",
                                "linear": self.qhead.impl_name if self.qw is not None else "module",
                                "moe": self.moe_impl.impl_name if self.moe_impl else None}
        self.num_layers = len(model.layers)
        self.vocab_size = self.cfg.vocab_size
        self.tps = None
        if self.tp > 1:
            self._full_heads = (self.nq, self.nkv)
            self._make_shards()
            self.nq, self.nkv = self.tps.nq, self.tps.nkv
            if self.qw is not None:
                self.implementations["linear"] = self.qhead.impl_name

    def _lin(self, w, bias=None):
        from ..modules import heuristics as H
        return H.instantiate_linear(H.LinearConfig(w.shape[1], w.shape[0], w.dtype, self._weight_quant, w.device.type),
                                    w, bias, self._pins)

    def _make_shards(self):
        self.tps = _TPShards(self.model, self.tp, self.tp_rank, *self._full_heads, self.head_dim)
        if self._weight_quant:  # quantize this rank's slices (row scales are per output row)
            self.qw = [{k: self._lin(v) for k, v in d.items() if k in ("qkv", "o", "gu", "down")}
                       for d in self.tps.layers]
            self.qhead = self._lin(self.tps.head)

    def refresh_shards(self):
        """Re-slice the tensor-parallel shards from the (updated) module weights -- the hybrid
        engine calls this before each generation, after training steps changed the weights."""
        if self.tps is not None:
            self._make_shards()

    @property
    def device(self):
        return next(self.model.parameters()).device

    @property
    def dtype(self):
        return next(self.model.parameters()).dtype

    def _attention(self, qkv, kv_layer, batch):
        nq, D = self.nq, self.head_dim
        scale = D ** -0.5
        q = qkv[:, :nq]
        use_flash = native.use_hip(qkv) and self.attn_impl.flash_prefill and D == 128 and qkv.dtype == torch.bfloat16
        flash_ids = [i for i in range(batch.num_seqs)
                     if use_flash and batch.host_seen[i] == 0 and batch.host_q_len[i] >= FLASH_PREFILL_MIN] \
            if use_flash else []
        if not flash_ids:
            return paged_attention(q, kv_layer, batch.block_table, batch.q_start, batch.q_len, batch.kv_len, scale,
                                   batch.max_kv_len)
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
            o, _ = torch.ops.sxe.flash_attn_fwd(x[:, :, :nq], x[:, :, nq:nq + self.nkv], x[:, :, nq + self.nkv:],
                                                True, float(scale))
            out[s:s + n] = o[0, :n]
        if rest:
            idx = torch.tensor(rest, device=qkv.device)
            o = paged_attention(q, kv_layer, batch.block_table.index_select(0, idx).contiguous(),
                                batch.q_start.index_select(0, idx).contiguous(),
                                batch.q_len.index_select(0, idx).contiguous(),
                                batch.kv_len.index_select(0, idx).contiguous(), scale,
                                max(batch.host_kv_len[i] for i in rest))
            for i in rest:
                s, n = batch.host_q_start[i], batch.host_q_len[i]
                out[s:s + n] = o[s:s + n]
        return out

    def _proj(self, mod, x, li, key):
        if self.tps is not None:
            if self.qw is not None:
                y = self.qw[li][key](x)
            else:
                y = linear(x, self.tps.layers[li][key])
            if key in ("o", "down"):  # row-parallel: partial sums over this rank's heads / FFN columns
                from .... import comm as dist
                dist.all_reduce(y, group=self.tp_group)
            return y
        # FP8 weights pay off where the GEMM is weight-streaming bound (<= 16 rows: W8A16 skinny
        # kernel); larger batches keep the module's bf16 weight on hipBLASLt
        if self.qw is not None and key in self.qw[li]:
            return self.qw[li][key](x)
        return mod(x)

    # decode (<= 4 tokens): RMSNorm folded into the QKV / gate_up GEMMs and SwiGLU into the down GEMM
    # (skinny_gemm.hip prologues) -- three latency-bound launches fewer per layer
    FUSE_MAX_T = 4

    def _fusable(self, T):
        return (self.tps is None and T <= self.FUSE_MAX_T and not self.is_moe and self.device.type == "cuda" and native.hip_available()
                and os.environ.get("SXE_DECODE_FUSE", "1") == "1")

    def _attn_o(self, attn, qkv, kv_layer, batch, li, T):
        """Attention + o_proj. Decode: the KV-split merge runs inside the o_proj GEMM launch
        (paged_attention_parts + fused_merge_linear) -- one latency-bound launch fewer per layer."""
        if (self._fusable(T) and getattr(attn.o_proj, "bias", None) is None and native.use_hip(qkv)
                and os.environ.get("SXE_DECODE_FUSE_ATTN", "1") == "1"):
            from ....ops.linear import _pro_weight, fused_merge_linear
            w = self._wobj(attn.o_proj, li, "o")
            if _pro_weight(w) is not None:
                out, parts = paged_attention_parts(qkv[:, :self.nq], kv_layer, batch.block_table, batch.q_start,
                                                   batch.q_len, batch.kv_len, self.head_dim ** -0.5, batch.max_kv_len)
                if parts is not None:
                    y = fused_merge_linear(parts[0], parts[1], w)
                    if y is not None:
                        return y
                    from ....ops.paged_attention import merge_attention_parts
                    out = merge_attention_parts(parts[0], parts[1], qkv.dtype)  # keep the computed splits
                return self._proj(attn.o_proj, out.reshape(T, self.nq * self.head_dim), li, "o")
        o = self._attention(qkv, kv_layer, batch)
        return self._proj(attn.o_proj, o.reshape(T, self.nq * self.head_dim), li, "o")

    def _wobj(self, mod, li, key):
        if self.qw is not None and key in self.qw[li]:
            impl = self.qw[li][key]
            return getattr(impl, "q", None) if getattr(impl, "q", None) is not None else getattr(impl, "weight", None)
        return mod.weight

    def _norm_proj(self, norm, x, res, mod, li, key):
        """(norm(x + res) @ W^T, h) through the fused kernel, else the separate launches."""
        if self._fusable(x.shape[0]) and getattr(mod, "bias", None) is None:
            from ....ops.linear import fused_rms_linear
            r = fused_rms_linear(x, res, norm.weight, norm.eps, self._wobj(mod, li, key))
            if r is not None:
                return r
        a, h = (norm(x), x) if res is None else norm(x, res)
        return self._proj(mod, a, li, key), h

    def _mlp(self, layer, m, li=0, gu=None):
        """``gu``: the gate_up projection when the caller already ran it (fused with the norm)."""
        if hasattr(layer, "mlp"):
            mlp = layer.mlp
            if gu is None:
                gu = self._proj(mlp.gate_up_proj, m, li, "gu")
            if self._fusable(gu.shape[0]) and getattr(mlp.down_proj, "bias", None) is None:
                from ....ops.linear import fused_swiglu_linear
                y = fused_swiglu_linear(gu, self._wobj(mlp.down_proj, li, "down"))
                if y is not None:
                    return y
            return self._proj(mlp.down_proj, swiglu(gu), li, "down")
        moe = layer.block_sparse_moe if hasattr(layer, "block_sparse_moe") else layer.moe
        if self.tps is not None:  # this rank's expert columns -> partial sums -> one all-reduce
            d = self.tps.layers[li]
            y = self._moe_dropless(moe.deepspeed_moe, m, d["e_gu"], d["e_down"])
            from .... import comm as dist
            dist.all_reduce(y, group=self.tp_group)
            return y
        return self._moe_dropless(moe.deepspeed_moe, m)

    def _moe_dropless(self, moe, m, w_gu=None, w_down=None):
        """Exact top-k routing for inference (no capacity, no dropped tokens): tokens are grouped
        by expert (one argsort), each expert runs its two GEMMs on its rows, results are scattered
        back weighted by the renormalised top-k gate probabilities (reference
        ragged_ops/top_k_gating + moe_scatter + moe_gather)."""
        gate, ex = moe.gate, moe.experts
        assert moe.ep_size == 1, "ragged inference runs experts locally (ep_size == 1)"
        w_gu = ex.w_gate_up if w_gu is None else w_gu
        w_down = ex.w_down if w_down is None else w_down
        k = gate.k
        logits = F.linear(m.float(), gate.wg.weight.float())
        if self.moe_impl is not None and self.moe_impl.use_hip_gating and logits.is_cuda:
            from ....ops.moe import topk_softmax  # fused softmax + top-k kernel (moe.hip)
            probs, topi = topk_softmax(logits, k)
            topw = probs.gather(1, topi)
        else:
            probs = torch.softmax(logits, dim=-1)
            topw, topi = probs.topk(k, dim=-1)
        topw = topw / topw.sum(-1, keepdim=True)
        flat = topi.reshape(-1)
        order = torch.argsort(flat, stable=True)
        tok = order // k
        counts = torch.bincount(flat, minlength=ex.num_local_experts).tolist()
        xs = m.index_select(0, tok)
        ws = topw.reshape(-1).index_select(0, order).to(m.dtype).unsqueeze(1)
        out = torch.zeros_like(m)
        o = 0
        for e, c in enumerate(counts):
            if c == 0:
                continue
            y = torch.matmul(swiglu(torch.matmul(xs[o:o + c], w_gu[e])), w_down[e])
            out.index_add_(0, tok[o:o + c], y * ws[o:o + c])
            o += c
        return out

    @torch.no_grad()
    def forward(self, batch, kv_cache):
        model = self.model
        rope = model.rope(self.device)
        if batch.max_kv_len > rope.max_pos:  # the HIP RoPE kernels index the cos/sin table unchecked
            raise ValueError(f"sequence length {batch.max_kv_len} exceeds the model's RoPE table "
                             f"({rope.max_pos} positions, max_position_embeddings)")
        T = batch.num_tokens
        x = self.embed_impl(batch.input_ids) if self.embed_impl is not None else model.embed_tokens(batch.input_ids)
        res = None
        for li, layer in enumerate(model.layers):
            attn = layer.self_attn
            kv_layer = kv_cache.layer(li)
            r = None
            if (self._fusable(T) and self.head_dim == 128 and getattr(attn.qkv_proj, "bias", None) is None
                    and os.environ.get("SXE_DECODE_FUSE_ATTN", "1") == "1"):
                # decode: RMSNorm prologue + QKV GEMM + RoPE / KV-append epilogue in one launch
                from ....ops.linear import fused_rms_rope_linear
                ln = layer.input_layernorm
                r = fused_rms_rope_linear(x, res, ln.weight, ln.eps, self._wobj(attn.qkv_proj, li, "qkv"), rope,
                                          batch.positions, kv_layer, batch.slots, self.nq, self.nkv)
            if r is not None:
                qkv, h = r
                qkv = qkv.view(T, self.nq + 2 * self.nkv, self.head_dim)
                o = self._attn_o(attn, qkv, kv_layer, batch, li, T)
            else:
                qkv, h = self._norm_proj(layer.input_layernorm, x, res, attn.qkv_proj, li, "qkv")
                qkv = qkv.view(T, self.nq + 2 * self.nkv, self.head_dim)
                # RoPE on q/k + append of k/v to the paged cache: one launch (paged_attn.hip)
                rope_kv_cache_append(qkv, rope, batch.positions, kv_layer, batch.slots, self.nq, self.nkv)
                o = self._attn_o(attn, qkv, kv_layer, batch, li, T)
            if hasattr(layer, "mlp"):
                gu, h2 = self._norm_proj(layer.post_attention_layernorm, o, h, layer.mlp.gate_up_proj, li, "gu")
                x, res = self._mlp(layer, None, li, gu=gu), h2
            else:
                m, h2 = layer.post_attention_layernorm(o, h)
                x, res = self._mlp(layer, m, li), h2
        last = batch.last_idx
        h = model.norm(gather_rows(x, last), gather_rows(res, last))[0]
        if self.tps is not None:  # vocab-parallel head: gather every rank's logit columns
            from .... import comm as dist
            part = (self.qhead(h) if self.qw is not None else linear(h, self.tps.head)).float()
            full = torch.empty(self.tp * part.shape[0], part.shape[1], dtype=part.dtype, device=part.device)
            dist.all_gather_into_tensor(full, part, group=self.tp_group)
            return full.view(self.tp, -1, part.shape[1]).permute(1, 0, 2).reshape(part.shape[0], -1)[:, :self.tps.vocab]
        if self.qw is not None:
            return self.qhead(h).float()
        return linear(h, model.lm_head.weight).float()
