"""Linear layer whose weight gradient is written straight into the ZeRO gradient buffer.

If a weight carries ``_sxe_grad_target`` (installed by the ZeRO optimizers), the backward weight-grad
GEMM writes its result directly where the optimizer wants it:
  * fp32 accumulator (single-rank / persistent units): ONE hipBLASLt GEMM with fp32 output and
    beta = 1 (``aten::addmm.dtype_out``) -- no bf16 ``p.grad`` tensor, no separate fp32 add pass,
    and micro-batch accumulation happens at fp32 precision inside the GEMM epilogue;
  * bf16 reduce-scatter staging slot (multi-rank units): the GEMM output IS the send buffer.
then calls ``_sxe_grad_done`` so the optimizer can launch the unit's reduce-scatter. Without a
target it behaves exactly like ``torch.nn.functional.linear``. (The reference's analogue is
Megatron-style ``gradient_accumulation_fusion``; DeepSpeed's ZeRO copies each ``p.grad`` into an
IPG bucket instead, stage_1_and_2.py:1137-1139.)
"""
import os
import weakref

import torch
import torch.nn.functional as F

# Large weight-gradient GEMMs (MLP projections, LM head) run faster as two HBM-speed transposes +
# a forward-layout ("TN") bf16 GEMM + an fp32 accumulate than as one fp32-output GEMM in the
# token-major "NT" layout: hipBLASLt reaches 1.47-1.61 PF in TN vs 1.06-1.19 PF in NT on MI355X
# (tools/wgrad_layout_exp.py, tools/wgrad_tn_exp.py: -0.13 ms per 28672x4096 / 4096x14336 call,
# -0.47 ms for the 128256x4096 LM head, at K = 8192 tokens). Smaller weights keep the fused path.
TN_MIN_ELEMS = int(os.environ.get("SXE_WGRAD_TN_MIN_ELEMS", 32 * 2**20))
# TN weight gradient into an fp32 accumulator: one fp32-output GEMM with beta = 1 (hipBLASLt "BSS"
# kernels), or (SXE_WGRAD_TN_FP32OUT=0) the bf16-output TN GEMM -- the faster kernel family -- plus
# an fp32 accumulate pass (what ops/mlp.py's weight_grad_tn does for the MLP weights)
TN_FP32_OUT = os.environ.get("SXE_WGRAD_TN_FP32OUT", "1") == "1"

# Decode-shaped products (<= 4 rows, no autograd) stream the weight through the MFMA skinny-GEMM
# kernel (csrc/kernels/skinny_gemm.hip) instead of hipBLASLt's general tiles. Measured on MI355X
# (tools/skinny_bench.py, profiles/skinny_bench.log), Llama-3-8B shapes, M = 1: o_proj 7.3 vs
# 11.8 us, gate_up 42 vs 56 us, down 24.8 vs 25.7 us, LM head 169 vs 180 us, QKV 12.4 vs 10.6 us;
# at M = 8-16 hipBLASLt is as fast or faster (the kernel supports M <= 16).
SKINNY_MAX_M = int(os.environ.get("SXE_SKINNY_MAX_M", 4))


def _skinny(x, weight, bias):
    if torch.compiler.is_compiling():  # data_ptr() is not traceable; graphs keep the library GEMM
        return None
    K = x.shape[-1]
    if not (x.is_cuda and x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and weight.dim() == 2
            and weight.is_contiguous() and K % 8 == 0 and weight.data_ptr() % 16 == 0):
        return None
    if bias is not None and not (bias.dtype == torch.bfloat16 and bias.is_contiguous()):
        return None
    x2 = x.reshape(-1, K)
    if not (0 < x2.shape[0] <= SKINNY_MAX_M and x2.stride(1) == 1 and x2.stride(0) % 8 == 0
            and x2.data_ptr() % 16 == 0):
        return None
    from . import native
    native.require_hip()
    return torch.ops.sxe.skinny_gemm(x2, weight, bias).view(*x.shape[:-1], weight.shape[0])


def _pro_weight(weight):
    """(w, scale) for the fused-prologue skinny kernels: a bf16 [N, K] tensor or an FP8Weight."""
    if isinstance(weight, torch.Tensor):
        if weight.dtype == torch.bfloat16 and weight.dim() == 2 and weight.is_contiguous() and weight.data_ptr() % 16 == 0:
            return weight, None
        return None
    from .fp_quantizer import FP8Weight
    if not isinstance(weight, FP8Weight):  # other quantized formats (MX, FP6/FP4 planes, int) run unfused
        return None
    q, sc = weight.q, weight.scale
    if q.element_size() == 1 and q.dim() == 2 and q.is_contiguous():
        return q.view(torch.uint8), sc
    return None


def _pro_ok(x, rows_max=4):
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and 0 < x.shape[0] <= rows_max
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 and not x.requires_grad)


def fused_rms_linear(x, residual, norm_weight, eps, weight, bias=None):
    """Decode (<= 4 rows): ``linear(rms_norm(x + residual), weight)`` in ONE launch
    (skinny_gemm.hip PRO_RMS). Returns (y, h = x + residual) -- h is x itself without a residual --
    or None when the fused kernel does not cover the operands (the caller runs the unfused ops)."""
    wk = _pro_weight(weight)
    if wk is None or not _pro_ok(x) or norm_weight.dtype != torch.bfloat16 or not norm_weight.is_contiguous():
        return None
    if residual is not None and (residual.shape != x.shape or residual.stride() != x.stride()
                                 or residual.dtype != x.dtype):
        return None
    w, sc = wk
    if x.shape[1] != w.shape[1]:
        return None
    y, h = torch.ops.sxe.skinny_gemm_pro(x, residual, norm_weight, float(eps), w, sc, bias, 1)
    return y, (h if residual is not None else x)


def fused_rms_rope_linear(x, residual, norm_weight, eps, weight, rope, positions, cache, slots, nq, nkv):
    """Decode (<= 4 rows) QKV projection in ONE launch: residual + RMSNorm prologue, GEMM, and the
    RoPE + paged-KV-append epilogue (skinny_gemm.hip ``skinny_gemm_pro_rope``; head dim 128).
    Returns (qkv with q / k rotated, h) -- the rotated k and v are already in ``cache`` -- or None
    when not covered (the caller runs fused_rms_linear + rope_kv_cache_append)."""
    wk = _pro_weight(weight)
    if (wk is None or not _pro_ok(x) or norm_weight.dtype != torch.bfloat16 or not norm_weight.is_contiguous()
            or rope.cos.shape[-1] != 64 or not cache.is_contiguous() or cache.dim() != 5 or cache.shape[-1] != 128):
        return None
    if residual is not None and (residual.shape != x.shape or residual.stride() != x.stride()
                                 or residual.dtype != x.dtype):
        return None
    w, sc = wk
    if x.shape[1] != w.shape[1] or w.shape[0] != (nq + 2 * nkv) * 128:
        return None
    y, h = torch.ops.sxe.skinny_gemm_pro_rope(x, residual, norm_weight, float(eps), w, sc, rope.cos, rope.sin,
                                              positions.reshape(-1).contiguous().long(), slots, cache, int(nq), int(nkv))
    return y, (h if residual is not None else x)


def fused_swiglu_linear(gu, weight, bias=None):
    """Decode (<= 4 rows): ``linear(silu(gu[:, :I]) * gu[:, I:], weight)`` in ONE launch
    (skinny_gemm.hip PRO_SWIGLU); None when not covered."""
    wk = _pro_weight(weight)
    if wk is None or not _pro_ok(gu):
        return None
    w, sc = wk
    if gu.shape[1] != 2 * w.shape[1]:
        return None
    return torch.ops.sxe.skinny_gemm_pro(gu, None, None, 0.0, w, sc, bias, 2)[0]


def fused_merge_linear(part_o, part_ml, weight, bias=None):
    """Decode (<= 4 rows): ``linear(merge(part_o, part_ml), weight)`` in ONE launch -- the
    flash-decoding merge of paged attention's KV-split partials runs as the o_proj skinny GEMM's
    prologue (skinny_gemm.hip PRO_MERGE). None when the weight is not covered (bf16 / FP8 only)."""
    wk = _pro_weight(weight)
    if wk is None or not part_o.is_cuda or part_o.shape[1] > 4:
        return None
    w, sc = wk
    if w.shape[1] != part_o.shape[2] * part_o.shape[3]:
        return None
    return torch.ops.sxe.skinny_gemm_merge(part_o, part_ml, w, sc, bias)


# Hand-written weight-gradient GEMM (csrc/kernels/gemm_wgrad.hip: k-major operands read through LDS
# with ds_read_b64_tr_b16, fp32 accumulate in the epilogue): no transposed copies of dY / X at all.
# Measured on MI355X at 8192 tokens (tools/wgrad_exp.py, profiles/wgrad_kernel.log): 28672x4096
# 1.59 ms vs 1.63 (transposes + hipBLASLt TN fp32-out), 4096x14336 0.84 vs 0.89, 4096x4096 0.24 vs
# 0.25 (NT fp32-out); it loses where its 256x256 tile grid leaves a partial last wave of blocks
# (6144x4096: 1.5 waves over 256 CUs, see WGRAD_MIN_TILES) and on the LM head, which keep the
# library paths.
SXE_WGRAD = os.environ.get("SXE_WGRAD", "1") == "1"
# smallest non-multiple-of-256 tile count for the hand-written kernel: the fused QKV projection (384
# tiles, 1.5 waves) wins in isolation at 8192 tokens (0.43 vs 0.46 ms) but not inside the
# Llama-3-8B step at 16,384 tokens per micro-step (0.78 vs 0.74 ms per call,
# profiles/r05/bench_llama3_8b_zero3_1gpu_step_final.md, headline_wgrad_norm_ab.log)
WGRAD_MIN_TILES = int(os.environ.get("SXE_WGRAD_MIN_TILES", "768"))


def _sxe_wgrad_ok(gy2, x2, buf):
    if not (SXE_WGRAD and gy2.is_cuda and buf.dtype == torch.float32 and gy2.dtype == torch.bfloat16
            and x2.dtype == torch.bfloat16 and buf.is_contiguous() and gy2.stride(1) == 1 and x2.stride(1) == 1):
        return False
    K, M, N = gy2.shape[0], gy2.shape[1], x2.shape[1]
    if K % 128 or M % 256 or N % 256 or gy2.stride(0) % 8 or x2.stride(0) % 8 or M * N >= 2 ** 27:
        return False
    tiles = (M // 256) * (N // 256)
    return tiles % 256 == 0 or tiles >= WGRAD_MIN_TILES


def _tn_ok(gy2, x2):
    return (gy2.is_cuda and gy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 and TN_MIN_ELEMS > 0
            and gy2.shape[1] * x2.shape[1] >= TN_MIN_ELEMS and gy2.shape[0] % 64 == 0 and gy2.shape[1] % 64 == 0
            and x2.shape[1] % 64 == 0 and gy2.is_contiguous() and x2.is_contiguous())


# Data-gradient GEMMs dX = dY W run in hipBLASLt's "NN" layout at 1.03-1.35 PF on MI355X; with W^T
# materialised by the HBM-speed transpose they run in the forward layout at 1.25-1.56 PF
# (tools/gemm_layout_bench.py, profiles/gemm_layout.log: net -0.03..-0.06 ms per Llama-3-8B layer
# GEMM, -0.48 ms for the LM head, at 8192 tokens). The transpose reads/writes only the weight.
DGRAD_WT_MIN_ELEMS = int(os.environ.get("SXE_DGRAD_WT_MIN_ELEMS", 16 * 2**20))


# The transposed weights are constant between optimizer steps: with gradient accumulation each
# micro-step's backward (and each chunk of a chunked LM-head loss) would transpose the same weight
# again (the transpose kernel was 1.7 % of the Llama-3-8B ZeRO-3 step at 2 micro-steps). The engine
# enables this cache for gradient_accumulation_steps > 1 and clears it after every optimizer step
# and checkpoint load; it holds at most SXE_WT_CACHE_GB of transposes (ZeRO-3 models whose
# gathered weights do not stay resident simply stop caching at the cap).
WT_CACHE = False
WT_CACHE_MAX_BYTES = int(float(os.environ.get("SXE_WT_CACHE_GB", "20")) * 2**30)
_wt_cache = {}
_wt_cache_bytes = 0


def invalidate_transposed_weights():
    global _wt_cache_bytes
    _wt_cache.clear()
    _wt_cache_bytes = 0


def _transpose16(t):
    return torch.ops.sxe.transpose16(t)


def _transposed_weight(w):
    global _wt_cache_bytes
    if not WT_CACHE or not isinstance(w, torch.nn.Parameter):
        return _transpose16(w)
    hit = _wt_cache.get(id(w))
    # a weight rebound to other storage (ZeRO-3 gather into a new buffer) or bumped by an in-place
    # write through the Parameter itself misses instead of returning a stale transpose; writers that
    # go through other views of a flat buffer call invalidate_transposed_weights()
    if (hit is not None and hit[0]() is w and hit[1].shape == w.shape[::-1] and hit[2] == w.data_ptr()
            and hit[3] == w._version):
        return hit[1]
    if hit is not None:
        _wt_cache.pop(id(w))
        _wt_cache_bytes -= hit[1].numel() * hit[1].element_size()
    wt = _transpose16(w)
    nbytes = wt.numel() * wt.element_size()
    if _wt_cache_bytes + nbytes <= WT_CACHE_MAX_BYTES:
        _wt_cache[id(w)] = (weakref.ref(w), wt, w.data_ptr(), w._version)
        _wt_cache_bytes += nbytes
    return wt


def transposed_weight_cache_bytes():
    return _wt_cache_bytes


def configure_transposed_weight_cache(enabled, free_bytes=None):
    """Turn the cache on / off; with ``free_bytes`` (free HBM after the engine is built) the cap is
    at most a quarter of it, so the cache never takes memory a configuration needs to fit."""
    global WT_CACHE, WT_CACHE_MAX_BYTES
    WT_CACHE = bool(enabled)
    cap = int(float(os.environ.get("SXE_WT_CACHE_GB", "20")) * 2**30)
    if free_bytes is not None:
        cap = min(cap, int(free_bytes) // 4)
    WT_CACHE_MAX_BYTES = cap
    invalidate_transposed_weights()
    return cap


def data_grad(gy, w):
    """dX = gy @ w for w [N, K] (gy [..., N])."""
    if (DGRAD_WT_MIN_ELEMS > 0 and gy.is_cuda and gy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and w.dim() == 2 and w.is_contiguous() and w.numel() >= DGRAD_WT_MIN_ELEMS and w.shape[0] % 64 == 0
            and w.shape[1] % 64 == 0 and gy.numel() // gy.shape[-1] >= 2048):
        return torch.matmul(gy, _transposed_weight(w).t())
    return torch.matmul(gy, w)


def grad_target(w):
    """The optimizer's direct weight-grad target of ``w`` (``_sxe_grad_target``), or None when the
    gradient must take autograd's ``.grad`` path instead: a partial gradient of a tiled / recomputed
    sub-graph (``_sxe_grad_partial``, set by sequence/tiled.py for every tile but the last -- the
    reference's ``ds_grad_is_ready = False``, runtime/sequence_parallel/ulysses_sp.py:720-724), or a
    ``.grad`` that already holds such partial sums (the last tile adds into it, and the ZeRO hook
    then delivers the total once)."""
    tgt = getattr(w, "_sxe_grad_target", None)
    if tgt is None or getattr(w, "_sxe_grad_partial", False) or w.grad is not None:
        return None
    return tgt


def write_weight_grad(w, gy2, x2):
    """dW = gy2^T @ x2 into the optimizer-provided target of `w`; returns True if handled."""
    tgt = grad_target(w)
    if tgt is None:
        return False
    buf, accumulate = tgt(w)
    if _sxe_wgrad_ok(gy2, x2, buf):
        torch.ops.sxe.wgrad_gemm_(gy2, x2, buf, 1.0, bool(accumulate))
    elif _tn_ok(gy2, x2) and buf.is_contiguous():
        a, b = torch.ops.sxe.transpose16(gy2), torch.ops.sxe.transpose16(x2).t()
        if buf.dtype == gy2.dtype and not accumulate:
            torch.mm(a, b, out=buf)  # the reduce-scatter staging slot of a multi-rank unit
        elif buf.dtype == torch.float32 and TN_FP32_OUT:
            # fp32-out TN GEMM accumulating in its epilogue (beta = 1): no bf16 dW round trip and no
            # separate fp32 add pass (28672x4096 at 8192 tokens: 1.62 vs 1.74 ms, wgrad_tn_fp32_exp)
            torch.ops.aten.addmm.dtype_out(buf, a, b, torch.float32, beta=1 if accumulate else 0, alpha=1, out=buf)
        else:
            dw = torch.mm(a, b).view_as(buf)
            buf.add_(dw) if accumulate else buf.copy_(dw)
    elif buf.dtype == torch.float32 and gy2.dtype != torch.float32:
        if gy2.is_cuda:
            torch.ops.aten.addmm.dtype_out(buf, gy2.t(), x2, torch.float32, beta=1 if accumulate else 0, alpha=1,
                                           out=buf)
        else:  # CPU processes (gloo plumbing runs): no fp32-out GEMM for 16-bit inputs there
            dw = (gy2.t() @ x2).float()
            buf.add_(dw) if accumulate else buf.copy_(dw)
    elif accumulate:
        buf.addmm_(gy2.t(), x2)
    else:
        torch.mm(gy2.t(), x2, out=buf)
    w._sxe_grad_done(w)
    return True


def _autocast_dtype(x):
    """The torch.autocast compute dtype active for ``x``'s device, or None."""
    dev = x.device.type
    if dev in ("cuda", "cpu") and torch.is_autocast_enabled(dev):
        return torch.get_autocast_dtype(dev)
    return None


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.param = None
        ac = _autocast_dtype(x)
        if ac is not None and weight.dtype != ac:
            # torch_autocast training (runtime/torch_autocast.py): fp32 master-precision parameters,
            # GEMMs in the autocast dtype. The fp32 Parameter keeps receiving its gradient through
            # the optimizer's direct weight-grad target; the bf16 copies are what backward reads.
            ctx.param = weight
            x, weight = x.to(ac), weight.to(ac)
            bias = bias.to(ac) if bias is not None else None
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        wp = ctx.param if ctx.param is not None else w
        if gy.dtype != x.dtype:
            gy = gy.to(x.dtype)
        gy2 = gy.reshape(-1, gy.shape[-1])
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = data_grad(gy, w)
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, x.shape[-1])
            if not write_weight_grad(wp, gy2, x2):
                dw = gy2.t() @ x2
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = gy2.sum(0)
        return dx, dw, db


def linear(x, weight, bias=None):
    if not isinstance(weight, torch.Tensor):  # quantized inference weight (ops/fp_quantizer.FP8Weight)
        return weight.linear(x, bias)
    grad = torch.is_grad_enabled() and (weight.requires_grad or x.requires_grad)
    if grad and weight.requires_grad and hasattr(weight, "_sxe_grad_target"):
        return _Linear.apply(x, weight, bias)
    if not grad and SKINNY_MAX_M > 0 and x.is_cuda:
        y = _skinny(x, weight, bias)
        if y is not None:
            return y
    return F.linear(x, weight, bias)


class Linear(torch.nn.Linear):
    """``nn.Linear`` whose GEMMs go through ``linear`` (fused weight-grad into ZeRO buffers).
    AutoTP swaps it for a column/row-parallel layer with the same call signature.

    ``init_std``: initialise the weight N(0, init_std) (bias zero) inside the constructor, i.e.
    on the whole tensor before a partitioning ``zero.Init`` cuts it -- the initial model then
    depends only on the seed, not on the number of ranks."""

    _sxe_lower_precision_safe = True  # torch_autocast: GEMM weights may communicate in bf16 / fp16

    def __init__(self, in_features, out_features, bias=True, device=None, dtype=None, init_std=None):
        super().__init__(in_features, out_features, bias=bias, device=device, dtype=dtype)
        if init_std is not None:
            with torch.no_grad():
                self.weight.normal_(0.0, init_std)
                if self.bias is not None:
                    self.bias.zero_()
            self._sxe_inited = True

    def forward(self, x, skip_bias=False):
        return linear(x, self.weight, None if skip_bias else self.bias)


class Embedding(torch.nn.Embedding):
    """``nn.Embedding`` with the constructor-time N(0, init_std) init of ``Linear``."""

    def __init__(self, num_embeddings, embedding_dim, init_std=None, **kw):
        super().__init__(num_embeddings, embedding_dim, **kw)
        if init_std is not None:
            with torch.no_grad():
                self.weight.normal_(0.0, init_std)
            self._sxe_inited = True
