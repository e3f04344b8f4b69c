"""Floating-point quantizer (FP8 e4m3 / FP6 e3m2 / FP4 e2m1, group-scaled) and FP8 GEMMs.

Parity: reference ops/fp_quantizer/quantize.py:17 ``FP_Quantize`` (``quantize(x, q_bits,
q_mantisa_bits, stochastic_mode, return_meta_tensor)``, ``dequantize``, ``selective_dequantize``,
``get_scales``) and ops/fp_quantizer/fp8_gemm.py ``matmul_fp8`` (Triton FP8-weight GEMM,
fp8_gemm_triton.py:19,67).

MI355X-first:
* FP8 uses gfx950's OCP e4m3 hardware converters (quant.hip); FP6 (e3m2) and FP4 (e2m1) are the
  MX element formats CDNA4's ``mfma_scale`` instructions consume; on the GPU they are produced and
  decoded by the HIP kernels of mxfp.hip (nearest-representable rounding, ties to the smaller
  magnitude -- bit-identical to the value-table path used on CPU; FP4 packed 2 per byte, FP6 one
  code per byte) with one fp32 scale per group.
* ``FPxWeight`` (FP6-LLM counterpart, reference inference/v2 'wf6af16'): per-output-row scaled
  FP6 or FP4 weights in a bit-plane layout whose decode is byte-parallel in registers; decode-sized
  inputs (<= 16 rows) stream 0.75 (FP6) / 0.5 (FP4) bytes per weight through the skinny MFMA
  kernel; larger inputs run the bit planes straight through the block-scaled MFMA GEMM
  (mx_gemm.hip: exact e3m2 / e2m1 -> e4m3 transcode in registers, MXFP8 activations).
* ``fp8_linear`` runs the GEMM on the block-scaled FP8 matrix cores: the hand-written MX kernel
  (mx_gemm.hip, ``v_mfma_scale_f32_32x32x64_f8f6f4``) with MXFP8 activations (one E8M0 exponent
  per 32 values, quantised by a HIP pass) against the e4m3 weight codes with unit block exponents
  and the per-output-row weight scale in its epilogue. Measured (profiles/mx_gemm_bench.log,
  2048-8192 tokens): 0.83-1.26x bf16 hipBLASLt including the activation pass -- ahead on the
  Llama-3-8B MLP shapes, behind at N <= 6144; hipBLASLt's row-wise ``_scaled_mm`` (the previous
  route) ran 0.23-1.37x. Shapes the MX kernel does not tile (N or K not a multiple of 128) keep
  ``_scaled_mm``.
* ``matmul_fp8`` keeps the reference's weight-only semantics (bf16 activations x group-scaled
  fp8 weights, reference fp8_gemm_triton.py:19-67) by dequantising the weight in K slices of at
  most ``MATMUL_FP8_SLICE`` rows into one reused bf16 buffer and accumulating the slice GEMMs, so
  no full-size bf16 weight is ever allocated (the Triton kernel dequantises per K tile in
  registers; here a slice is staged through HBM).
"""
import math

import torch

from . import native
from .quantizer import dequantize_fp8, quantize_fp8

_FMT = {8: (4, 3), 6: (3, 2), 4: (2, 1)}  # q_bits -> (exponent bits, mantissa bits)


def _value_table(ebits, mbits):
    """All non-negative representable magnitudes of an OCP/MX float format (no inf/nan)."""
    bias = 2 ** (ebits - 1) - 1
    vals = set()
    for e in range(2 ** ebits):
        for m in range(2 ** mbits):
            if e == 0:
                v = (m / 2 ** mbits) * 2.0 ** (1 - bias)
            else:
                v = (1 + m / 2 ** mbits) * 2.0 ** (e - bias)
            vals.add(v)
    return torch.tensor(sorted(vals), dtype=torch.float32)


_TABLES = {b: _value_table(*f) for b, f in _FMT.items() if b != 8}


def _encode(x, bits):
    """x (already scaled into range) -> integer codes: sign bit | magnitude index."""
    tab = _TABLES[bits].to(x.device)
    mid = (tab[1:] + tab[:-1]) / 2
    mag = torch.bucketize(x.abs(), mid)
    sign = (x < 0).to(torch.int32)
    return (sign << (bits - 1)) | mag.to(torch.int32)


def _decode(codes, bits):
    tab = _TABLES[bits].to(codes.device)
    c = codes.to(torch.int64)
    mag = tab[c & ((1 << (bits - 1)) - 1)]
    return torch.where((c >> (bits - 1)) & 1 == 1, -mag, mag)


class FP_Quantize:
    """Group-wise FP quantizer with the reference's interface."""

    def __init__(self, group_size=512):
        self.group_size = group_size
        self.orig_dtype = None
        self.orig_shape = None
        self.scale = None
        self.q_bits = 8

    def quantize(self, input, q_bits=8, q_mantisa_bits=3, stochastic_mode=False, return_meta_tensor=False):
        assert q_bits in _FMT and _FMT[q_bits][1] == q_mantisa_bits, \
            f"supported (q_bits, mantissa): {[(b, f[1]) for b, f in _FMT.items()]}"
        assert not stochastic_mode, "stochastic rounding is not implemented"
        self.orig_dtype, self.orig_shape, self.q_bits = input.dtype, input.shape, q_bits
        x = input.contiguous().reshape(-1)
        assert x.numel() % self.group_size == 0, "numel must be a multiple of group_size"
        if q_bits == 8:
            q, s = quantize_fp8(x, self.group_size)
        elif x.is_cuda and native.use_hip(x):
            q, s = torch.ops.sxe.fpx_quantize(x, q_bits, self.group_size)
        else:
            g = x.float().reshape(-1, self.group_size)
            amax = g.abs().amax(1)
            fmax = float(_TABLES[q_bits][-1])
            s = torch.where(amax > 0, amax / fmax, torch.ones_like(amax))
            codes = _encode(g / s[:, None], q_bits).reshape(-1).to(torch.uint8)
            q = (codes[0::2] | (codes[1::2] << 4)) if q_bits == 4 else codes
        self.scale = s
        return (q, s) if return_meta_tensor else q

    def get_scales(self):
        return self.scale

    def dequantize(self, input_q, fp_out=None, q_bits=None, q_mantisa_bits=None, scale=None):
        bits = q_bits or self.q_bits
        s = scale if scale is not None else self.scale
        n = s.numel() * self.group_size
        if bits == 8:
            out = dequantize_fp8(input_q, s, self.group_size, out=fp_out, dtype=self.orig_dtype or torch.bfloat16)
        elif input_q.is_cuda and native.use_hip(input_q):
            v = torch.ops.sxe.fpx_dequantize(input_q.contiguous(), s.float().contiguous(), bits, self.group_size, n,
                                             self.orig_dtype or torch.bfloat16)
            out = fp_out.reshape(-1).copy_(v) if fp_out is not None else v
        else:
            codes = input_q
            if bits == 4:
                codes = torch.stack([input_q & 0xF, input_q >> 4], 1).reshape(-1)
            v = _decode(codes[:n], bits).reshape(-1, self.group_size) * s.reshape(-1, 1)
            v = v.reshape(-1).to(self.orig_dtype or torch.bfloat16)
            out = fp_out.reshape(-1).copy_(v) if fp_out is not None else v
        if fp_out is None and self.orig_shape is not None and out.numel() == torch.Size(self.orig_shape).numel():
            return out.view(self.orig_shape)
        return out

    def selective_dequantize(self, input_q, indexes, fp_out=None, q_bits=None, q_mantisa_bits=None, scale=None):
        """Dequantize only the rows ``indexes`` of a [rows, ...] quantized tensor (rows a multiple of
        groups), e.g. the experts routed to in an MoE layer."""
        bits = q_bits or self.q_bits
        s = (scale if scale is not None else self.scale)
        rows = self.orig_shape[0]
        per_row = torch.Size(self.orig_shape[1:]).numel()
        gpr = per_row // self.group_size
        bpr = per_row * bits // 8 if bits != 6 else per_row
        q_rows = input_q.reshape(rows, bpr)[indexes]
        s_rows = s.reshape(rows, gpr)[indexes]
        sub = FP_Quantize(self.group_size)
        sub.orig_dtype, sub.orig_shape, sub.q_bits = self.orig_dtype, (len(indexes),) + tuple(self.orig_shape[1:]), bits
        return sub.dequantize(q_rows.reshape(-1), fp_out, bits, scale=s_rows.reshape(-1))


# ---------------------------------------------------------------------------------------- FP8 GEMMs
def quantize_weight_fp8_rowwise(w):
    """w [N, K] -> (fp8 e4m3 [N, K], fp32 scales [N])."""
    q, s = quantize_fp8(w.reshape(-1), w.shape[1])
    return q.view(torch.float8_e4m3fn).view(w.shape), s


_UNIT_EXP = {}


def _unit_exponents(N, K, device):
    """E8M0 block exponents of 1.0 for an [N, K] e4m3 weight used as MXFP8 (cached: a HIP-graph
    capture must not allocate)."""
    key = (N, K // 32, str(device))
    t = _UNIT_EXP.get(key)
    if t is None:
        t = _UNIT_EXP[key] = torch.full((N, K // 32), 127, dtype=torch.uint8, device=device)
    return t


def fp8_linear(x, w_q, w_scale, bias=None, out_dtype=torch.bfloat16):
    """y = x @ (w_q * w_scale[:, None])^T on the FP8 matrix cores. x [..., K] bf16/fp32, w_q [N, K]
    float8_e4m3fn, w_scale [N] fp32. GPU: MXFP8 activations x e4m3 weights on the block-scaled MX
    GEMM (per-row weight scale in the epilogue); CPU: the same product from dequantised fp32."""
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    N = w_q.shape[0]
    if x2.is_cuda and K % 128 == 0 and N % 128 == 0:
        from .mx import mx_linear
        native.require_hip()
        wq8 = w_q.view(torch.uint8)
        y = mx_linear(x2, wq8, _unit_exponents(N, K, x2.device), "mxfp8", bias, col_scale=w_scale)
        return y.to(out_dtype).view(*x.shape[:-1], N)
    if x2.is_cuda and K % 16 == 0 and N % 16 == 0:
        native.require_hip()
        q, s = quantize_fp8(x2, K)
        y = torch._scaled_mm(q.view(torch.float8_e4m3fn).view(x2.shape), w_q.t(), scale_a=s.view(-1, 1),
                             scale_b=w_scale.view(1, -1), bias=bias, out_dtype=out_dtype)
    else:
        q, s = quantize_fp8(x2, K)
        xd = q.view(torch.float8_e4m3fn).float().view(x2.shape) * s.view(-1, 1)
        wd = w_q.float() * w_scale.view(-1, 1)
        y = (xd @ wd.t()).to(out_dtype)
        if bias is not None:
            y = y + bias.to(out_dtype)
    return y.view(*x.shape[:-1], N)


MATMUL_FP8_SLICE = 1024  # weight rows (K) dequantised per slice in matmul_fp8


def matmul_fp8(inp, weight, scale, quantization_group_size):
    """Reference ``matmul_fp8``: inp [M, K] (bf16/fp16) x weight [K, N] stored as fp8 (uint8 codes
    or float8_e4m3fn) with one scale per ``quantization_group_size`` consecutive weight elements.
    The weight is dequantised K-slice by K-slice into one reused buffer (never the whole weight)."""
    wq = weight.view(torch.uint8) if weight.dtype != torch.uint8 else weight
    K, N = weight.shape
    g = int(quantization_group_size)
    flat, sc = wq.reshape(-1), scale.reshape(-1)
    step = g // math.gcd(g, N)  # slices start on a scale-group boundary: rows * N % g == 0
    rows = max(step, (MATMUL_FP8_SLICE // step) * step)
    if rows >= K:
        return torch.matmul(inp, dequantize_fp8(flat, sc, g, dtype=inp.dtype).view(K, N))
    buf = torch.empty(rows * N, dtype=inp.dtype, device=inp.device)
    x2 = inp.reshape(-1, K)
    out = torch.zeros(x2.shape[0], N, dtype=torch.float32, device=inp.device)  # fp32 sum over slices
    for k0 in range(0, K, rows):
        k1 = min(K, k0 + rows)
        e0, e1 = k0 * N, k1 * N
        seg = dequantize_fp8(flat[e0:e1], sc[e0 // g:(e1 + g - 1) // g], g, out=buf[:e1 - e0], dtype=inp.dtype)
        w = seg.view(k1 - k0, N)
        if out.is_cuda:  # fp32-out GEMM accumulating in its epilogue: no bf16 partial products
            torch.ops.aten.addmm.dtype_out(out, x2[:, k0:k1], w, torch.float32, beta=1, alpha=1, out=out)
        else:
            out.addmm_(x2[:, k0:k1].float(), w.float())
    return out.to(inp.dtype).view(*inp.shape[:-1], N)

class FP8Weight:
    """Row-scaled FP8 (e4m3) weight of a linear layer, [N, K] -> used through ``ops.linear.linear``:
    decode-sized inputs (<= 16 rows) stream the FP8 bytes through the skinny MFMA kernel
    (skinny_gemm.hip, W8A16: weights converted to bf16 in registers, half the HBM bytes of bf16);
    larger inputs run ``fp8_linear`` on the FP8 matrix cores (activations quantized per row)."""

    def __init__(self, w):
        self.q, self.scale = quantize_weight_fp8_rowwise(w.detach())
        self.shape = tuple(w.shape)
        self.dtype = w.dtype

    def linear(self, x, bias=None):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if (x2.is_cuda and x2.dtype == torch.bfloat16 and 0 < x2.shape[0] <= 16 and K % 16 == 0
                and x2.stride(-1) == 1 and x2.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0):
            native.require_hip()
            b = bias.to(torch.bfloat16).contiguous() if bias is not None else None
            y = torch.ops.sxe.skinny_gemm_fp8w(x2, self.q.view(torch.uint8), self.scale, b)
            return y.view(*x.shape[:-1], self.q.shape[0])
        return fp8_linear(x, self.q, self.scale, bias, out_dtype=x.dtype)

    def dequantize(self):
        return (self.q.float() * self.scale.view(-1, 1)).to(self.dtype)


class FP8Linear(torch.nn.Module):
    """Inference linear with an FP8 (row-scaled) weight; the GEMM runs on the FP8 matrix cores."""

    def __init__(self, linear: torch.nn.Linear):
        super().__init__()
        q, s = quantize_weight_fp8_rowwise(linear.weight.detach())
        self.register_buffer("weight_q", q)
        self.register_buffer("weight_scale", s)
        self.bias = linear.bias
        self.in_features, self.out_features = linear.in_features, linear.out_features

    def forward(self, x):
        b = self.bias.to(x.dtype) if self.bias is not None else None
        return fp8_linear(x, self.weight_q, self.weight_scale, b, out_dtype=x.dtype)


# ------------------------------------------------------------------------- FP6 / FP4 weights
def _codes(w, bits):
    """w [N, K] -> (per-element codes uint8 [N, K], per-row scales fp32 [N])."""
    N, K = w.shape
    fq = FP_Quantize(group_size=K)
    q = fq.quantize(w.contiguous(), q_bits=bits, q_mantisa_bits=_FMT[bits][1])
    if bits == 4:
        q = torch.stack([q & 0xF, q >> 4], 1)
    return q.reshape(N, K), fq.get_scales().float()


def _nibble_words(c):
    """[N, K] 4-bit values -> [N, K/2] bytes, each 32-bit word (8 values) byte b = v_b | v_{b+4} << 4."""
    N, K = c.shape
    v = c.reshape(N, K // 8, 2, 4)
    return (v[:, :, 0] | (v[:, :, 1] << 4)).reshape(N, K // 2).contiguous()


def _crumb_words(m):
    """[N, K] 2-bit values -> [N, K/4] bytes, each 32-bit word (16 values) byte b = v_b | v_{b+4} << 2
    | v_{b+8} << 4 | v_{b+12} << 6."""
    N, K = m.shape
    v = m.reshape(N, K // 16, 4, 4)
    return (v[:, :, 0] | (v[:, :, 1] << 2) | (v[:, :, 2] << 4) | (v[:, :, 3] << 6)).reshape(N, K // 4).contiguous()


class FPxWeight:
    """Per-output-row scaled FP6 (e3m2) or FP4 (e2m1) weight of a linear layer, [N, K] (K a
    multiple of 128), in the bit-plane layout of csrc/kernels/mxfp.hip: FP4 = one nibble plane,
    FP6 = the (sign | exponent) nibble plane + a 2-bit mantissa plane."""

    def __init__(self, w, bits=6):
        assert bits in (4, 6), "FPxWeight: bits 4 or 6"
        N, K = w.shape
        assert K % 128 == 0, "FPxWeight: in_features must be a multiple of 128"
        self.bits, self.shape, self.dtype = bits, (N, K), w.dtype
        codes, self.scale = _codes(w.detach(), bits)
        if bits == 4:
            self.wa, self.wb = _nibble_words(codes), None
        else:
            self.wa, self.wb = _nibble_words(codes >> 2), _crumb_words(codes & 3)
        # unit E8M0 block exponents for the MX GEMM (the per-row scale is its epilogue scale); made
        # here, not lazily, so a HIP-graph capture never allocates it
        self._e127 = torch.full((1, K // 32), 127, dtype=torch.uint8, device=self.wa.device)

    def _codes_back(self):
        N, K = self.shape
        a = self.wa.reshape(N, K // 8, 4)
        nib = torch.stack([a & 0xF, a >> 4], 2).reshape(N, K)
        if self.bits == 4:
            return nib
        b = self.wb.reshape(N, K // 16, 4)
        crumbs = torch.stack([(b >> (2 * j)) & 3 for j in range(4)], 2).reshape(N, K)
        return (nib << 2) | crumbs

    def dequantize(self, dtype=torch.bfloat16):
        if self.wa.is_cuda and native.use_hip(self.wa):
            return torch.ops.sxe.fpxw_unpack(self.wa, self.wb, self.scale, self.bits).to(dtype)
        v = _decode(self._codes_back().reshape(-1), self.bits).reshape(self.shape)
        return (v * self.scale.view(-1, 1)).to(dtype)

    def linear(self, x, bias=None):
        """Decode-sized inputs (<= 16 rows): W{6,4}A16 on the skinny kernel. Larger inputs: the bit
        planes go straight into the block-scaled MFMA GEMM (mx_gemm.hip, transcoded to e4m3 in
        registers, activations quantised to MXFP8 on the fly, the per-row scale in the epilogue) --
        the weight is never widened in HBM. CPU: the dequantised fp32 product."""
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        N = self.shape[0]
        if (x2.is_cuda and x2.dtype == torch.bfloat16 and 0 < x2.shape[0] <= 16 and x2.stride(-1) == 1
                and x2.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0):
            native.require_hip()
            b = bias.to(torch.bfloat16).contiguous() if bias is not None else None
            y = torch.ops.sxe.skinny_gemm_fpxw(x2, self.wa, self.wb, self.scale, b, self.bits)
            return y.view(*x.shape[:-1], N)
        if x2.is_cuda and N % 128 == 0 and x2.shape[0] > 0:
            native.require_hip()
            q, s = torch.ops.sxe.mx_quant_fp8(x2.to(torch.bfloat16).contiguous())
            b = bias.to(torch.bfloat16).contiguous() if bias is not None else None
            y = torch.ops.sxe.mx_gemm(q, s, self.wa, self._e127, 16 if self.bits == 6 else 17, b, self.scale, self.wb)
            return y.view(*x.shape[:-1], N).to(x.dtype)
        y = torch.nn.functional.linear(x2, self.dequantize(x2.dtype), bias.to(x2.dtype) if bias is not None else None)
        return y.view(*x.shape[:-1], N)


def quantized_weight(w, kind):
    """Inference weight quantization by name: 'fp8' (W8A16), 'fp6' / 'wf6af16' (FP6-LLM), 'fp4',
    'int8' / 'int4' (W8A16 / W4A16 on the mixed-precision grouped kernel), and the OCP-MX formats
    'mxfp8' / 'mxfp6' / 'mxfp4' (W{8,6,4}A8 on gfx950's block-scaled matrix cores, ops/mx.py)."""
    if kind in ("int8", "int4"):
        from .moe import IntWeight
        return IntWeight(w, 8 if kind == "int8" else 4)
    if kind in ("mxfp8", "mxfp6", "mxfp6_e2m3", "mxfp4"):
        from .mx import MXWeight
        return MXWeight(w, kind)
    if kind == "fp8":
        return FP8Weight(w)
    if kind in ("fp6", "wf6af16"):
        return FPxWeight(w, 6)
    if kind in ("fp4", "wf4af16"):
        return FPxWeight(w, 4)
    raise ValueError(f"unknown weight quantization {kind!r} (fp8 | fp6 | fp4 | int8 | int4 | mxfp8 | mxfp6 | mxfp4)")
