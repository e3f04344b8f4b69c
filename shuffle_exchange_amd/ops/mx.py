"""OCP-MX (microscaling) weights and the block-scaled GEMM on gfx950's scaled matrix cores.

An MX tensor stores every 32 consecutive elements along K as low-bit codes plus ONE shared
power-of-two exponent (E8M0 byte, bias 127). CDNA4's ``v_mfma_scale_f32_32x32x64_f8f6f4`` consumes
exactly that: the codes as the operand and the exponent byte per lane, dequantising inside the
matrix core (csrc/kernels/mx_gemm.hip). Element formats (MFMA format code):

  ``mxfp8``  e4m3  (0)   8 bits, max 448
  ``mxfp6``  e3m2  (3)   6 bits, max 28      -- the FP6-LLM element format
  ``mxfp6_e2m3`` (2)     6 bits, max 7.5
  ``mxfp4``  e2m1  (4)   4 bits, max 6

Packing (what the MFMA reads, see mx_gemm.hip): element j of a row sits at bits [w j, w j + w) of
the row's little-endian byte stream -- fp8 one byte each, fp4 two per byte (low nibble first),
fp6 four elements per three bytes.

``MXWeight`` is the inference weight built on it (reference counterparts: inference/v2
``wf6af16`` FP6-LLM linear, inference/v2/kernels/core_ops/cuda_linear/linear_kernels_cuda.cu:70,216,
and ops/fp_quantizer): prefill activations are quantised on the fly to MXFP8 (one HIP pass) and
the GEMM runs on the FP8/FP6/FP4 matrix cores; decode (<= 16 rows) streams the MX codes through a
skinny kernel that decodes them in registers (csrc/kernels/skinny_dq.hip) -- the weight stays in
its MX bytes end to end.
On the CPU the same quantise-then-multiply semantics run in PyTorch (the numerics oracle).
"""
import torch

from . import native

# name -> (MFMA format code, exponent bits, mantissa bits, element bits, max magnitude)
FORMATS = {
    "mxfp8": (0, 4, 3, 8, 448.0),
    "mxfp6": (3, 3, 2, 6, 28.0),
    "mxfp6_e2m3": (2, 2, 3, 6, 7.5),
    "mxfp4": (4, 2, 1, 4, 6.0),
}
BLOCK = 32
_SKINNY = ("mxfp8", "mxfp6", "mxfp4")  # formats the decode kernel (skinny_dq.hip) reads


def _values(ebits, mbits):
    """Magnitudes of codes 0 .. 2^(e+m) - 1 of a float format without inf / nan (index == bits)."""
    bias = 2 ** (ebits - 1) - 1
    out = []
    for e in range(2 ** ebits):
        for m in range(2 ** mbits):
            out.append((m / 2 ** mbits) * 2.0 ** (1 - bias) if e == 0 else (1 + m / 2 ** mbits) * 2.0 ** (e - bias))
    return torch.tensor(out, dtype=torch.float32)


def _block_exponent(amax, fmax):
    """Smallest power-of-two exponent e with amax / 2^e <= fmax (so no element saturates)."""
    e = torch.ceil(torch.log2(torch.clamp(amax, min=1e-30) / fmax))
    e = torch.where(amax > 0, e, torch.full_like(e, -127.0)).clamp(-127, 127)
    over = amax * torch.exp2(-e) > fmax
    return (e + over.to(e.dtype)).clamp(-127, 127)


def _encode(v, fmt):
    """Scaled values (|v| <= max) -> integer codes (sign | magnitude bits), nearest, ties to even code."""
    code, eb, mb, bits, _ = FORMATS[fmt]
    if bits == 8:
        return v.to(torch.float8_e4m3fn).view(torch.uint8).to(torch.int32)
    tab = _values(eb, mb).to(v.device)
    mid = (tab[1:] + tab[:-1]) / 2
    a = v.abs()
    mag = torch.bucketize(a, mid)  # ties go to the lower code; move exact-tie odd codes up to even
    tie = (mag < len(tab) - 1) & (a == mid[mag.clamp(max=len(mid) - 1)]) & (mag % 2 == 1)
    mag = mag + tie.to(mag.dtype)
    return ((v < 0).to(torch.int32) << (bits - 1)) | mag.to(torch.int32)


def _decode(codes, fmt):
    code, eb, mb, bits, _ = FORMATS[fmt]
    c = codes.to(torch.int64)
    if bits == 8:
        return c.to(torch.uint8).view(torch.float8_e4m3fn).float()
    mag = _values(eb, mb).to(codes.device)[c & ((1 << (bits - 1)) - 1)]
    return torch.where((c >> (bits - 1)) & 1 == 1, -mag, mag)


def pack(codes, bits):
    """[R, K] integer codes -> [R, K * bits / 8] uint8 in the MFMA's contiguous bit order."""
    R, K = codes.shape
    c = codes.to(torch.int64)
    if bits == 8:
        return c.to(torch.uint8).contiguous()
    if bits == 4:
        c = c.reshape(R, K // 2, 2)
        return (c[..., 0] | (c[..., 1] << 4)).to(torch.uint8).contiguous()
    c = c.reshape(R, K // 4, 4)
    v = c[..., 0] | (c[..., 1] << 6) | (c[..., 2] << 12) | (c[..., 3] << 18)
    return torch.stack([v & 0xFF, (v >> 8) & 0xFF, (v >> 16) & 0xFF], -1).reshape(R, K * 3 // 4).to(torch.uint8)


def unpack(packed, bits, K):
    R = packed.shape[0]
    p = packed.to(torch.int64)
    if bits == 8:
        return p
    if bits == 4:
        return torch.stack([p & 0xF, p >> 4], -1).reshape(R, K)
    p = p.reshape(R, K // 4, 3)
    v = p[..., 0] | (p[..., 1] << 8) | (p[..., 2] << 16)
    return torch.stack([(v >> (6 * j)) & 0x3F for j in range(4)], -1).reshape(R, K)


def quantize(x, fmt):
    """x [R, K] (K % 32 == 0) -> (packed codes uint8 [R, K * bits / 8], E8M0 exponents uint8 [R, K / 32])."""
    code, _, _, bits, fmax = FORMATS[fmt]
    R, K = x.shape
    assert K % BLOCK == 0, "MX quantisation needs K % 32 == 0"
    g = x.float().reshape(R, K // BLOCK, BLOCK)
    e = _block_exponent(g.abs().amax(-1), fmax)
    codes = _encode(g * torch.exp2(-e)[..., None], fmt).reshape(R, K)
    return pack(codes, bits), (e + 127).to(torch.uint8)


def dequantize(packed, scales, fmt, K):
    """Inverse of ``quantize``: fp32 [R, K]."""
    bits = FORMATS[fmt][3]
    v = _decode(unpack(packed, bits, K), fmt).reshape(packed.shape[0], K // BLOCK, BLOCK)
    return (v * torch.exp2(scales.float() - 127.0)[..., None]).reshape(packed.shape[0], K)


def quantize_act(x):
    """Activations [M, K] -> MXFP8 (codes, exponents): the HIP pass on the GPU, PyTorch on the CPU."""
    if x.is_cuda and native.use_hip(x):
        q, s = torch.ops.sxe.mx_quant_fp8(x.to(torch.bfloat16).contiguous())
        return q, s
    return quantize(x.to(torch.bfloat16).float(), "mxfp8")


def mx_linear(x, wq, ws, fmt, bias=None, col_scale=None):
    """y = MXFP8(x) @ MX(wq, ws)^T (+ bias) (* col_scale), bf16 out. x [..., K]; wq/ws from ``quantize``."""
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    N = ws.shape[0]
    if x2.is_cuda:
        native.require_hip()
        q, s = torch.ops.sxe.mx_quant_fp8(x2.to(torch.bfloat16).contiguous())
        b = bias.to(torch.bfloat16).contiguous() if bias is not None else None
        y = torch.ops.sxe.mx_gemm(q, s, wq, ws, FORMATS[fmt][0], b, col_scale)
    else:
        q, s = quantize(x2.to(torch.bfloat16).float(), "mxfp8")
        y = dequantize(q, s, "mxfp8", K) @ dequantize(wq, ws, fmt, K).t()
        if col_scale is not None:
            y = y * col_scale.float()
        if bias is not None:
            y = y + bias.float()
        y = y.to(torch.bfloat16)
    return y.view(*x.shape[:-1], N)


class MXWeight:
    """A linear layer's weight [N, K] in an OCP-MX format (``mxfp8`` / ``mxfp6`` / ``mxfp6_e2m3`` /
    ``mxfp4``), K % 128 == 0 and N % 128 == 0 for the GPU kernels. ``linear``: decode-sized inputs
    run weight-only (bf16 activations) on the skinny dequantising kernel; prefill-sized inputs are
    quantised to MXFP8 for the block-scaled MFMA GEMM (W{8,6,4}A8). HBM holds bits/8 bytes per
    weight plus one exponent byte per 32."""

    def __init__(self, w, fmt="mxfp6"):
        assert fmt in FORMATS, f"MX format {fmt!r}: one of {sorted(FORMATS)}"
        N, K = w.shape
        assert K % 128 == 0, "MXWeight: in_features must be a multiple of 128"
        self.fmt, self.shape, self.dtype = fmt, (N, K), w.dtype
        self.q, self.scale = quantize(w.detach(), fmt)

    @property
    def nbytes(self):
        return self.q.numel() + self.scale.numel()

    def dequantize(self, dtype=torch.bfloat16):
        return dequantize(self.q, self.scale, self.fmt, self.shape[1]).to(dtype)

    def linear(self, x, bias=None):
        """<= 16 rows (decode): weight-only, bf16 activations, the codes decoded in registers by the
        skinny kernel (csrc/kernels/skinny_dq.hip) -- HBM streams bits/8 bytes per weight. More
        rows: MXFP8 activations x MX weights on the block-scaled matrix cores (``mx_linear``)."""
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if (x2.is_cuda and self.fmt in _SKINNY and 0 < x2.shape[0] <= 16 and x2.dtype == torch.bfloat16
                and x2.stride(-1) == 1 and x2.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0):
            native.require_hip()
            b = bias.to(torch.bfloat16).contiguous() if bias is not None else None
            y = torch.ops.sxe.skinny_gemm_dq(x2, self.q, self.scale, FORMATS[self.fmt][0], 32, b)
            return y.view(*x.shape[:-1], self.shape[0])
        return mx_linear(x, self.q, self.scale, self.fmt, bias).to(x.dtype)

    def to(self, device):
        self.q, self.scale = self.q.to(device), self.scale.to(device)
        return self


class MXLinear(torch.nn.Module):
    """Inference ``nn.Linear`` replacement holding an ``MXWeight``."""

    def __init__(self, linear: torch.nn.Linear, fmt="mxfp6"):
        super().__init__()
        w = MXWeight(linear.weight.detach(), fmt)
        self.fmt = fmt
        self.register_buffer("weight_q", w.q)
        self.register_buffer("weight_scale", w.scale)
        self.bias = linear.bias
        self.in_features, self.out_features = linear.in_features, linear.out_features

    def forward(self, x):
        return mx_linear(x, self.weight_q, self.weight_scale, self.fmt, self.bias).to(x.dtype)
