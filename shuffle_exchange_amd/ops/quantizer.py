"""Group-wise quantization (int8 / int4 symmetric, FP8 e4m3) -- HIP kernels in quant.hip.

Parity: reference ops/quantizer (``ds_quantize_*``), ZeRO++ ``CUDAQuantizer``
(runtime/zero/partition_parameters.py:824-863), ops/fp_quantizer (``FP_Quantize.quantize /
dequantize``). Every op has a PyTorch reference used on CPU and as the test oracle.
"""
import torch

from . import native


def _ref_quant(x, group, bits):
    xf = x.float().reshape(-1, group)
    qmax = 127.0 if bits == 8 else 7.0
    m = xf.abs().amax(1)
    s = torch.where(m > 0, m / qmax, torch.ones_like(m))
    q = torch.clamp(torch.round(xf / s[:, None]), -qmax, qmax).to(torch.int32).reshape(-1)
    if bits == 8:
        return q.to(torch.int8).view(torch.uint8), s
    lo, hi = q[0::2] & 0xF, q[1::2] & 0xF
    return (lo | (hi << 4)).to(torch.uint8), s


def _ref_dequant(q, scales, group, bits, n, dtype):
    if bits == 8:
        v = q.view(torch.int8).float()
    else:
        b = q.to(torch.int32)
        lo, hi = b & 0xF, (b >> 4) & 0xF
        v = torch.stack([lo, hi], 1).reshape(-1)
        v = torch.where(v >= 8, v - 16, v).float()
    return (v[:n].reshape(-1, group) * scales.reshape(-1, 1)).reshape(-1).to(dtype)


def quantize(x, group_size=128, bits=8):
    """x (any shape, numel % group_size == 0) -> (packed uint8, fp32 scales [numel/group])."""
    x = x.contiguous().reshape(-1)
    if native.use_hip(x):
        q, s = torch.ops.sxe.quantize_sym(x, int(group_size), int(bits))
        return q, s
    return _ref_quant(x, group_size, bits)


def dequantize(q, scales, group_size=128, bits=8, out=None, numel=None, dtype=torch.bfloat16):
    n = out.numel() if out is not None else (numel if numel is not None else scales.numel() * group_size)
    if out is None:
        out = torch.empty(n, dtype=dtype, device=q.device)
    if native.use_hip(q):
        torch.ops.sxe.dequantize_sym_(q, scales, int(group_size), int(bits), out.reshape(-1))
        return out
    out.reshape(-1).copy_(_ref_dequant(q, scales, group_size, bits, n, out.dtype))
    return out


def dequant_reduce(q, scales, W, group_size, bits, out, alpha=1.0, accumulate=False):
    """out (fp32 [m]) (+)= alpha * sum_w dequant(q[w]) for W equal quantized chunks."""
    m = out.numel()
    if native.use_hip(q):
        torch.ops.sxe.dequant_reduce_(q, scales, int(W), int(group_size), int(bits), out, float(alpha),
                                      bool(accumulate))
        return out
    per = m if bits == 8 else m // 2
    acc = sum(_ref_dequant(q[w * per:(w + 1) * per], scales[w * (m // group_size):(w + 1) * (m // group_size)],
                           group_size, bits, m, torch.float32) for w in range(W))
    if accumulate:
        out.add_(acc, alpha=alpha)
    else:
        out.copy_(acc * alpha)
    return out


def loco_quantize(x, err, err_beta, group_size=128, bits=8):
    """LoCo error-feedback quantization (reference runtime/comm/coalesced_collectives.py
    ``all_to_all_loco_quant_reduce`` / ``loco_swizzle_quant``): quantize x + err_beta * err and
    return (q, scales, new_err) with new_err = compensated - dequant(q) (fp32)."""
    comp = x.float().reshape(-1) if err is None else x.float().reshape(-1).add(err.float().reshape(-1), alpha=err_beta)
    q, sc = quantize(comp, group_size, bits)
    deq = dequantize(q, sc, group_size, bits, numel=comp.numel(), dtype=torch.float32)
    return q, sc, comp - deq


def quantize_fp8(x, group_size=128):
    x = x.contiguous().reshape(-1)
    if native.use_hip(x):
        q, s = torch.ops.sxe.quantize_fp8(x, int(group_size))
        return q, s
    xf = x.float().reshape(-1, group_size)
    m = xf.abs().amax(1)
    s = torch.where(m > 0, m / 448.0, torch.ones_like(m))
    q = (xf / s[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8).reshape(-1)
    return q, s


def dequantize_fp8(q, scales, group_size=128, out=None, dtype=torch.bfloat16):
    n = q.numel()
    if out is None:
        out = torch.empty(n, dtype=dtype, device=q.device)
    if native.use_hip(q):
        torch.ops.sxe.dequantize_fp8_(q, scales, int(group_size), out.reshape(-1))
        return out
    v = q.view(torch.float8_e4m3fn).float().reshape(-1, group_size) * scales.reshape(-1, 1)
    out.reshape(-1).copy_(v.reshape(-1))
    return out


def __getattr__(name):  # FP_Quantize lives in ops/fp_quantizer.py (FP8/FP6/FP4)
    if name == "FP_Quantize":
        from .fp_quantizer import FP_Quantize
        return FP_Quantize
    raise AttributeError(name)
