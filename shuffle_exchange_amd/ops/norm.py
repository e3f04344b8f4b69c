"""RMSNorm / LayerNorm with an optional fused residual add (HIP kernels, autograd-aware).

``rms_norm(x, w, eps, residual=r)`` returns ``(y, h)`` with ``h = x + r`` (the new residual
stream) and ``y = rmsnorm(h) * w`` -- the "pre-RMS" fusion of the reference's inference kernel
(deepspeed/inference/v2/kernels/core_ops/cuda_rms_norm/rms_norm_cuda.cu:84), here with a backward.
"""
import torch
import torch.nn as nn

from . import native


def _ref_norm(x, w, b, eps, layernorm):
    xf = x.float()
    if layernorm:
        mean = xf.mean(-1, keepdim=True)
        var = (xf - mean).pow(2).mean(-1, keepdim=True)
        y = (xf - mean) * torch.rsqrt(var + eps) * w.float()
        if b is not None:
            y = y + b.float()
    else:
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype)


class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps, layernorm):
        shape = x.shape
        x2 = x.contiguous().view(-1, shape[-1])
        r2 = residual.contiguous().view(-1, shape[-1]) if residual is not None else None
        y, rstd, mean, h = torch.ops.sxe.norm_fwd(x2, r2, weight, bias, float(eps), bool(layernorm))
        hin = h if residual is not None else x2
        ctx.save_for_backward(hin, rstd, mean if layernorm else None, weight)
        ctx.layernorm = layernorm
        ctx.has_res = residual is not None
        ctx.has_bias = bias is not None
        ctx.shape = shape
        y = y.view(shape)
        if residual is not None:
            return y, h.view(shape)
        return y, None

    @staticmethod
    def backward(ctx, dy, dh):
        hin, rstd, mean, weight = ctx.saved_tensors
        H = ctx.shape[-1]
        dy2 = dy.contiguous().view(-1, H)
        dres = dh.contiguous().view(-1, H) if (ctx.has_res and dh is not None) else None
        dx, dw, db = torch.ops.sxe.norm_bwd(dy2, hin, rstd, mean, weight, dres, bool(ctx.layernorm))
        dx = dx.view(ctx.shape)
        from .linear import grad_target
        tgt_fn = grad_target(weight)
        if tgt_fn is not None and ctx.needs_input_grad[2]:
            # the fp32 dgamma goes straight into the optimizer's buffer (no bf16 round trip, no
            # mixed-dtype accumulate in a hook)
            tgt, acc = tgt_fn(weight)
            (tgt.view(-1).add_ if acc else tgt.view(-1).copy_)(dw.view(-1))
            weight._sxe_grad_done(weight)
            dw = None
        else:
            dw = dw.to(weight.dtype)
        db = db.to(weight.dtype) if ctx.has_bias else None
        return dx, (dx if ctx.has_res else None), dw, db, None, None


def rms_norm(x, weight, eps=1e-6, residual=None):
    """Returns y (and the new residual h = x + residual when ``residual`` is given)."""
    if native.use_hip(x):
        y, h = _NormFn.apply(x, residual, weight, None, eps, False)
        return (y, h) if residual is not None else y
    h = x + residual if residual is not None else x
    y = _ref_norm(h, weight, None, eps, False)
    return (y, h) if residual is not None else y


def layer_norm(x, weight, bias=None, eps=1e-5, residual=None):
    if native.use_hip(x):
        y, h = _NormFn.apply(x, residual, weight, bias, eps, True)
        return (y, h) if residual is not None else y
    h = x + residual if residual is not None else x
    y = _ref_norm(h, weight, bias, eps, True)
    return (y, h) if residual is not None else y


class RMSNorm(nn.Module):
    def __init__(self, dim, eps=1e-6, dtype=None, device=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim, dtype=dtype, device=device))

    def forward(self, x, residual=None):
        return rms_norm(x, self.weight, self.eps, residual)


class LayerNorm(nn.Module):
    def __init__(self, dim, eps=1e-5, bias=True, dtype=None, device=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim, dtype=dtype, device=device))
        self.bias = nn.Parameter(torch.zeros(dim, dtype=dtype, device=device)) if bias else None

    def forward(self, x, residual=None):
        return layer_norm(x, self.weight, self.bias, self.eps, residual)
