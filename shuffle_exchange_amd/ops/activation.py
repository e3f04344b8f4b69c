"""Gated (SwiGLU/GeGLU/ReGLU) and bias+activation ops with HIP forward/backward kernels.

Training layout for the gated MLP: the gate and up projections are ONE GEMM producing
``[T, 2I] = [gate | up]``; ``swiglu(gu)`` returns ``silu(gate) * up``.
"""
import torch
import torch.nn.functional as F

from . import native

ACT = {"identity": 0, "relu": 1, "gelu": 2, "silu": 3, "gelu_exact": 4, "quick_gelu": 5,
       # HF activation names
       "gelu_new": 2, "gelu_pytorch_tanh": 2, "gelu_fast": 2, "swish": 3}


def _act_ref(x, act):
    if act == 1:
        return F.relu(x)
    if act == 2:
        return F.gelu(x, approximate="tanh")
    if act == 3:
        return F.silu(x)
    if act == 4:
        return F.gelu(x)
    if act == 5:
        return x * torch.sigmoid(1.702 * x)
    return x


class _Gated(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, act):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        ctx.act = act
        return torch.ops.sxe.gated_act_fwd(gu, act)

    @staticmethod
    def backward(ctx, dout):
        (gu,) = ctx.saved_tensors
        return torch.ops.sxe.gated_act_bwd(dout.contiguous(), gu, ctx.act), None


def gated_act(gu, act="silu"):
    a = ACT[act] if isinstance(act, str) else int(act)
    if native.use_hip(gu):
        return _Gated.apply(gu, a)
    g, u = gu.chunk(2, dim=-1)
    return (_act_ref(g.float(), a) * u.float()).to(gu.dtype)


def swiglu(gu):
    return gated_act(gu, "silu")


class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, act):
        x = x.contiguous()
        ctx.save_for_backward(x, bias)
        ctx.act = act
        return torch.ops.sxe.bias_act_fwd(x, bias, act)

    @staticmethod
    def backward(ctx, dy):
        x, bias = ctx.saved_tensors
        dx = torch.ops.sxe.bias_act_bwd(dy.contiguous(), x, bias, ctx.act)
        db = dx.view(-1, dx.shape[-1]).float().sum(0).to(bias.dtype) if bias is not None else None
        return dx, db, None


def bias_act(x, bias=None, act="gelu"):
    a = ACT[act] if isinstance(act, str) else int(act)
    if native.use_hip(x) and x.shape[-1] % 8 == 0:
        return _BiasAct.apply(x, bias, a)
    y = x.float() + (bias.float() if bias is not None else 0.0)
    return _act_ref(y, a).to(x.dtype)


def bias_gelu(x, bias=None):
    return bias_act(x, bias, "gelu")
