"""Fused SwiGLU MLP for training on gfx950: ``down(silu(gate) * up)`` with ``[gate | up]`` as ONE
projection, arranged so every weight-gradient GEMM runs in hipBLASLt's fast K-contiguous layout.

Why: dW = dY^T X reduces over tokens, the ROW index of both token-major operands. hipBLASLt runs
that "NT" product -- and this repo's hand-written k-major kernel (csrc/kernels/gemm_wgrad.hip) --
at 1.06-1.18 PF on MI355X, while the same product with both operands token-minor ("TN", the
forward layout) runs at 1.34-1.48 PF (tools/wgrad_tn16k_exp.py, 16,384 tokens). Making the
token-minor copies with a separate transpose costs as much HBM time as it saves, so the producers
write them:

* forward: the dual-layout gated kernel (csrc/kernels/act.hip ``gated_act_fwd_dual``) writes h for
  the down projection AND h^T, which is what backward keeps (h itself is dropped after the GEMM --
  the same saved bytes as before);
* backward: ``gated_act_bwd_dual`` writes dgu for the gate|up data-gradient GEMM AND dgu^T for its
  weight gradient, from the same registers/LDS tile;
* the two small operands (the MLP input x^T, saved instead of x, and dOut^T) go through the
  HBM-speed transpose kernel.

Each weight gradient is a bf16 TN GEMM (as autograd's own bf16 weight gradients are) added into
the ZeRO fp32 accumulator, or written straight into a bf16 reduce-scatter slot. The measured
alternatives (fp32-out TN with beta = 1; the k-major kernel) lose at these shapes: the fp32-out
GEMM cost the whole Llama-3-8B step 2.8 % (24,602 vs 25,302 tokens/s in one box session,
profiles/r05/headline_wgrad_norm_ab.log) although it drops the cast / add passes.
Reference counterpart: the MLP of deepspeed/model_implementations / the HF Llama MLP the reference
trains through autograd (no fused MLP exists there); parity is autograd's result (tests/test_mlp_tn.py).
"""
import os

import torch
import torch.nn.functional as F

from . import native
from .linear import Linear, data_grad

ACT_SILU = 3
ENABLED = os.environ.get("SXE_MLP_TN", "1") == "1"


def dual_variant(inter):
    """Tile of the dual-layout gated kernels: 64 tokens x 256 columns where the intermediate size
    allows (5.0-5.2 TB/s at 16k tokens x 14336 vs 4.1 TB/s for 64 x 64 tiles, profiles/act_layout_exp.log),
    else 64 x 128, else 64 x 64."""
    return 4 if inter % 256 == 0 else 1 if inter % 128 == 0 else 0


STASH = os.environ.get("SXE_WGRAD_STASH", "1") == "1"


def _may_stash(w, gyT):
    """The optimizer lets this micro-step's weight gradient be written late (``_sxe_grad_defer``:
    before the accumulation boundary, single-rank fp32 accumulator) and the pair kernel applies."""
    defer = getattr(w, "_sxe_grad_defer", None)
    return STASH and defer is not None and gyT.is_cuda and gyT.dtype == torch.bfloat16 and defer(w)


def flush_stashed_wgrad(w):
    """Write a stashed bf16 weight gradient that no later micro-step consumed (the parameter got no
    gradient at the accumulation boundary) into the optimizer's target."""
    stash = w.__dict__.pop("_sxe_bstash", None)
    if stash is None:
        return
    buf, accumulate = w._sxe_grad_target(w)
    b2 = buf.view(w.shape)
    b2.add_(stash) if accumulate else b2.copy_(stash)
    w._sxe_grad_done(w)


def drop_stashed_wgrad(w):
    """zero_grad before the boundary: the partial accumulation is discarded with the rest."""
    w.__dict__.pop("_sxe_bstash", None)


def weight_grad_tn(w, gyT, xT, fp32_out=False):
    """dW = gyT @ xT^T (gyT [N, T], xT [K, T], both token-minor): written into the optimizer's
    target for ``w`` when it has one (returns None), else returned. ``fp32_out``: an fp32
    accumulator takes ONE fp32-output GEMM with beta = 1 instead of bf16 GEMM + add (faster for the
    fused QKV projection: 0.62 vs 0.73 ms at 16k tokens, profiles/r06/wgrad_variants_16k.log)."""
    from .linear import grad_target
    tgt = grad_target(w)
    dw = None
    if tgt is None:
        return torch.mm(gyT, xT.t())
    stash = w.__dict__.pop("_sxe_bstash", None)
    if stash is None and not fp32_out and _may_stash(w, gyT):
        # before the accumulation boundary of a single-rank unit: keep this micro-step's bf16 product
        # and fold it into the accumulator together with the next one (acc2_bf16_: one fp32 pass
        # for the pair instead of one per micro-step); _sxe_grad_done runs with that write
        w.__dict__["_sxe_bstash"] = torch.mm(gyT, xT.t())
        return None
    buf, accumulate = tgt(w)
    if stash is not None:
        dw = torch.mm(gyT, xT.t())
        if buf.dtype == torch.float32 and buf.is_contiguous():
            torch.ops.sxe.acc2_bf16_(buf, stash, dw.view_as(stash), bool(accumulate))
        else:
            b2 = buf.view(w.shape)
            b2.add_(stash) if accumulate else b2.copy_(stash)
            b2.add_(dw)
        w._sxe_grad_done(w)
        return None
    if buf.dtype == gyT.dtype and not accumulate and buf.is_contiguous():
        torch.mm(gyT, xT.t(), out=buf.view(w.shape))  # bf16 reduce-scatter slot of a multi-rank unit
    elif fp32_out and buf.dtype == torch.float32 and buf.is_contiguous():
        b2 = buf.view(w.shape)
        torch.ops.aten.addmm.dtype_out(b2, gyT, xT.t(), torch.float32, beta=1 if accumulate else 0, alpha=1, out=b2)
    else:
        dw = torch.mm(gyT, xT.t()).view_as(buf)
        buf.add_(dw) if accumulate else buf.copy_(dw)
    w._sxe_grad_done(w)
    return None


class _SwiGLUMLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wgu, wd):
        x2 = x.reshape(-1, x.shape[-1])
        gu = F.linear(x2, wgu)
        v = dual_variant(wd.shape[1])
        h, hT = torch.ops.sxe.gated_act_fwd_dual(gu, ACT_SILU, v)
        out = F.linear(h, wd)
        del h
        xT = torch.ops.sxe.transpose16(x2) if ctx.needs_input_grad[1] else None
        ctx.save_for_backward(xT, gu, hT, wgu, wd)
        ctx.x_shape, ctx.variant = x.shape, v
        return out.view(*x.shape[:-1], wd.shape[0])

    @staticmethod
    def backward(ctx, dout):
        xT, gu, hT, wgu, wd = ctx.saved_tensors
        d2 = dout.reshape(-1, dout.shape[-1]).contiguous()
        dwd = dwgu = dx = None
        dh = data_grad(d2, wd)
        if ctx.needs_input_grad[2]:
            dwd = weight_grad_tn(wd, torch.ops.sxe.transpose16(d2), hT)
        del hT
        dgu, dguT = torch.ops.sxe.gated_act_bwd_dual(dh, gu, ACT_SILU, ctx.variant)
        del dh
        if ctx.needs_input_grad[0]:
            dx = data_grad(dgu, wgu).view(ctx.x_shape)
        del dgu
        if ctx.needs_input_grad[1]:
            dwgu = weight_grad_tn(wgu, dguT, xT)
        return dx, dwgu, dwd


def _plain(lin):
    return (type(lin) is Linear and lin.bias is None and isinstance(lin.weight, torch.Tensor)
            and lin.weight.dtype == torch.bfloat16 and lin.weight.dim() == 2 and lin.weight.is_contiguous())


def fused_ok(x, gate_up, down):
    """The fused path applies: GPU bf16 training step, plain (not TP / LoRA / quantized) bias-free
    projections, token count and widths multiples of 64 (the dual kernels' tile)."""
    if not (ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and torch.is_grad_enabled()):
        return False
    if not (_plain(gate_up) and _plain(down)):
        return False
    wgu, wd = gate_up.weight, down.weight
    if not (wgu.requires_grad or wd.requires_grad or x.requires_grad):
        return False
    T = x.numel() // x.shape[-1]
    H, I2 = wgu.shape[1], wgu.shape[0]
    return (T % 64 == 0 and T > 0 and H % 64 == 0 and I2 % 128 == 0 and wd.shape == (H, I2 // 2)
            and x.shape[-1] == H and native.use_hip(x))


def swiglu_mlp(x, gate_up, down):
    """``down(swiglu(gate_up(x)))`` for two ops.linear.Linear modules (fused when ``fused_ok``)."""
    if fused_ok(x, gate_up, down):
        return _SwiGLUMLP.apply(x, gate_up.weight, down.weight)
    from .activation import swiglu
    return down(swiglu(gate_up(x)))
