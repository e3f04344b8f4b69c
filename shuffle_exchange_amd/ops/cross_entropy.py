"""Softmax cross-entropy for LM heads (HIP kernels).

``cross_entropy(logits, target)`` -- standard autograd op (fwd saves lse; bwd writes grads).
``fused_linear_cross_entropy(h, W, target)`` -- LM head + loss in one autograd node: the logits
buffer is overwritten in place with d(loss)/d(logits) during the forward (loss is the graph's
terminal node, so the gradient is known up to the scalar upstream factor), the backward is just two
GEMMs. Peak memory is one bf16 [T, V] buffer instead of logits + fp32 softmax + grad, and
``chunk_tokens`` bounds even that (ALST's TiledLoss, reference
runtime/sequence_parallel/ulysses_sp.py:915, plays the same role). On bf16 GPU training steps whose
shapes fit its tile, the gradient is instead written in the backward by ``xent_grad_dual``
(token-major over the logits + vocab-major copy for the TN weight-gradient GEMM, upstream scalar
folded in).
"""
import os

import torch
import torch.nn.functional as F

from . import native


class _XEnt(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index):
        logits2 = logits.contiguous().view(-1, logits.shape[-1])
        loss, lse = torch.ops.sxe.xent_fwd(logits2, target.reshape(-1).contiguous(), int(ignore_index), False, None, 1.0)
        ctx.save_for_backward(logits2, target.reshape(-1).contiguous(), lse)
        ctx.ignore_index = ignore_index
        ctx.shape = logits.shape
        return loss.view(logits.shape[:-1])

    @staticmethod
    def backward(ctx, dloss):
        logits2, target, lse = ctx.saved_tensors
        g = torch.ops.sxe.xent_bwd(logits2, target, lse, dloss.reshape(-1).float().contiguous(), int(ctx.ignore_index),
                                   False)
        return g.view(ctx.shape), None, None


def cross_entropy(logits, target, ignore_index=-100, reduction="mean"):
    if native.use_hip(logits):
        per_tok = _XEnt.apply(logits, target, ignore_index)
    else:
        per_tok = F.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), target.reshape(-1),
                                  ignore_index=ignore_index, reduction="none").view(target.shape)
    if reduction == "none":
        return per_tok
    if reduction == "sum":
        return per_tok.sum()
    n = (target != ignore_index).sum().clamp_min(1)
    return per_tok.sum() / n


DUAL = os.environ.get("SXE_XENT_DUAL", "1") == "1"


def _dual_ok(h2, weight):
    """The dual-layout gradient path applies: bf16 GPU operands, tokens % 64, vocab % 256, hidden % 64
    (the kernel's tile and the transpose kernel's)."""
    return (DUAL and h2.is_cuda and h2.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and weight.dim() == 2 and h2.shape[0] % 64 == 0 and h2.shape[0] > 0 and weight.shape[0] % 256 == 0
            and h2.shape[1] % 64 == 0 and h2.is_contiguous() and native.use_hip(h2))


class _FusedLinearXEnt(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, weight, target, ignore_index, chunk_tokens, reduction="mean"):
        H = h.shape[-1]
        h2 = h.reshape(-1, H)
        tgt = target.reshape(-1).contiguous()
        T = h2.shape[0]
        if reduction == "sum":
            n_valid = torch.ones((), device=h.device, dtype=torch.float32)
        else:
            n_valid = (tgt != ignore_index).sum().clamp_min(1).float()
        inv_n = (1.0 / n_valid).reshape(1)
        need_grad = torch.is_grad_enabled() or h.requires_grad or weight.requires_grad
        chunk = T if not chunk_tokens else min(int(chunk_tokens), T)
        if chunk == T and need_grad and _dual_ok(h2, weight):
            # dual layout: the forward computes only loss + lse; the backward writes the scaled
            # gradient over the logits AND its vocab-major transpose in one pass (xent_grad_dual),
            # so the LM-head weight gradient is a TN GEMM with no transpose of the 4 GB gradient
            logits = torch.matmul(h2, weight.t())
            loss, lse = torch.ops.sxe.xent_fwd(logits, tgt, int(ignore_index), False, None, 1.0)
            ctx.save_for_backward(logits, lse, tgt, inv_n, h2, weight)
            ctx.mode = "dual"
            ctx.ignore_index = int(ignore_index)
            ctx.hshape = h.shape
            return loss.sum() / n_valid
        if chunk == T:
            # unchunked: keep d(loss)/d(logits) (written over the logits) and do both GEMMs in
            # backward, where the weight-grad GEMM can land directly in the optimizer's buffer
            logits = torch.matmul(h2, weight.t())
            loss, _ = torch.ops.sxe.xent_fwd(logits, tgt, int(ignore_index), need_grad, inv_n, 1.0)
            ctx.save_for_backward(logits if need_grad else None, h2, weight)
            ctx.mode = "dlogits"
            ctx.hshape = h.shape
            return loss.sum() / n_valid
        ctx.mode = "chunked"
        loss_sum = torch.zeros((), device=h.device, dtype=torch.float32)
        dh = torch.empty_like(h2) if need_grad else None
        dW = None
        for s in range(0, T, chunk):
            e = min(T, s + chunk)
            logits = torch.matmul(h2[s:e], weight.t())
            loss, _ = torch.ops.sxe.xent_fwd(logits, tgt[s:e], int(ignore_index), need_grad, inv_n, 1.0)
            loss_sum = loss_sum + loss.sum()
            if need_grad:
                torch.matmul(logits, weight, out=dh[s:e])
                part = torch.matmul(logits.t(), h2[s:e])
                if dW is None:
                    dW = part if chunk == T else part.float()
                else:
                    dW.add_(part.float())
            del logits
        ctx.save_for_backward(dh, dW)
        ctx.wdtype = weight.dtype
        ctx.hshape = h.shape
        return loss_sum / n_valid

    @staticmethod
    def backward(ctx, gout):
        if ctx.mode == "dual":
            logits, lse, tgt, inv_n, h2, weight = ctx.saved_tensors
            gT = torch.ops.sxe.xent_grad_dual(logits, tgt, lse, ctx.ignore_index, inv_n,
                                              gout.detach().float().reshape(1).contiguous())
            from .linear import data_grad
            from .mlp import weight_grad_tn
            dh = data_grad(logits, weight).view(ctx.hshape)  # logits now hold the gradient
            del logits
            dW = None
            if ctx.needs_input_grad[1]:
                dW = weight_grad_tn(weight, gT, torch.ops.sxe.transpose16(h2))
            return dh, dW, None, None, None, None
        if ctx.mode == "dlogits":
            dl, h2, weight = ctx.saved_tensors
            dl.mul_(gout.to(dl.dtype))  # upstream scalar (1/GAS, loss scale, ...), in place
            from .linear import data_grad, write_weight_grad
            dh = data_grad(dl, weight).view(ctx.hshape)
            dW = None
            if ctx.needs_input_grad[1]:
                if not write_weight_grad(weight, dl, h2):
                    dW = dl.t() @ h2
            return dh, dW, None, None, None, None
        dh, dW = ctx.saved_tensors
        g = gout.to(torch.float32)
        dh = (dh * g.to(dh.dtype)).view(ctx.hshape)
        dW = (dW * g.to(dW.dtype)).to(ctx.wdtype)
        return dh, dW, None, None, None, None


def fused_linear_cross_entropy(h, weight, target, ignore_index=-100, chunk_tokens=None, reduction="mean"):
    """CE of ``h @ weight.T`` against ``target`` (ignore_index excluded); mean or sum."""
    if native.use_hip(h):
        return _FusedLinearXEnt.apply(h, weight, target, ignore_index, chunk_tokens, reduction)
    logits = torch.matmul(h, weight.t()).float()
    return F.cross_entropy(logits.reshape(-1, logits.shape[-1]), target.reshape(-1), ignore_index=ignore_index,
                           reduction=reduction)
