"""Evoformer attention with pair / mask biases (reference ops/deepspeed4science/evoformer_attn.py:
``DS4Sci_EvoformerAttention`` over a CUTLASS kernel, not in the snapshot).

O = softmax(Q K^T / sqrt(D) + bias1 + bias2) V with Q/K/V [B, N, L, H, D], bias1 [B, N, 1, 1, L]
(MSA row mask) and bias2 [B, 1, H, L, L] (pair bias), gradients for Q, K, V and both biases.

GPU (bf16, head dim 32 / 64): the fused gfx950 flash kernels of csrc/kernels/evoformer.hip --
biases added inside the online softmax, no L x L matrix materialised, dbias1 / dbias2 accumulated
by the dK/dV kernel. Elsewhere (CPU, other dtypes / head dims): a query-chunked PyTorch computation
(each chunk recomputed in the backward, so only one chunk's L x L probabilities are ever live).
Parity with the CUTLASS kernel is unpinned (not vendored); the tests check the exact formula.
"""
import math

import torch
from torch.utils.checkpoint import checkpoint

from .. import native

CHUNK = 256


def _chunk_attn(q, k, v, b1, b2, scale):
    # q [B, N, c, H, D] -> [B, N, H, c, D]
    qh, kh, vh = q.transpose(-2, -3), k.transpose(-2, -3), v.transpose(-2, -3)
    s = torch.matmul(qh.float(), kh.float().transpose(-1, -2)) * scale
    if b1 is not None:
        s = s + b1.float()
    if b2 is not None:
        s = s + b2.float()
    p = torch.softmax(s, dim=-1)
    return torch.matmul(p, vh.float()).to(q.dtype).transpose(-2, -3)


def evoformer_attention(Q, K, V, bias1=None, bias2=None, chunk=CHUNK):
    if _hip_ok(Q, K, V):
        return EvoformerFusedAttention.apply(Q, K, V, bias1, bias2)
    scale = 1.0 / math.sqrt(Q.shape[-1])
    L = Q.shape[-3]
    outs = []
    for c0 in range(0, L, chunk):
        q = Q[..., c0:c0 + chunk, :, :]
        b2 = bias2[..., c0:c0 + chunk, :] if bias2 is not None else None
        if torch.is_grad_enabled() and (Q.requires_grad or K.requires_grad or V.requires_grad):
            outs.append(checkpoint(_chunk_attn, q, K, V, bias1, b2, scale, use_reentrant=False))
        else:
            outs.append(_chunk_attn(q, K, V, bias1, b2, scale))
    return torch.cat(outs, dim=-3)


def _hip_ok(Q, K, V):
    return (Q.is_cuda and native.use_hip(Q) and Q.dtype == torch.bfloat16 and Q.shape[-1] in (32, 64)
            and Q.shape == K.shape == V.shape and Q.shape[-3] > 0)


class EvoformerFusedAttention(torch.autograd.Function):
    """Fused HIP forward / backward (evoformer.hip); returns dbias1 / dbias2 in the bias dtypes."""

    @staticmethod
    def forward(ctx, q, k, v, bias1=None, bias2=None):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        b1 = bias1.float().contiguous() if bias1 is not None else None
        b2 = bias2.float().contiguous() if bias2 is not None else None
        o, lse = torch.ops.sxe.evoformer_fwd(q, k, v, b1, b2)
        ctx.save_for_backward(q, k, v, o, lse, b1, b2)
        ctx.bias_dtypes = (bias1.dtype if bias1 is not None else None, bias2.dtype if bias2 is not None else None)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, b1, b2 = ctx.saved_tensors
        B, N, L, H, _ = q.shape
        Lp = lse.shape[-1]
        delta = torch.zeros(B * N, H, Lp, dtype=torch.float32, device=q.device)
        delta[:, :, :L] = (do.float() * o.float()).sum(-1).reshape(B * N, L, H).transpose(1, 2)
        need1 = b1 is not None and ctx.needs_input_grad[3]
        need2 = b2 is not None and ctx.needs_input_grad[4]
        dq, dk, dv, db1, db2 = torch.ops.sxe.evoformer_bwd(do.contiguous().to(q.dtype), q, k, v, lse, delta, b1, b2,
                                                           need1, need2)
        db1 = db1.to(ctx.bias_dtypes[0]) if need1 else None
        db2 = db2.to(ctx.bias_dtypes[1]) if need2 else None
        return dq, dk, dv, db1, db2


def DS4Sci_EvoformerAttention(Q, K, V, biases):
    assert len(biases) <= 2
    biases = list(biases) + [None] * (2 - len(biases))
    if biases[0] is not None:
        assert biases[0].shape == (Q.shape[0], Q.shape[1], 1, 1, Q.shape[2]), "bias1 shape is incorrect"
    if biases[1] is not None:
        assert biases[1].shape == (Q.shape[0], 1, Q.shape[3], Q.shape[2], Q.shape[2]), "bias2 shape is incorrect"
    return evoformer_attention(Q, K, V, biases[0], biases[1])
