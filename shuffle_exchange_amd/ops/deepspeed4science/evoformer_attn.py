"""Evoformer attention with pair / mask biases (reference ops/deepspeed4science/evoformer_attn.py:
``DS4Sci_EvoformerAttention`` over a CUTLASS kernel, not in the snapshot).

O = softmax(Q K^T / sqrt(D) + bias1 + bias2) V with Q/K/V [B, N, L, H, D], bias1 [B, N, 1, 1, L]
(MSA row mask) and bias2 [B, 1, H, L, L] (pair bias), gradients for Q, K, V and both biases.
Implemented as a query-chunked computation in PyTorch (every chunk recomputed in the backward, so
the L x L probabilities of only one chunk are ever live): the attention matrices are small-D
(<= 64) batched GEMMs that hipBLASLt handles, and the memory bound -- the reason the reference has
a fused kernel -- is kept by the chunking. Parity with the CUTLASS kernel is unpinned (not
vendored); the tests check the exact formula.
"""
import math

import torch
from torch.utils.checkpoint import checkpoint

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


class EvoformerFusedAttention(torch.autograd.Function):
    """Kept for API parity: forwards to the chunked implementation (autograd handles the backward)."""

    @staticmethod
    def apply(q, k, v, bias1=None, bias2=None):
        return evoformer_attention(q, k, v, bias1, bias2)


def DS4Sci_EvoformerAttention(Q, K, V, biases):
    assert len(biases) <= 2
    biases = list(biases) + [None] * (2 - len(biases))
    if biases[0] is not None:
        assert biases[0].shape == (Q.shape[0], Q.shape[1], 1, 1, Q.shape[2]), "bias1 shape is incorrect"
    if biases[1] is not None:
        assert biases[1].shape == (Q.shape[0], 1, Q.shape[3], Q.shape[2], Q.shape[2]), "bias2 shape is incorrect"
    return evoformer_attention(Q, K, V, biases[0], biases[1])
