"""Shape functions ("fake" kernels) of the HIP ops a training step runs, so Dynamo / AOT autograd
can trace models that call ``torch.ops.sxe.*`` (compile/fx_backend.py). Each mirrors the output
allocation of its kernel in csrc/kernels/*.hip; in-place ops declare their mutation in the schema
and return nothing. Imported only by the FX graph compiler on a GPU process."""
import torch

from . import native

native.require_hip()
_reg = torch.library.register_fake


def _rows(x):
    return x.numel() // x.shape[-1]


@_reg("sxe::norm_fwd")
def _norm_fwd(x, residual, weight, bias, eps, layernorm):
    r = _rows(x)
    f = x.new_empty((r,), dtype=torch.float32)
    mean = x.new_empty((r,) if layernorm else (0,), dtype=torch.float32)
    h = torch.empty_like(x) if residual is not None else x.new_empty((0,))
    return [torch.empty_like(x), f, mean, h]


@_reg("sxe::norm_bwd")
def _norm_bwd(dy, x, rstd, mean, weight, dres, layernorm):
    H = x.shape[-1]
    return [torch.empty_like(x), x.new_empty((H,), dtype=torch.float32),
            x.new_empty((H,) if layernorm else (0,), dtype=torch.float32)]


@_reg("sxe::rope_")
def _rope(x, cos, sin, pos, seq_len, pos_offset, inverse):
    return None


@_reg("sxe::gated_act_fwd")
def _gated_fwd(gu, act):
    return gu.new_empty(gu.shape[:-1] + (gu.shape[-1] // 2,))


@_reg("sxe::gated_act_bwd")
def _gated_bwd(dout, gu, act):
    return torch.empty_like(gu)


@_reg("sxe::gated_act_fwd_dual")
def _gated_fwd_dual(gu, act, variant=0):
    I = gu.shape[-1] // 2
    T = gu.numel() // gu.shape[-1]
    return gu.new_empty(gu.shape[:-1] + (I,)), gu.new_empty((I, T))


@_reg("sxe::gated_act_bwd_dual")
def _gated_bwd_dual(dout, gu, act, variant=0):
    T = gu.numel() // gu.shape[-1]
    return torch.empty_like(gu), gu.new_empty((gu.shape[-1], T))


@_reg("sxe::bias_act_fwd")
def _bias_act_fwd(x, bias, act):
    return torch.empty_like(x)


@_reg("sxe::bias_act_bwd")
def _bias_act_bwd(dy, x, bias, act):
    return torch.empty_like(x)


@_reg("sxe::flash_attn_fwd")
def _fa_fwd(q, k, v, causal, scale, kv_len=-1, causal_offset=-(1 << 40)):
    B, Sq, H, D = q.shape
    return [q.new_empty((B, Sq, H, v.shape[-1])), q.new_empty((B, H, Sq), dtype=torch.float32)]


@_reg("sxe::flash_attn_bwd")
def _fa_bwd(dout, q, k, v, o, lse, dq, dk, dv, causal, scale, kv_len=-1, causal_offset=-(1 << 40)):
    return None


@_reg("sxe::xent_fwd")
def _xent_fwd(logits, target, ignore_index, inplace_grad, scale, grad_scale):
    r = logits.shape[0]
    return logits.new_empty((r,), dtype=torch.float32), logits.new_empty((r,), dtype=torch.float32)


@_reg("sxe::xent_bwd")
def _xent_bwd(logits, target, lse, dloss, ignore_index, inplace):
    return torch.empty_like(logits)


@_reg("sxe::xent_grad_dual")
def _xent_grad_dual(logits, target, lse, ignore_index, scale_a, scale_b):
    return logits.new_empty((logits.shape[1], logits.shape[0]))


@_reg("sxe::acc2_bf16_")
def _acc2(dst, a, b, accumulate):
    return None


@_reg("sxe::transpose16")
def _transpose16(x):
    return x.new_empty((x.shape[1], x.shape[0]))


@_reg("sxe::wgrad_gemm_")
def _wgrad(a, b, c, alpha, accumulate):
    return None


@_reg("sxe::gather_rows")
def _gather_rows(src, idx, offset=0, add=None):
    return src.new_empty((idx.numel(),) + tuple(src.shape[1:]))


@_reg("sxe::scatter_rows_")
def _scatter_rows(dst, idx, src):
    return None
