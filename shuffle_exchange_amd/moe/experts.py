"""Expert containers (parity: reference deepspeed/moe/experts.py:13 ``Experts``).

``Experts``        generic: deep copies of any expert module, run one after another on their
                   capacity block (the reference's behaviour).
``GroupedSwiGLUExperts`` MI355X fast path for Llama/Mixtral experts: the E_local experts' weights
                   are stacked, so gate|up and down are each ONE batched hipBLASLt GEMM over
                   [E_local, tokens, H] with the HIP SwiGLU kernel between them.
Every expert parameter is tagged ``allreduce = False`` and ``group_name`` (reference convention)
so the ZeRO optimizers reduce its gradient over the expert-data-parallel group only.
"""
import copy
import os

import torch
import torch.nn as nn

from ..ops.activation import swiglu


class Experts(nn.Module):
    def __init__(self, expert, num_local_experts=1, expert_group_name=None):
        super().__init__()
        self.deepspeed_experts = nn.ModuleList([copy.deepcopy(expert) for _ in range(num_local_experts)])
        self.num_local_experts = num_local_experts
        for e in self.deepspeed_experts:
            for p in e.parameters():
                p.allreduce = False
                p.group_name = expert_group_name

    def forward(self, inputs):
        # inputs: [E_local, tokens, H]
        outs = [e(chunk) for chunk, e in zip(inputs.unbind(0), self.deepspeed_experts)]
        out = []
        for o in outs:
            out.append(o[0] if isinstance(o, tuple) else o)
        return torch.stack(out, dim=0)


class GroupedSwiGLUExperts(nn.Module):
    def __init__(self, hidden_size, intermediate_size, num_local_experts, expert_group_name=None, init_std=0.02):
        super().__init__()
        self.num_local_experts = num_local_experts
        self.w_gate_up = nn.Parameter(torch.empty(num_local_experts, hidden_size, 2 * intermediate_size))
        self.w_down = nn.Parameter(torch.empty(num_local_experts, intermediate_size, hidden_size))
        with torch.no_grad():
            self.w_gate_up.normal_(0.0, init_std)
            self.w_down.normal_(0.0, init_std)
        for p in (self.w_gate_up, self.w_down):
            p.allreduce = False
            p.group_name = expert_group_name

    def forward(self, x):
        # x: [E_local, C, H] -> [E_local, C, 2I] -> SwiGLU (one HIP launch for all experts) -> [E_local, C, H]
        if _fused_ok(x, self.w_gate_up, self.w_down):
            return _GroupedSwiGLU.apply(x, self.w_gate_up, self.w_down)
        return grouped_mm(swiglu(grouped_mm(x, self.w_gate_up)), self.w_down)


# Opt-in (SXE_MOE_TN=1): unlike the dense MLP (16k tokens of reduction) the experts' weight
# gradients reduce over only C capacity tokens, and the token-minor TN GEMMs measured no faster
# than the k-major wgrad kernel there (Mixtral-arch 8 layers: 311.8 vs 309.9 ms per step with
# fp32-out accumulating GEMMs, 332.6 ms with bf16 GEMMs + fp32 add passes).
MOE_TN = os.environ.get("SXE_MOE_TN", "0") == "1"


def _fused_ok(x, w_gu, w_down):
    from ..ops import native
    if not (MOE_TN and x.is_cuda and x.dtype == torch.bfloat16 and torch.is_grad_enabled()
            and w_gu.dtype == torch.bfloat16 and w_down.dtype == torch.bfloat16 and x.dim() == 3):
        return False
    E, C, H = x.shape
    I2 = w_gu.shape[2]
    return ((E * C) % 64 == 0 and C > 0 and H % 64 == 0 and I2 % 128 == 0 and w_down.shape[1:] == (I2 // 2, H)
            and native.use_hip(x))


def _expert_wgrad_tn(w, e, aT, bT, buf_acc):
    """dW[e] = aT @ bT^T (both token-minor slices of one expert): into the optimizer target when
    there is one (``buf_acc`` = (buf, accumulate)), else returned."""
    if buf_acc is None:
        return torch.mm(aT, bT.t())
    buf, acc = buf_acc
    if buf.dtype == torch.float32:
        # fp32-out GEMM accumulating in its epilogue: with only C tokens of reduction a separate
        # fp32 add pass over the expert's weight gradient would cost as much as the GEMM itself
        torch.ops.aten.addmm.dtype_out(buf[e], aT, bT.t(), torch.float32, beta=1 if acc else 0, alpha=1,
                                       out=buf[e])
    else:
        dw = torch.mm(aT, bT.t())
        buf[e].add_(dw) if acc else buf[e].copy_(dw)
    return None


class _GroupedSwiGLU(torch.autograd.Function):
    """The experts' SwiGLU MLP with the dense MLP's token-minor weight-gradient scheme (ops/mlp.py):
    the dual-layout gated kernels write h^T / dgu^T over all E*C rows next to the token-major
    outputs, so each expert's weight gradients are hipBLASLt "TN" GEMMs on column slices of them
    (1.3-1.5 PF vs 1.0-1.2 PF for the k-major product at these shapes) instead of k-strided ones."""

    @staticmethod
    def forward(ctx, x, w_gu, w_down):
        from ..ops import mlp as mlp_ops
        E, C, H = x.shape
        x = x.contiguous()
        gu = x.new_empty(E, C, w_gu.shape[2])
        for e in range(E):
            torch.mm(x[e], w_gu[e], out=gu[e])
        v = mlp_ops.dual_variant(w_down.shape[1])
        h, hT = torch.ops.sxe.gated_act_fwd_dual(gu.view(E * C, -1), mlp_ops.ACT_SILU, v)
        h = h.view(E, C, -1)
        out = x.new_empty(E, C, H)
        for e in range(E):
            torch.mm(h[e], w_down[e], out=out[e])
        del h
        xT = torch.ops.sxe.transpose16(x.view(E * C, H)) if ctx.needs_input_grad[1] else None
        ctx.save_for_backward(xT, gu, hT, w_gu, w_down)
        ctx.variant = v
        return out

    @staticmethod
    def backward(ctx, dout):
        from ..ops import mlp as mlp_ops
        xT, gu, hT, w_gu, w_down = ctx.saved_tensors
        E, C, I2 = gu.shape
        H = w_down.shape[2]
        dout = dout.contiguous()
        dx = dwgu = dwd = None
        dh = dout.new_empty(E, C, I2 // 2)
        for e in range(E):
            torch.mm(dout[e], w_down[e].t(), out=dh[e])
        sl = [slice(e * C, (e + 1) * C) for e in range(E)]
        if ctx.needs_input_grad[2]:
            doutT = torch.ops.sxe.transpose16(dout.view(E * C, H))
            tgt = getattr(w_down, "_sxe_grad_target", None)
            ba = tgt(w_down) if tgt is not None else None
            parts = [_expert_wgrad_tn(w_down, e, hT[:, sl[e]], doutT[:, sl[e]], ba) for e in range(E)]
            if ba is None:
                dwd = torch.stack(parts)
            else:
                w_down._sxe_grad_done(w_down)
            del doutT
        del hT
        dgu, dguT = torch.ops.sxe.gated_act_bwd_dual(dh.view(E * C, -1), gu.view(E * C, -1), mlp_ops.ACT_SILU,
                                                     ctx.variant)
        del dh
        dgu = dgu.view(E, C, I2)
        if ctx.needs_input_grad[0]:
            dx = dout.new_empty(E, C, H)
            for e in range(E):
                torch.mm(dgu[e], w_gu[e].t(), out=dx[e])
        del dgu
        if ctx.needs_input_grad[1]:
            tgt = getattr(w_gu, "_sxe_grad_target", None)
            ba = tgt(w_gu) if tgt is not None else None
            parts = [_expert_wgrad_tn(w_gu, e, xT[:, sl[e]], dguT[:, sl[e]], ba) for e in range(E)]
            if ba is None:
                dwgu = torch.stack(parts)
            else:
                w_gu._sxe_grad_done(w_gu)
        return dx, dwgu, dwd


class _GroupedMM(torch.autograd.Function):
    """y[e] = x[e] @ W[e] for x [E, C, K], W [E, K, N]: one plain 2-D hipBLASLt GEMM per expert,
    written in place into the output (no stacking copies). Backward: dX per expert in place, and
    dW straight into the ZeRO gradient buffer of W (fp32 accumulate with beta = 1 inside the GEMM,
    like ops/linear.py) -- autograd's select/stack backward would instead materialise a zeroed
    full-size [E, K, N] gradient per expert and sum them (measured: 36 % of a Mixtral step).
    Plain GEMMs rather than torch.bmm: the strided-batched backward of bmm under the TunableOp
    lookup-only path faulted on MI355X at Mixtral sizes (illegal address in the autograd thread)."""

    @staticmethod
    def forward(ctx, x, w):
        E, C, _ = x.shape
        x = x.contiguous()
        y = x.new_empty(E, C, w.shape[2])
        for e in range(E):
            torch.mm(x[e], w[e], out=y[e])
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        E = x.shape[0]
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            for e in range(E):
                torch.mm(dy[e], w[e].t(), out=dx[e])
        if ctx.needs_input_grad[1]:
            tgt = getattr(w, "_sxe_grad_target", None)
            if tgt is not None:
                from ..ops.linear import _sxe_wgrad_ok
                buf, acc = tgt(w)
                for e in range(E):
                    if _sxe_wgrad_ok(x[e], dy[e], buf[e]):  # hand-written k-major wgrad GEMM (gemm_wgrad.hip)
                        torch.ops.sxe.wgrad_gemm_(x[e], dy[e], buf[e], 1.0, bool(acc))
                    elif buf.dtype == torch.float32 and dy.dtype != torch.float32 and dy.is_cuda:
                        torch.ops.aten.addmm.dtype_out(buf[e], x[e].t(), dy[e], torch.float32, beta=1 if acc else 0,
                                                       alpha=1, out=buf[e])
                    elif buf.dtype != dy.dtype:
                        d = (x[e].t() @ dy[e]).to(buf.dtype)
                        buf[e].add_(d) if acc else buf[e].copy_(d)
                    elif acc:
                        buf[e].addmm_(x[e].t(), dy[e])
                    else:
                        torch.mm(x[e].t(), dy[e], out=buf[e])
                w._sxe_grad_done(w)
            else:
                dw = torch.empty_like(w)
                for e in range(E):
                    torch.mm(x[e].t(), dy[e], out=dw[e])
        return dx, dw


def grouped_mm(x, w):
    return _GroupedMM.apply(x, w)
