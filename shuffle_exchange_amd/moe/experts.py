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

# SXE_MOE_DEFER_WGRAD=0: write the expert weight gradients every micro-step (see _GroupedMM)
DEFER_WGRAD = os.environ.get("SXE_MOE_DEFER_WGRAD", "1") == "1"


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

        self.tp_group = None

    def expert_tp_shard_(self, tp_group):
        """Expert tensor parallelism (reference MoE ``enable_expert_tensor_parallelism``): keep this
        TP rank's 1/tp of the gate and up columns and the matching rows of down. The input is then
        ``copy_to_tp`` (its gradient all-reduced over TP) and the output ``reduce_from_tp``."""
        from .. import comm as dist
        tp, r = dist.get_world_size(tp_group), dist.get_rank(tp_group)
        if tp == 1:
            return
        inter = self.w_down.shape[1]
        assert inter % tp == 0, f"expert intermediate size {inter} not divisible by tp {tp}"
        s = inter // tp
        with torch.no_grad():
            gu = self.w_gate_up.data
            gu = torch.cat([gu[..., r * s:(r + 1) * s], gu[..., inter + r * s:inter + (r + 1) * s]], -1).contiguous()
            down = self.w_down.data[:, r * s:(r + 1) * s].contiguous()
        for name, t in (("w_gate_up", gu), ("w_down", down)):
            old = getattr(self, name)
            new = nn.Parameter(t, requires_grad=old.requires_grad)
            new.allreduce, new.group_name, new.tensor_model_parallel = False, old.group_name, True
            setattr(self, name, new)
        self.tp_group = tp_group

    def forward(self, x):
        # x: [E_local, C, H] -> [E_local, C, 2I] -> SwiGLU (one HIP launch for all experts) -> [E_local, C, H]
        # (the dense MLP's token-minor weight-gradient scheme, ops/mlp.py, measured no faster here: the
        # experts reduce over only C capacity tokens -- Mixtral-arch 8 layers 311.8 vs 309.9 ms/step)
        if self.tp_group is not None:
            from ..module_inject.layers import copy_to_tp, reduce_from_tp
            x = copy_to_tp(x, self.tp_group)
            return reduce_from_tp(grouped_mm(swiglu(grouped_mm(x, self.w_gate_up)), self.w_down), self.tp_group)
        return grouped_mm(swiglu(grouped_mm(x, self.w_gate_up)), self.w_down)


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
            from ..ops.linear import grad_target
            tgt = grad_target(w)
            defer = getattr(w, "_sxe_grad_defer", None)
            if tgt is not None and DEFER_WGRAD and defer is not None and defer(w):
                # before the accumulation boundary: keep (x, dy) and write the weight gradient once, at
                # the boundary, over all micro-steps' tokens -- one fp32 write of the expert's gradient
                # per step instead of a write plus a read-modify-write per micro-step
                w.__dict__.setdefault("_sxe_wstash", []).append((x, dy))
                return dx, None
            stash = w.__dict__.pop("_sxe_wstash", None)
            prev = None  # one stashed micro-step: its (x, dy) are the first K segment of the product
            if stash and len(stash) == 1:
                prev = stash[0]
            elif stash:
                x = torch.cat([a for a, _ in stash] + [x], dim=1)
                dy = torch.cat([g for _, g in stash] + [dy], dim=1)
            if tgt is not None:
                buf, acc = tgt(w)
                for e in range(E):
                    if prev is not None:
                        x1, g1 = prev[0][e], prev[1][e]
                        if _wgrad2_ok(x1, g1, x[e], dy[e], buf[e]):
                            torch.ops.sxe.wgrad_gemm2_(x1, g1, x[e], dy[e], buf[e], 1.0, bool(acc))
                            continue
                        _expert_wgrad(x1, g1, buf[e], acc)
                        _expert_wgrad(x[e], dy[e], buf[e], True)
                        continue
                    _expert_wgrad(x[e], dy[e], buf[e], acc)
                w._sxe_grad_done(w)
            else:
                dw = torch.empty_like(w)
                for e in range(E):
                    torch.mm(x[e].t(), dy[e], out=dw[e])
        return dx, dw


def _expert_wgrad(xe, ge, be, acc):
    """be (+)= xe^T ge for one expert: the hand-written k-major wgrad GEMM (gemm_wgrad.hip) where its
    shapes allow, else an fp32-out library GEMM accumulating in its epilogue."""
    from ..ops.linear import _sxe_wgrad_ok
    if _sxe_wgrad_ok(xe, ge, be):
        torch.ops.sxe.wgrad_gemm_(xe, ge, be, 1.0, bool(acc))
    elif be.dtype == torch.float32 and ge.dtype != torch.float32 and ge.is_cuda:
        torch.ops.aten.addmm.dtype_out(be, xe.t(), ge, torch.float32, beta=1 if acc else 0, alpha=1, out=be)
    elif be.dtype != ge.dtype:
        d = (xe.t() @ ge).to(be.dtype)
        be.add_(d) if acc else be.copy_(d)
    elif acc:
        be.addmm_(xe.t(), ge)
    else:
        torch.mm(xe.t(), ge, out=be)


def _wgrad2_ok(x1, g1, x2, g2, be):
    """The two-segment wgrad kernel covers [x1; x2]^T [g1; g2] (no concatenated copy)."""
    from ..ops.linear import _sxe_wgrad_ok
    return (_sxe_wgrad_ok(x1, g1, be) and _sxe_wgrad_ok(x2, g2, be) and x1.stride(0) == x2.stride(0)
            and g1.stride(0) == g2.stride(0))


def grouped_mm(x, w):
    return _GroupedMM.apply(x, w)


def flush_deferred_wgrad(w):
    """Write a weight gradient still held as (x, dy) pairs (no backward reached ``w`` at the
    accumulation boundary): the same GEMMs as _GroupedMM's boundary pass."""
    stash = w.__dict__.pop("_sxe_wstash", None)
    if not stash:
        return
    x = torch.cat([a for a, _ in stash], dim=1)
    dy = torch.cat([g for _, g in stash], dim=1)
    defer, w._sxe_grad_defer = w._sxe_grad_defer, None
    try:
        _GroupedMM.backward(_FlushCtx(x, w), dy)
    finally:
        w._sxe_grad_defer = defer


class _FlushCtx:
    needs_input_grad = (False, True)

    def __init__(self, x, w):
        self.saved_tensors = (x, w)
