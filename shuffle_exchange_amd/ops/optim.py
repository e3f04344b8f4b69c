"""Fused optimizers (HIP kernels on GPU, PyTorch reference on CPU).

Parity targets in the reference: ``FusedAdam`` (deepspeed/ops/adam/fused_adam.py:18, step at
:107-193), ``FusedLion`` (deepspeed/ops/lion/fused_lion.py:17), ``FusedLamb``
(deepspeed/ops/lamb/fused_lamb.py:14). The ZeRO optimizers call the *flat* functional forms
(``adam_flat_`` etc.) on their fp32 master partitions; the kernel also writes the bf16/fp16 working
copy, so the separate fp32->bit16 copy of the reference (stage_1_and_2.py:2174-2176) disappears.
"""
import math

import torch

from . import native


# ------------------------------------------------------------------------------------------------
# flat functional forms
def _ref_scale(grad_scale, scale_t):
    s = torch.tensor(float(grad_scale), dtype=torch.float32)
    if scale_t is not None:
        s = s * scale_t.detach().float().cpu().reshape(-1)[0]
    return s


def adam_flat_(p, g, m, v, lp=None, *, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=1,
               adamw=True, bias_correction=True, grad_scale=1.0, scale_t=None, skip_t=None):
    """One Adam/AdamW step on flat fp32 state. ``grad_scale`` (host) and ``scale_t`` (device
    scalar) multiply the gradient; ``skip_t`` (device scalar) != 0 turns the call into a no-op."""
    if native.use_hip(p):
        torch.ops.sxe.adam_flat_(p, g, m, v, lp, scale_t, skip_t, float(lr), float(beta1), float(beta2), float(eps),
                                 float(weight_decay), int(step), bool(adamw), bool(bias_correction), float(grad_scale))
        return
    if skip_t is not None and float(skip_t.reshape(-1)[0]) != 0.0:
        return
    gs = g.float() * _ref_scale(grad_scale, scale_t).to(p.device)
    if not adamw and weight_decay != 0.0:
        gs = gs + weight_decay * p
    m.mul_(beta1).add_(gs, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(gs, gs, value=1 - beta2)
    bc1 = 1 - beta1 ** step if bias_correction else 1.0
    bc2 = 1 - beta2 ** step if bias_correction else 1.0
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    if adamw and weight_decay != 0.0:
        p.mul_(1 - lr * weight_decay)
    p.addcdiv_(m, denom, value=-lr / bc1)
    if lp is not None:
        lp.copy_(p)


def lion_flat_(p, g, m, lp=None, *, lr, beta1=0.9, beta2=0.99, weight_decay=0.0, grad_scale=1.0, scale_t=None,
               skip_t=None):
    if native.use_hip(p):
        torch.ops.sxe.lion_flat_(p, g, m, lp, scale_t, skip_t, float(lr), float(beta1), float(beta2),
                                 float(weight_decay), float(grad_scale))
        return
    if skip_t is not None and float(skip_t.reshape(-1)[0]) != 0.0:
        return
    gs = g.float() * _ref_scale(grad_scale, scale_t).to(p.device)
    u = (beta1 * m + (1 - beta1) * gs).sign()
    p.sub_(lr * (u + weight_decay * p))
    m.mul_(beta2).add_(gs, alpha=1 - beta2)
    if lp is not None:
        lp.copy_(p)


def adagrad_flat_(p, g, s, lp=None, *, lr, eps=1e-10, weight_decay=0.0, grad_scale=1.0, scale_t=None, skip_t=None):
    if native.use_hip(p):
        torch.ops.sxe.adagrad_flat_(p, g, s, lp, scale_t, skip_t, float(lr), float(eps), float(weight_decay),
                                    float(grad_scale))
        return
    if skip_t is not None and float(skip_t.reshape(-1)[0]) != 0.0:
        return
    gs = g.float() * _ref_scale(grad_scale, scale_t).to(p.device) + weight_decay * p
    s.addcmul_(gs, gs)
    p.addcdiv_(gs, s.sqrt().add_(eps), value=-lr)
    if lp is not None:
        lp.copy_(p)


def sumsq(x):
    """Sum of squares in fp32 (inf/NaN propagate: doubles as the overflow check)."""
    if x.is_cuda and native.hip_available() and x.is_contiguous() and x.data_ptr() % 16 == 0 and x.numel() > 0:
        return torch.ops.sxe.sumsq(x)
    return x.float().pow(2).sum()


# ------------------------------------------------------------------------------------------------
# torch.optim front-ends over parameter lists
class FusedAdam(torch.optim.Optimizer):
    """Adam/AdamW over parameter lists with one multi-tensor HIP launch per dtype group.

    Non-fp32 parameters get an fp32 master copy in the optimizer state and the kernel writes the
    updated bit16 value back (mixed-precision FusedAdam)."""

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, adam_w_mode=True,
                 weight_decay=0.0, amsgrad=False, set_grad_none=True):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support AMSGrad")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.adam_w_mode = adam_w_mode
        self.set_grad_none = set_grad_none

    def zero_grad(self, set_to_none=True):
        super().zero_grad(set_to_none=set_to_none if self.set_grad_none else False)

    @torch.no_grad()
    def step(self, closure=None, grad_scale=1.0, scale_t=None, skip_t=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            b1, b2 = group["betas"]
            buckets = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    master = p.detach().float() if p.dtype != torch.float32 else None
                    if master is not None:
                        st["master_param"] = master
                    ref = master if master is not None else p
                    st["exp_avg"] = torch.zeros_like(ref, dtype=torch.float32)
                    st["exp_avg_sq"] = torch.zeros_like(ref, dtype=torch.float32)
                st["step"] += 1
                key = (p.device, p.dtype, p.grad.dtype, st["step"])
                buckets.setdefault(key, []).append(p)
            for (dev, pdt, gdt, step), plist in buckets.items():
                masters = [self.state[p].get("master_param", p) for p in plist]
                grads = [p.grad.contiguous() for p in plist]
                ms = [self.state[p]["exp_avg"] for p in plist]
                vs = [self.state[p]["exp_avg_sq"] for p in plist]
                lps = [p for p in plist] if pdt != torch.float32 else []
                if dev.type == "cuda":
                    native.require_hip()
                    torch.ops.sxe.multi_tensor_adam_(masters, grads, ms, vs, lps, scale_t, skip_t, float(group["lr"]),
                                                     float(b1), float(b2), float(group["eps"]),
                                                     float(group["weight_decay"]), int(step), bool(self.adam_w_mode),
                                                     bool(group["bias_correction"]), float(grad_scale))
                else:
                    for i, p in enumerate(plist):
                        adam_flat_(masters[i], grads[i], ms[i], vs[i], lps[i] if lps else None, lr=group["lr"],
                                   beta1=b1, beta2=b2, eps=group["eps"], weight_decay=group["weight_decay"], step=step,
                                   adamw=self.adam_w_mode, bias_correction=group["bias_correction"],
                                   grad_scale=grad_scale, scale_t=scale_t, skip_t=skip_t)
        return loss


class FusedLion(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-4, betas=(0.9, 0.99), weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["master_param"] = p.detach().float().clone() if p.dtype != torch.float32 else None
                    st["exp_avg"] = torch.zeros(p.shape, dtype=torch.float32, device=p.device)
                master = st["master_param"] if st["master_param"] is not None else p
                lion_flat_(master.view(-1), p.grad.contiguous().view(-1), st["exp_avg"].view(-1),
                           p.view(-1) if st["master_param"] is not None else None, lr=group["lr"], beta1=b1, beta2=b2,
                           weight_decay=group["weight_decay"])
        return loss


class FusedAdagrad(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-2, eps=1e-10, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["master_param"] = p.detach().float().clone() if p.dtype != torch.float32 else None
                    st["exp_avg_sq"] = torch.zeros(p.shape, dtype=torch.float32, device=p.device)
                master = st["master_param"] if st["master_param"] is not None else p
                adagrad_flat_(master.view(-1), p.grad.contiguous().view(-1), st["exp_avg_sq"].view(-1),
                              p.view(-1) if st["master_param"] is not None else None, lr=group["lr"], eps=group["eps"],
                              weight_decay=group["weight_decay"])
        return loss


LAMB_BLOCK_ELEMS = 8192  # elements per HIP block of the LAMB kernels (one segment per block)


def lamb_block_table(segments, device):
    """(blk [nblk, 2] int64 element ranges, seg_id [nblk] int64) for segments [(seg_index, start,
    numel)] of a flat buffer: no block straddles two segments (each segment = one parameter)."""
    rows, ids = [], []
    for sid, start, n in segments:
        for b in range(start, start + n, LAMB_BLOCK_ELEMS):
            rows.append((b, min(b + LAMB_BLOCK_ELEMS, start + n)))
            ids.append(sid)
    blk = torch.tensor(rows, dtype=torch.int64).reshape(-1, 2).to(device)
    return blk, torch.tensor(ids, dtype=torch.int64).to(device)


def lamb_flat_(p, g, m, v, lp, table, nseg, *, lr, beta1, beta2, eps, weight_decay, step, bias_correction=True,
               min_coeff=0.01, max_coeff=10.0, scale_t=None, skip_t=None, norm_group=None, coeffs=None):
    """LAMB on a flat fp32 master whose segments are (fragments of) separate parameters: per-segment
    trust ratios (csrc/kernels/optim.hip lamb_stage1_/lamb_stage2_). ``norm_group``: all-reduce the
    per-segment norms over the ranks that hold the other fragments of the same parameters."""
    bc1 = 1 - beta1 ** step if bias_correction else 1.0
    bc2 = 1 - beta2 ** step if bias_correction else 1.0
    blk, seg_id = table
    sums = torch.zeros(nseg, 2, dtype=torch.float32, device=p.device)
    if p.is_cuda and native.use_hip(p):
        torch.ops.sxe.lamb_stage1_(p, g, m, v, blk, seg_id, sums, scale_t, skip_t, float(lr), float(beta1),
                                   float(beta2), float(eps), float(weight_decay), float(bc1), float(bc2), 1.0)
        if norm_group is not None:
            from .. import comm as dist
            dist.all_reduce(sums, group=norm_group)
        torch.ops.sxe.lamb_stage2_(p, m, v, lp, blk, seg_id, sums, coeffs, skip_t, float(lr), float(eps),
                                   float(weight_decay), float(bc1), float(bc2), float(min_coeff), float(max_coeff))
        return
    # CPU reference path (gloo plumbing): the same two stages in torch
    if skip_t is not None and float(skip_t.reshape(-1)[0]) != 0.0:
        return
    gs = g.float() * (scale_t.reshape(()) if scale_t is not None else 1.0)
    m.mul_(beta1).add_(gs, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(gs, gs, value=1 - beta2)
    u = (m / bc1) / ((v / bc2).sqrt() + eps) + weight_decay * p
    rows = blk.cpu().tolist()
    ids = seg_id.cpu().tolist()
    for (b, e), sid in zip(rows, ids):
        sums[sid, 0] += p[b:e].pow(2).sum()
        sums[sid, 1] += u[b:e].pow(2).sum()
    if norm_group is not None:
        from .. import comm as dist
        dist.all_reduce(sums, group=norm_group)
    wn, un = sums[:, 0].sqrt(), sums[:, 1].sqrt()
    coeff = torch.where((wn > 0) & (un > 0), wn / un.clamp(min=1e-30), torch.ones_like(wn)).clamp(min_coeff, max_coeff)
    if coeffs is not None:
        coeffs.copy_(coeff)
    for (b, e), sid in zip(rows, ids):
        p[b:e].sub_(u[b:e] * (lr * coeff[sid]))
    if lp is not None:
        lp.copy_(p)


class FusedLamb(torch.optim.Optimizer):
    """LAMB (reference deepspeed/ops/lamb/fused_lamb.py:14): Adam direction scaled per tensor by
    the trust ratio ||p|| / ||update||, clamped to [min_coeff, max_coeff]. GPU tensors run the
    two-stage HIP kernels (one segment per parameter); under ZeRO the engine runs the same kernels
    over the flat partitions with the trust ratio of each WHOLE parameter (runtime/zero/base.py)."""

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 max_grad_norm=0.0, max_coeff=10.0, min_coeff=0.01):
        super().__init__(params, dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                                      weight_decay=weight_decay, max_coeff=max_coeff, min_coeff=min_coeff))
        self.lamb_coeffs = []

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.lamb_coeffs = []
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros(p.shape, dtype=torch.float32, device=p.device)
                    st["exp_avg_sq"] = torch.zeros(p.shape, dtype=torch.float32, device=p.device)
                st["step"] += 1
                if p.is_cuda and p.dtype == torch.float32 and p.is_contiguous():
                    if "table" not in st:
                        st["table"] = lamb_block_table([(0, 0, p.numel())], p.device)
                    coeff = torch.empty(1, device=p.device)
                    lamb_flat_(p.view(-1), p.grad.contiguous().view(-1), st["exp_avg"].view(-1),
                               st["exp_avg_sq"].view(-1), None, st["table"], 1, lr=group["lr"], beta1=b1, beta2=b2,
                               eps=group["eps"], weight_decay=group["weight_decay"], step=st["step"],
                               bias_correction=group["bias_correction"], min_coeff=group["min_coeff"],
                               max_coeff=group["max_coeff"], coeffs=coeff)
                    self.lamb_coeffs.append(coeff[0])
                    continue
                g = p.grad.float()
                m, v = st["exp_avg"], st["exp_avg_sq"]
                m.mul_(b1).add_(g, alpha=1 - b1)
                v.mul_(b2).addcmul_(g, g, value=1 - b2)
                bc1 = 1 - b1 ** st["step"] if group["bias_correction"] else 1.0
                bc2 = 1 - b2 ** st["step"] if group["bias_correction"] else 1.0
                upd = (m / bc1) / ((v / bc2).sqrt() + group["eps"])
                pf = p.float()
                if group["weight_decay"]:
                    upd.add_(pf, alpha=group["weight_decay"])
                wn, un = pf.norm(), upd.norm()
                coeff = torch.where((wn > 0) & (un > 0), wn / un, torch.ones_like(wn))
                coeff = coeff.clamp(group["min_coeff"], group["max_coeff"])
                self.lamb_coeffs.append(coeff)
                p.copy_(pf - group["lr"] * coeff * upd)
        return loss


# ------------------------------------------------------------------------------------------------
# muP (maximal update parametrization) optimizers -- reference engine optimizer types MuAdam /
# MuAdamW / MuSGD (runtime/engine.py:1473-1569, backed by the ``mup`` package's optim.py).
def _mup_shape(p):
    """(ninf, width_mult, fanin_fanout_ratio) of a parameter: from ``p.infshape`` when ``mup``'s
    set_base_shapes ran, else from ``p.mup_width_mult`` (matrix-like if 2-D+, vector-like if 1-D)."""
    inf = getattr(p, "infshape", None)
    if inf is not None:
        ratio = inf.fanin_fanout_mult_ratio() if inf.ninf() == 2 else inf.width_mult()
        return inf.ninf(), inf.width_mult(), ratio
    wm = float(getattr(p, "mup_width_mult", 1.0))
    if wm == 1.0:
        return 0, 1.0, 1.0
    return (2 if p.dim() >= 2 else 1), wm, wm


def mup_param_groups(params, kind, decoupled_wd=False, defaults=None):
    """Split param groups by muP width multiplier. ``kind`` 'adam': matrix-like (two infinite dims)
    lr / width_mult; 'sgd': vector-like lr * width_mult, matrix-like lr / fanin_fanout_ratio.
    Multipliers land in ``lr_mult`` / ``wd_mult`` so LR schedules keep them (lr_schedules._set_lrs)."""
    groups = list(params)
    if not groups or not isinstance(groups[0], dict):
        groups = [{"params": groups}]
    out = []
    for g in groups:
        rest = dict(defaults or {})
        rest.update({k: v for k, v in g.items() if k != "params"})
        buckets = {}
        for p in g["params"]:
            ninf, wm, ratio = _mup_shape(p)
            if ninf > 2:
                raise NotImplementedError("muP: more than 2 infinite dimensions")
            if kind == "adam":
                lr_mult = 1.0 / wm if ninf == 2 else 1.0
            else:
                lr_mult = wm if ninf == 1 else (1.0 / ratio if ninf == 2 else 1.0)
            buckets.setdefault(lr_mult, []).append(p)
        for lr_mult, ps in buckets.items():
            ng = dict(rest, params=ps, lr_mult=lr_mult)
            if "lr" in ng:
                ng["lr"] = ng["lr"] * lr_mult
            if not decoupled_wd and lr_mult != 1.0 and ng.get("weight_decay"):
                ng["weight_decay"] = ng["weight_decay"] / lr_mult
            out.append(ng)
    return out


def MuAdam(params, lr=1e-3, weight_decay=0.0, decoupled_wd=False, adam_w_mode=False, **kw):
    groups = mup_param_groups(params, "adam", decoupled_wd, {"lr": lr, "weight_decay": weight_decay})
    return FusedAdam(groups, lr=lr, weight_decay=weight_decay, adam_w_mode=adam_w_mode, **kw)


def MuAdamW(params, lr=1e-3, weight_decay=0.0, decoupled_wd=False, **kw):
    return MuAdam(params, lr=lr, weight_decay=weight_decay, decoupled_wd=decoupled_wd, adam_w_mode=True, **kw)


def MuSGD(params, lr=1e-3, weight_decay=0.0, decoupled_wd=False, **kw):
    groups = mup_param_groups(params, "sgd", decoupled_wd, {"lr": lr, "weight_decay": weight_decay})
    return torch.optim.SGD(groups, lr=lr, weight_decay=weight_decay, **kw)
