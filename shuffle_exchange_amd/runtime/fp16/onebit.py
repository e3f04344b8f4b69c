"""Communication-compressed optimizers: 1-bit Adam, 0/1 Adam, 1-bit LAMB.

Parity: reference runtime/fp16/onebit/adam.py (``OnebitAdam`` :14, warm-up with full-precision
all-reduce until ``freeze_step``, then frozen variance + 1-bit error-compensated momentum
all-reduce), zoadam.py (``ZeroOneAdam``: variance refreshed at exponentially spaced steps until
``var_freeze_step``, then momentum-only updates synchronised with 1-bit all-reduce at growing
``local_step`` intervals), lamb.py (``OnebitLamb``: frozen per-tensor trust-ratio scaling after the
warm-up, compressed momentum).

Integration (MI355X-first): the engine runs these on ZeRO stage 0 (as the reference requires). The
stage-0 optimizer flattens every parameter group into one fp32 master, so each compressed
all-reduce is ONE two-stage collective over the whole group (the reference issues one per
parameter). While ``comm_active`` is False the engine all-reduces gradients as usual; afterwards it
skips the gradient all-reduce and the optimizer's compressed momentum sync is the only
communication.
"""
import math

import torch

from ... import comm as dist
from ..comm.compressed import CompressedBackend


class _OnebitBase(torch.optim.Optimizer):
    #: the engine must not all-reduce gradients while this is True
    comm_active = False

    def __init__(self, params, defaults, deepspeed=None, comm_backend_name="nccl", group=None):
        super().__init__(params, defaults)
        self.deepspeed = deepspeed
        self.comm_backend_name = comm_backend_name
        self._group = group
        self._backend = None

    @property
    def backend(self):
        if self._backend is None:
            self._backend = CompressedBackend(self._group)
        return self._backend

    def set_group(self, group):
        self._group = group
        self._backend = None

    def _errors(self, state, p):
        if "worker_error" not in state:
            state["worker_error"], state["server_error"] = self.backend.make_errors(p.numel(), p.device)
        return state["worker_error"], state["server_error"]

    def _sync_momentum(self, state, p, exp_avg):
        if self.backend.size > 1:
            we, se = self._errors(state, p)
            self.backend.compressed_allreduce(exp_avg, we, se)
        if "exp_avg_mask" in self.param_groups[0]:
            exp_avg.mul_(self.param_groups[0]["exp_avg_mask"].to(exp_avg.device))

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        # compression errors are rank-local and not checkpointed: restart them from zero
        for st in self.state.values():
            st.pop("worker_error", None)
            st.pop("server_error", None)
        self._refresh_phase()

    def _refresh_phase(self):
        pass


class OnebitAdam(_OnebitBase):
    def __init__(self, params, deepspeed=None, lr=1e-3, freeze_step=100000, bias_correction=True, betas=(0.9, 0.999),
                 eps=1e-8, eps_inside_sqrt=False, weight_decay=0.0, max_grad_norm=0.0, amsgrad=False, cuda_aware=False,
                 comm_backend_name="nccl", group=None):
        if amsgrad:
            raise RuntimeError("1-bit Adam does not support the AMSGrad variant")
        super().__init__(params, dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                                      weight_decay=weight_decay, max_grad_norm=max_grad_norm), deepspeed,
                         comm_backend_name, group)
        self.freeze_step = int(freeze_step)
        self.eps_mode = 0 if eps_inside_sqrt else 1
        self.cuda_aware = cuda_aware

    def _refresh_phase(self):
        steps = [st.get("step", 0) for st in self.state.values()]
        self.comm_active = bool(steps) and max(steps) >= self.freeze_step

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                m, v = st["exp_avg"], st["exp_avg_sq"]
                if not self.comm_active:
                    # warm-up: gradients were all-reduced by the engine; plain Adam
                    m.mul_(b1).add_(g, alpha=1 - b1)
                    v.mul_(b2).addcmul_(g, g, value=1 - b2)
                else:
                    # variance frozen; local momentum, then 1-bit error-compensated average
                    m.mul_(b1).add_(g, alpha=1 - b1)
                    self._sync_momentum(st, p, m)
                upd = m / (v.sqrt() + group["eps"])
                if group["weight_decay"] > 0:
                    upd.add_(p, alpha=group["weight_decay"])
                p.add_(upd, alpha=-group["lr"])
        if not self.comm_active:
            steps = [st["step"] for st in self.state.values() if "step" in st]
            if steps and max(steps) >= self.freeze_step:
                self.comm_active = True
        return loss


class ZeroOneAdam(_OnebitBase):
    """0/1 Adam: adaptive variance freezing + 1-bit momentum sync with growing local-step gaps."""

    def __init__(self, params, deepspeed=None, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
                 eps_inside_sqrt=False, weight_decay=0.0, max_grad_norm=0.0, var_freeze_step=100000,
                 var_update_scaler=16, local_step_scaler=32678, local_step_clipper=16, amsgrad=False, cuda_aware=False,
                 comm_backend_name="nccl", group=None):
        super().__init__(params, dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                                      weight_decay=weight_decay, max_grad_norm=max_grad_norm), deepspeed,
                         comm_backend_name, group)
        self.var_freeze_step = int(var_freeze_step)
        self.var_update_scaler = int(var_update_scaler)
        self.local_step_scaler = int(local_step_scaler)
        self.local_step_clipper = int(local_step_clipper)
        self.var_interval = 1
        self.var_counter = 0
        self.local_interval = 1
        self.local_counter = 0

    def _refresh_phase(self):
        steps = [st.get("step", 0) for st in self.state.values()]
        self.comm_active = bool(steps) and max(steps) >= self.var_freeze_step

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        frozen = self.comm_active
        update_var = False
        sync_now = True
        if not frozen:
            self.var_counter += 1
            if self.var_counter >= self.var_interval:
                update_var = True
                self.var_counter = 0
        else:
            self.local_counter += 1
            sync_now = self.local_counter >= self.local_interval
            if sync_now:
                self.local_counter = 0
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                    st["momentum_accumulator"] = torch.zeros_like(p)
                st["step"] += 1
                m, v = st["exp_avg"], st["exp_avg_sq"]
                m.mul_(b1).add_(g, alpha=1 - b1)
                if not frozen:
                    if update_var:
                        v.mul_(b2).addcmul_(g, g, value=1 - b2)
                    upd = m / (v.sqrt() + group["eps"])
                else:
                    # local steps apply the local momentum; the accumulated update is reconciled
                    # across ranks with a 1-bit all-reduce every local_interval steps
                    acc = st["momentum_accumulator"]
                    acc.add_(m)
                    if sync_now:
                        self._sync_momentum(st, p, acc)
                        m.copy_(acc / max(1, self._last_interval()))
                        acc.zero_()
                    upd = m / (v.sqrt() + group["eps"])
                if group["weight_decay"] > 0:
                    upd.add_(p, alpha=group["weight_decay"])
                p.add_(upd, alpha=-group["lr"])
        steps = max((st["step"] for st in self.state.values() if "step" in st), default=0)
        if not frozen:
            if steps % self.var_update_scaler == 0:
                self.var_interval *= 2
            if steps >= self.var_freeze_step:
                self.comm_active = True
        elif sync_now and steps % self.local_step_scaler == 0:
            self.local_interval = min(self.local_step_clipper, self.local_interval * 2)
        return loss

    def _last_interval(self):
        return self.local_interval


class OnebitLamb(_OnebitBase):
    def __init__(self, params, deepspeed=None, lr=1e-3, freeze_step=100000, bias_correction=True, betas=(0.9, 0.999),
                 eps=1e-8, eps_inside_sqrt=False, weight_decay=0.0, max_grad_norm=0.0, max_coeff=10.0, min_coeff=0.01,
                 amsgrad=False, cuda_aware=False, comm_backend_name="nccl", coeff_beta=0.9, factor_max=4.0,
                 factor_min=0.5, factor_threshold=0.1, group=None):
        super().__init__(params, dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                                      weight_decay=weight_decay, max_grad_norm=max_grad_norm, max_coeff=max_coeff,
                                      min_coeff=min_coeff), deepspeed, comm_backend_name, group)
        self.freeze_step = int(freeze_step)
        self._segments = {}
        self.coeff_beta = coeff_beta
        self.factor_max, self.factor_min, self.factor_threshold = factor_max, factor_min, factor_threshold

    def _refresh_phase(self):
        steps = [st.get("step", 0) for st in self.state.values()]
        self.comm_active = bool(steps) and max(steps) >= self.freeze_step

    def set_segments(self, param, segments):
        """The engine trains flat per-group masters: LAMB's trust ratio is per original parameter,
        i.e. per (offset, numel) segment of the flat tensor."""
        self._segments[id(param)] = list(segments)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                segs = self._segments.get(id(p))
                if segs is not None:
                    self._step_segmented(group, p, segs)
                    continue
                g = p.grad
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                    st["lamb_coeff_freeze"] = 0.0
                    st["last_factor"] = 1.0
                st["step"] += 1
                m, v = st["exp_avg"], st["exp_avg_sq"]
                m.mul_(b1).add_(g, alpha=1 - b1)
                if not self.comm_active:
                    v.mul_(b2).addcmul_(g, g, value=1 - b2)
                else:
                    self._sync_momentum(st, p, m)
                upd = m / (v.sqrt() + group["eps"])
                if group["weight_decay"] > 0:
                    upd.add_(p, alpha=group["weight_decay"])
                if not self.comm_active:
                    wn, un = p.norm().item(), upd.norm().item()
                    coeff = (wn / un) if (wn > 0 and un > 0) else 1.0
                    coeff = max(min(coeff, group["max_coeff"]), group["min_coeff"])
                    st["lamb_coeff_freeze"] = self.coeff_beta * st["lamb_coeff_freeze"] + (1 - self.coeff_beta) * coeff
                else:
                    # frozen trust ratio, rescaled by how much the update norm drifted (bounded)
                    coeff = st["lamb_coeff_freeze"] * st["last_factor"]
                p.add_(upd, alpha=-group["lr"] * coeff)
        if not self.comm_active:
            steps = max((st["step"] for st in self.state.values() if "step" in st), default=0)
            if steps >= self.freeze_step:
                self.comm_active = True
        return loss

    def _step_segmented(self, group, p, segs):
        b1, b2 = group["betas"]
        g = p.grad
        st = self.state[p]
        if not st:
            st["step"] = 0
            st["exp_avg"] = torch.zeros_like(p)
            st["exp_avg_sq"] = torch.zeros_like(p)
            st["lamb_coeff_freeze"] = torch.zeros(len(segs), dtype=torch.float32)
        st["step"] += 1
        m, v = st["exp_avg"], st["exp_avg_sq"]
        m.mul_(b1).add_(g, alpha=1 - b1)
        if not self.comm_active:
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
        else:
            self._sync_momentum(st, p, m)
        upd = m / (v.sqrt() + group["eps"])
        if group["weight_decay"] > 0:
            upd.add_(p, alpha=group["weight_decay"])
        coeffs = st["lamb_coeff_freeze"]
        for j, (o, n) in enumerate(segs):
            if not self.comm_active:
                wn, un = p[o:o + n].norm().item(), upd[o:o + n].norm().item()
                c = (wn / un) if (wn > 0 and un > 0) else 1.0
                c = max(min(c, group["max_coeff"]), group["min_coeff"])
                coeffs[j] = self.coeff_beta * float(coeffs[j]) + (1 - self.coeff_beta) * c
            else:
                c = float(coeffs[j])
            p[o:o + n].add_(upd[o:o + n], alpha=-group["lr"] * c)


def build_onebit(name, params, group, **kw):
    kw.pop("torch_adam", None)
    kw.pop("adam_w_mode", None)
    if "betas" in kw:
        kw["betas"] = tuple(kw["betas"])
    cls = {"onebitadam": OnebitAdam, "zerooneadam": ZeroOneAdam, "onebitlamb": OnebitLamb}[name]
    return cls(params, group=group, **kw)
