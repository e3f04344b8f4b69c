"""MoQ: quantize-during-training of weights with a bit-width schedule.

Parity: reference runtime/quantize.py ``Quantizer`` :14 (q_start_bits -> q_target_bits, halving
period ``q_period`` scaled by the block eigenvalue when enabled, symmetric / asymmetric, nearest /
stochastic rounding, q_groups, mixed fp16 blending). Weights are fake-quantized in place after the
optimizer step (master weights untouched), grouped per ``q_groups`` rows.
"""
import torch


def fake_quantize(w, bits, groups=1, symmetric=True, stochastic=False):
    flat = w.detach().float().reshape(groups, -1)
    if symmetric:
        q = 2 ** (bits - 1) - 1
        s = flat.abs().amax(1, keepdim=True).clamp_min(1e-12) / q
        x = flat / s
        x = torch.floor(x + torch.rand_like(x)) if stochastic else torch.round(x)
        out = x.clamp(-q - 1, q) * s
    else:
        lo, hi = flat.amin(1, keepdim=True), flat.amax(1, keepdim=True)
        s = (hi - lo).clamp_min(1e-12) / (2 ** bits - 1)
        x = (flat - lo) / s
        x = torch.floor(x + torch.rand_like(x)) if stochastic else torch.round(x)
        out = x.clamp(0, 2 ** bits - 1) * s + lo
    return out.reshape(w.shape).to(w.dtype)


class Quantizer:
    def __init__(self, q_groups=1, q_mixed_fp16=False, q_change_ratio=0.01, q_type=0, q_rounding=0, q_verbose=False,
                 q_eigenvalue=False, use_quantizer_kernel=False, layer_num=0, q_start_bits=16, q_target_bits=8,
                 q_period=100):
        self.q_groups, self.q_mixed_fp16, self.q_change_ratio = q_groups, q_mixed_fp16, q_change_ratio
        self.symmetric = q_type == 0
        self.stochastic = q_rounding == 1
        self.q_eigenvalue = q_eigenvalue
        self.start_bits, self.target_bits, self.period = q_start_bits, q_target_bits, q_period
        self.bits = {}
        self.next_change = {}
        self.quantize_real_ratio = 1.0 if not q_mixed_fp16 else 0.0
        self.steps = 0

    def any_precision_switch(self):
        return any(self.steps >= n for n in self.next_change.values())

    @torch.no_grad()
    def quantize(self, parameter_group, overflow=False, eigenvalue_enabled=False, block_eigenvalue=None):
        if overflow:
            return
        self.steps += 1
        if self.q_mixed_fp16:
            self.quantize_real_ratio = min(1.0, self.quantize_real_ratio + self.q_change_ratio)
        for gi, group in enumerate(parameter_group):
            for pi, p in enumerate(group):
                if p.dim() < 2:
                    continue
                key = (gi, pi)
                if key not in self.bits:
                    self.bits[key] = self.start_bits
                    self.next_change[key] = self.period
                if self.steps >= self.next_change[key] and self.bits[key] > self.target_bits:
                    self.bits[key] = max(self.target_bits, self.bits[key] - 1)
                    scale = 1.0
                    if eigenvalue_enabled and block_eigenvalue is not None:
                        scale = 1.0 + float(block_eigenvalue.get(pi, (0.0, 0))[0])
                    self.next_change[key] = self.steps + int(self.period * scale)
                b = self.bits[key]
                if b >= 16:
                    continue
                groups = self.q_groups if p.shape[0] % self.q_groups == 0 else 1
                q = fake_quantize(p, b, groups, self.symmetric, self.stochastic)
                if self.q_mixed_fp16 and self.quantize_real_ratio < 1.0:
                    q = self.quantize_real_ratio * q + (1 - self.quantize_real_ratio) * p
                p.copy_(q)
