"""Flops profiler: per-module FLOPs / MACs / parameters / latency of a forward pass.

Parity: reference profiling/flops_profiler/profiler.py -- ``FlopsProfiler`` :30
(start_profile / stop_profile / reset_profile / end_profile, get_total_flops / macs / params /
duration, print_model_profile with module depth / top modules) and ``get_model_profile``.

Mechanism (instead of monkey-patching torch.nn.functional as the reference does): FLOPs are
counted at the ATen dispatch level with ``torch.utils.flop_counter.FlopCounterMode`` -- every
matmul / conv / SDPA the model issues is seen, including ones inside fused helpers -- and this
framework registers formulas for its own HIP ops (flash attention fwd/bwd, paged attention), which
no generic counter could know. Module attribution comes from the counter's module tracker;
latencies from HIP events around each module's forward.
"""
import time
from collections import defaultdict

import torch
import torch.nn as nn
from torch.utils.flop_counter import FlopCounterMode, register_flop_formula

_REGISTERED = {"done": False}


def _register_sxe_formulas():
    if _REGISTERED["done"]:
        return
    _REGISTERED["done"] = True
    try:  # PyTorch has formulas for its GPU SDPA kernels, not for the CPU flash kernel
        @register_flop_formula(torch.ops.aten._scaled_dot_product_flash_attention_for_cpu)
        def _sdpa_cpu(q, k, v, *a, out_shape=None, **kw):
            B, H, S, D = q
            return 2 * (2 * B * H * S * k[2] * D)  # Q K^T and P V, as torch counts its GPU SDPA
    except Exception:
        pass
    try:
        from ...ops import native
        if not native.hip_available():
            return
        ops = torch.ops.sxe

        def attn_flops(q_shape, k_shape, causal):
            B, S, H, D = q_shape
            Sk = k_shape[1]
            f = 4 * B * H * S * Sk * D
            return f // 2 if causal else f

        @register_flop_formula(ops.flash_attn_fwd)
        def _fa_fwd(q, k, v, causal, scale, *a, out_shape=None, **kw):
            return attn_flops(q, k, causal)

        @register_flop_formula(ops.flash_attn_bwd)
        def _fa_bwd(dout, q, k, v, *a, out_shape=None, **kw):
            causal = a[3] if len(a) > 3 else True
            return int(2.5 * attn_flops(q, k, causal))

        # hand-written GEMMs: 2 * rows * out * in
        @register_flop_formula(ops.skinny_gemm)
        def _skinny(x, w, *a, out_shape=None, **kw):
            return 2 * x[0] * w[0] * w[1]

        @register_flop_formula(ops.skinny_gemm_fp8w)
        def _skinny8(x, wq, *a, out_shape=None, **kw):
            return 2 * x[0] * wq[0] * wq[1]

        @register_flop_formula(ops.grouped_gemm)
        def _grouped(x, w, *a, out_shape=None, **kw):  # every row meets exactly one expert
            return 2 * x[0] * w[1] * w[2]

        @register_flop_formula(ops.wgrad_gemm_)
        def _wgrad(a, b, *rest, out_shape=None, **kw):  # c (+)= a^T b, a [K, M], b [K, N]
            return 2 * a[0] * a[1] * b[1]
    except Exception:  # formulas are optional; generic ops are still counted
        pass


def _fmt(n, unit=""):
    for s, d in (("T", 1e12), ("G", 1e9), ("M", 1e6), ("K", 1e3)):
        if abs(n) >= d:
            return f"{n / d:.2f} {s}{unit}"
    return f"{n:.0f} {unit}"


class FlopsProfiler:
    def __init__(self, model, ds_engine=None, recompute_fwd_factor=0.0):
        self.model = model
        self.ds_engine = ds_engine
        self.recompute_fwd_factor = recompute_fwd_factor
        self.started = False
        self._mode = None
        self._hooks = []
        self._lat = defaultdict(float)
        self._t0 = {}
        self._flops = {}
        self._duration = 0.0

    # ------------------------------------------------------------------------------ control
    def start_profile(self, ignore_list=None):
        _register_sxe_formulas()
        self.reset_profile()
        self._mode = FlopCounterMode(display=False)
        self._mode.__enter__()
        cuda = torch.cuda.is_available()

        def pre(mod, args):
            if cuda:
                torch.cuda.synchronize()
            self._t0[id(mod)] = time.perf_counter()

        def post(mod, args, out):
            if cuda:
                torch.cuda.synchronize()
            self._lat[id(mod)] += time.perf_counter() - self._t0.pop(id(mod), time.perf_counter())

        for m in self.model.modules():
            if ignore_list and type(m) in ignore_list:
                continue
            self._hooks.append(m.register_forward_pre_hook(pre))
            self._hooks.append(m.register_forward_hook(post))
        self._start = time.perf_counter()
        self.started = True

    def stop_profile(self):
        if not self.started:
            return
        self._duration = time.perf_counter() - self._start
        self._mode.__exit__(None, None, None)
        self._flops = self._mode.get_flop_counts()
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.started = False

    def reset_profile(self):
        self._lat.clear()
        self._t0.clear()
        self._flops = {}

    def end_profile(self):
        self.stop_profile()
        self.reset_profile()

    # ------------------------------------------------------------------------------ results
    def _module_flops(self, name):
        key = name if name else "Global"
        d = self._flops.get(key) or self._flops.get(type(self.model).__name__ + ("." + name if name else ""), {})
        return sum(d.values())

    def get_total_flops(self, as_string=False):
        tot = sum(self._flops.get("Global", {}).values())
        return _fmt(tot, "FLOPS") if as_string else tot

    def get_total_macs(self, as_string=False):
        m = self.get_total_flops() / 2
        return _fmt(m, "MACs") if as_string else m

    def get_total_params(self, as_string=False):
        n = sum(p.numel() for p in self.model.parameters())
        return _fmt(n) if as_string else n

    def get_total_duration(self, as_string=False):
        return f"{self._duration * 1e3:.2f} ms" if as_string else self._duration

    def module_profile(self):
        """[(name, depth, params, flops, latency_s)] for every module."""
        out = []
        for name, m in self.model.named_modules():
            depth = 0 if not name else name.count(".") + 1
            params = sum(p.numel() for p in m.parameters())
            fl = 0
            for k, v in self._flops.items():
                if k == "Global":
                    continue
                kk = k.split(".", 1)[1] if "." in k and k.split(".", 1)[0] == type(self.model).__name__ else k
                if kk == name or (not name and k == type(self.model).__name__):
                    fl = sum(v.values())
            if not name:
                fl = self.get_total_flops()
            out.append((name or type(self.model).__name__, depth, params, fl, self._lat.get(id(m), 0.0)))
        return out

    def print_model_profile(self, profile_step=1, module_depth=-1, top_modules=1, detailed=True, output_file=None):
        lines = []
        tot_f, dur = self.get_total_flops(), self._duration
        lines.append("-" * 80)
        lines.append(f"flops profiler: profile step {profile_step}")
        lines.append(f"params: {self.get_total_params(True)}   fwd FLOPs: {_fmt(tot_f, 'FLOPS')}   "
                     f"fwd MACs: {_fmt(tot_f / 2, 'MACs')}   fwd latency: {dur * 1e3:.2f} ms   "
                     f"fwd throughput: {_fmt(tot_f / dur if dur else 0, 'FLOPS')}")
        if self.recompute_fwd_factor or True:
            mult = 3 + self.recompute_fwd_factor
            lines.append(f"fwd+bwd FLOPs per step (x{mult:g}): {_fmt(tot_f * mult, 'FLOPS')}")
        prof = self.module_profile()
        by_depth = defaultdict(list)
        for name, d, params, fl, lat in prof:
            by_depth[d].append((name, params, fl, lat))
        for d in sorted(by_depth):
            if module_depth >= 0 and d > module_depth:
                break
            top = sorted(by_depth[d], key=lambda r: -r[2])[:max(1, top_modules)]
            lines.append(f"depth {d}: " + ", ".join(f"{n} ({_fmt(f, 'FLOPS')}, {lat * 1e3:.2f} ms)"
                                                   for n, _, f, lat in top))
        if detailed:
            for name, d, params, fl, lat in prof:
                if module_depth >= 0 and d > module_depth:
                    continue
                lines.append(f"{'  ' * d}{name}: params {_fmt(params)}, {_fmt(fl, 'FLOPS')}, {lat * 1e3:.3f} ms")
        lines.append("-" * 80)
        text = "\n".join(lines)
        if output_file:
            with open(output_file, "w") as f:
                f.write(text + "\n")
        else:
            print(text)
        return text


def get_model_profile(model, input_shape=None, args=None, kwargs=None, print_profile=True, detailed=True,
                      module_depth=-1, top_modules=1, warm_up=1, as_string=True, output_file=None,
                      ignore_modules=None, mode="forward"):
    """Profile one forward of ``model``; returns (flops, macs, params)."""
    args = list(args or [])
    kwargs = dict(kwargs or {})
    if input_shape is not None:
        dev = next(model.parameters()).device
        args = [torch.ones(input_shape, dtype=torch.long, device=dev)] + args
    with torch.no_grad():
        for _ in range(warm_up):
            model(*args, **kwargs)
        prof = FlopsProfiler(model)
        prof.start_profile(ignore_list=ignore_modules)
        model(*args, **kwargs)
        prof.stop_profile()
    flops, macs, params = prof.get_total_flops(), prof.get_total_macs(), prof.get_total_params()
    if print_profile:
        prof.print_model_profile(module_depth=module_depth, top_modules=top_modules, detailed=detailed,
                                 output_file=output_file)
    prof.end_profile()
    if as_string:
        return _fmt(flops, "FLOPS"), _fmt(macs, "MACs"), _fmt(params)
    return flops, macs, params
