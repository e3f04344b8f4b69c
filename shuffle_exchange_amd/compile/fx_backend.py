"""DeepCompile graph compiler for ZeRO stages 0, 1 and 2 (reference compile/backend.py:217
``make_backend``, compile/init_z1.py:18 ``init_z1``, compile/passes/zero1_compile.py).

``torch.compile`` (Dynamo) captures the model's forward; AOT autograd turns each captured region
into a forward and a backward FX graph; this backend runs the graph passes of compile/fx_graph.py
on them and executes the result as ordinary ATen / ``torch.ops.sxe`` calls (HIP kernels) -- no
Inductor and no generated Triton, so the compiled step runs the same gfx950 kernels as the eager
one. What the compiler adds is *where communication happens*: every parameter gradient is handed
to the ZeRO optimizer by a ``sxe_dc.reduce_grad`` node placed right after the op that produces it,
so bucket all-reduces (ZeRO-0) / reduce-scatters (ZeRO-2) / fp32 accumulation (ZeRO-1) start in
the middle of the compiled backward on the comm stream. (A compiled region is ONE autograd node:
without the pass, per-parameter grad hooks would all fire after the whole backward graph.)

The first execution of every graph runs through ``ProfilingInterpreter`` (per-node time and
memory); the summary is logged and kept in ``engine.compile_plan["fx"]``.

ZeRO-3 builds on this compiler (compile/fx_zero3.py: gather / release / prefetch nodes in the same
graphs). The reduce nodes address parameters by identity, so a graph is compiled per parameter set
(``ParamBoundGraph``).
"""
import itertools

import torch

from ..utils.logging import log_dist
from .fx_graph import GraphParams, ProfilingInterpreter, insert_grad_reduce, reduce_order, sink_reduces

_ACTIVE = {}  # compiler id -> FXCompiler (the custom op finds its compiler through it)


@torch.library.custom_op("sxe_dc::reduce_grad", mutates_args=())
def reduce_grad(grad: torch.Tensor, compiler_id: int, param_id: int) -> None:
    """Hand one parameter gradient to the ZeRO optimizer (graph-side equivalent of autograd's
    AccumulateGrad followed by the optimizer's post-accumulate hook)."""
    _ACTIVE[compiler_id].on_grad(param_id, grad)


@reduce_grad.register_fake
def _reduce_grad_fake(grad, compiler_id, param_id):
    return None


class ParamBoundGraph:
    """A Dynamo graph compiled once PER PARAMETER SET. The in-graph reduce (and ZeRO-3 fetch) nodes
    name parameters by the identities seen when the graph was traced, but Dynamo reuses one compiled
    frame for every module instance of the same class (a graph break inside a repeated decoder
    layer compiles the layer's frame once and runs it for each layer, the parameters then being
    ordinary graph inputs): a graph bound to layer 0 would hand layer 5's gradients to layer 0.
    Every call looks up the compiled graph of the parameters actually passed in and compiles a new
    one for an unseen set."""

    def __init__(self, build, example_inputs, pid_of):
        self.build = build
        self.slots = [i for i, t in enumerate(example_inputs) if torch.is_tensor(t) and id(t) in pid_of]
        self.fns = {self._key(example_inputs): build(list(example_inputs))}
        self._boxed_call = getattr(next(iter(self.fns.values())), "_boxed_call", False)

    def _key(self, args):
        return tuple(id(args[i]) for i in self.slots)

    def __call__(self, *args):
        flat = args[0] if len(args) == 1 and isinstance(args[0], list) else args
        key = self._key(flat)
        fn = self.fns.get(key)
        if fn is None:
            fn = self.fns[key] = self.build(list(flat))
        return fn(*args)


class FXCompiler:
    def __init__(self, engine, cfg):
        self.engine, self.cfg = engine, cfg
        self.id = id(self)
        _ACTIVE[self.id] = self
        self.params = [p for p in engine.module.parameters()]
        self.pid_of = {id(p): i for i, p in enumerate(self.params)}
        self._gids = itertools.count()
        self.graphs = {}          # graph id -> {"params": n, "reduces": n, "order": ..., "profile": {...}}
        self.reduced = 0          # gradients delivered by reduce nodes (tests / logs)
        self.profile_runs = int(cfg.extra.get("fx_profile_runs", 1)) if hasattr(cfg, "extra") else 1

    # --------------------------------------------------------------------------- graph-side op
    def on_grad(self, pid, grad):
        p = self.params[pid]
        opt = self.engine.optimizer
        if p.grad is None:
            p.grad = grad.detach()
        else:
            p.grad = p.grad + grad.detach()
        self.reduced += 1
        if opt is not None and hasattr(opt, "grad_ready"):
            opt.grad_ready(p)

    # ---------------------------------------------------------------------------- the backend
    def backend(self, gm, example_inputs):
        return ParamBoundGraph(lambda inputs: self.compile_graph(gm, inputs), example_inputs, self.pid_of)

    def compile_graph(self, gm, example_inputs):
        from functorch.compile import make_boxed_func
        from torch._functorch.aot_autograd import aot_module_simplified
        from torch._functorch.partitioners import min_cut_rematerialization_partition

        gid = next(self._gids)
        gp = GraphParams([(i, self.pid_of[id(t)]) for i, t in enumerate(example_inputs)
                          if torch.is_tensor(t) and id(t) in self.pid_of])
        rec = self.graphs.setdefault(gid, {"params": len(gp.index_to_pid), "reduces": 0, "profile": {}})
        cuda = any(torch.is_tensor(t) and t.is_cuda for t in example_inputs)

        def wrap(kind, g):
            runs = {"n": 0}
            fast = make_boxed_func(g.forward)

            def call(args):
                if runs["n"] < self.profile_runs:
                    runs["n"] += 1
                    it = ProfilingInterpreter(g, cuda)
                    out = it.run(*args)
                    rec["profile"][kind] = it.finish()
                    args.clear()
                    return out if isinstance(out, (list, tuple)) else [out]
                return fast(args)
            call._boxed_call = True
            return call

        def fw_compiler(g, sample_inputs):
            rec["fw_nodes"] = len(g.graph.nodes)
            return wrap("fwd", g)

        def bw_compiler(g, sample_inputs):
            rec["reduces"] = insert_grad_reduce(g, self.id, gp, torch.ops.sxe_dc.reduce_grad.default)
            sink_reduces(g)
            rec["order"] = reduce_order(g)
            return wrap("bwd", g)

        return aot_module_simplified(gm, example_inputs, fw_compiler=fw_compiler, bw_compiler=bw_compiler,
                                     partition_fn=min_cut_rematerialization_partition)

    def summary(self):
        parts = []
        for gid, r in self.graphs.items():
            pr = r.get("profile", {})
            f, b = pr.get("fwd", {}), pr.get("bwd", {})
            parts.append(f"graph {gid}: {r['params']} params, {r['reduces']} in-graph reduces, "
                         f"fwd {f.get('total_ms', 0):.2f} ms / bwd {b.get('total_ms', 0):.2f} ms profiled")
        return "; ".join(parts)


def compile_fx(engine, cfg, compile_kwargs=None):
    """Install the graph compiler on a ZeRO-0/1/2 engine: returns the compiled module callable."""
    opt = engine.optimizer
    assert opt is not None and hasattr(opt, "grad_ready"), "the FX graph compiler needs a ZeRO-0/1/2 optimizer"
    for p in engine.module.parameters():
        # weight-gradient GEMMs writing straight into ZeRO buffers (ops/linear.py) are an eager-mode
        # shortcut with Python side effects inside backward; the graph's reduce nodes replace them
        for a in ("_sxe_grad_target", "_sxe_grad_done"):
            if hasattr(p, a):
                delattr(p, a)
    if any(p.is_cuda for p in engine.module.parameters()):
        from ..ops import native
        native.require_hip()  # loaded before tracing: the dispatch predicates then stay lock-free
        from ..ops import fake_kernels  # noqa: F401  (shape functions of the HIP ops for tracing)
    fx = FXCompiler(engine, cfg)
    kw = {k: v for k, v in (compile_kwargs or {}).items() if k in ("dynamic", "fullgraph")}
    kw.setdefault("dynamic", False)
    compiled = torch.compile(engine.module, backend=fx.backend, **kw)
    log_dist(f"compile: FX graph compiler (ZeRO-{engine.zero_optimization_stage()}): in-graph gradient "
             f"reduction for {len(fx.params)} parameters", ranks=[0])
    return fx, compiled
