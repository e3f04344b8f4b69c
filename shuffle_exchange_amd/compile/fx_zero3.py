"""DeepCompile for ZeRO-3 as a graph compiler (reference compile/init_z3.py:21,
compile/passes/zero3_compile.py ``add_z3_gather_release``, passes/prefetch.py ``schedule_prefetch``,
passes/selective_gather.py, runtime ops of compile/util.py:49 ``dc.allgather_param`` /
``wait_allgather`` / ``release_param`` / ``reduce_grad``).

Dynamo captures the model's forward, AOT autograd splits it into a forward and a backward FX graph,
and the passes below place the ZeRO-3 collectives IN those graphs:

  * ``add_gather_release`` -- for every fetch group (a module's flat ZeRO-3 units) a
    ``sxe_dc.z3_fetch`` node right before the first node that reads one of its parameters and a
    ``sxe_dc.z3_release`` node right after the last one, in the forward and in the backward graph;
  * ``schedule_prefetch`` -- each fetch also launches the all-gathers of the next ``depth`` groups
    of the same graph (``wait = False``: RCCL on the all-gather stream, the graph's later fetch of
    that group only waits on its event), so the communication of group k+1 runs under the compute
    of group k;
  * ``selective_gather`` -- the groups used last in the forward (first in the backward) are not
    released after the forward while their bytes fit ``max_live_parameters``: their backward
    re-gather disappears (the reference's selective unsharding);
  * ``insert_grad_reduce`` (shared with the ZeRO-0/1/2 compiler, compile/fx_graph.py) -- every
    parameter gradient goes to the ZeRO-3 optimizer by a ``sxe_dc.reduce_grad`` node right where
    it is produced; the optimizer stages it and launches the unit's reduce-scatter on its own
    communicator (zero/stage3.py) while the backward graph goes on.

The graphs are executed as generated FX Python (no Inductor, no Triton): the same gfx950 kernels as
eager, with the collectives at compiler-chosen points. The optimizer runs in graph mode
(``ZeroStage3Optimizer.enter_graph_mode``): no module hooks, and released parameters keep their
full shapes over freed storage, which is what lets a shape-specialising tracer see them (the
reference patches FakeTensor for the same reason, compile/patch_fake_tensor.py).
"""
import logging

import torch

from ..utils.logging import log_dist
from .fx_backend import FXCompiler, _ACTIVE
from .fx_graph import GraphParams, insert_grad_reduce, output_node, sink_reduces, reduce_order


@torch.library.custom_op("sxe_dc::z3_fetch", mutates_args=())
def z3_fetch(compiler_id: int, fg: int, wait: bool, backward: bool) -> None:
    """Gather fetch group ``fg`` (wait = True: the current stream waits for it; False: launch only)."""
    _ACTIVE[compiler_id].fetch(fg, wait, backward)


@z3_fetch.register_fake
def _z3_fetch_fake(compiler_id, fg, wait, backward):
    return None


@torch.library.custom_op("sxe_dc::z3_release", mutates_args=())
def z3_release(compiler_id: int, fg: int, backward: bool) -> None:
    """Free the gathered storage of fetch group ``fg`` (its shard stays)."""
    _ACTIVE[compiler_id].release(fg, backward)


@z3_release.register_fake
def _z3_release_fake(compiler_id, fg, backward):
    return None


def _aliases(node):
    """``node`` and every node that is a view of it (transitively): they all read its storage."""
    views = _view_ops()
    out, stack = [node], [node]
    while stack:
        n = stack.pop()
        for u in n.users:
            if u.op == "call_function" and u.target in views and u.args and u.args[0] is n:
                out.append(u)
                stack.append(u)
    return out


def _param_groups_of(gm, placeholder_fg):
    """{fetch group: (first, last) node index reading its storage} over the graph's nodes -- the
    readers of a parameter include the readers of its views (``t(W)`` feeding a GEMM)."""
    nodes = list(gm.graph.nodes)
    pos = {n: i for i, n in enumerate(nodes)}
    span = {}
    for ph, fg in placeholder_fg.items():
        users = [pos[u] for a in _aliases(ph) for u in a.users]
        if not users:
            continue
        lo, hi = min(users), max(users)
        a, b = span.get(fg, (lo, hi))
        span[fg] = (min(a, lo), max(b, hi))
    return nodes, span


def add_gather_release(gm, cid, placeholder_fg, backward, keep=(), prefetch_depth=1):
    """Insert fetch / release nodes for every fetch group read by the graph; groups in ``keep`` are
    not released. Returns (fetch order, counts)."""
    nodes, span = _param_groups_of(gm, placeholder_fg)
    order = sorted(span, key=lambda fg: span[fg][0])
    g = gm.graph
    n_fetch = n_rel = n_pref = 0
    for k, fg in enumerate(order):
        lo, hi = span[fg]
        with g.inserting_before(nodes[lo]):
            g.call_function(torch.ops.sxe_dc.z3_fetch.default, (cid, fg, True, backward))
            n_fetch += 1
            # prefetch: launch the next groups' all-gathers now, under this group's compute
            for nxt in order[k + 1:k + 1 + prefetch_depth]:
                g.call_function(torch.ops.sxe_dc.z3_fetch.default, (cid, nxt, False, backward))
                n_pref += 1
        if fg not in keep:
            with g.inserting_after(nodes[hi]):
                g.call_function(torch.ops.sxe_dc.z3_release.default, (cid, fg, backward))
                n_rel += 1
    g.lint()
    gm.recompile()
    return order, {"fetch": n_fetch, "prefetch": n_pref, "release": n_rel}


_VIEW_OPS = None


def _view_ops():
    global _VIEW_OPS
    if _VIEW_OPS is None:
        a = torch.ops.aten
        _VIEW_OPS = {a.t.default, a.view.default, a._unsafe_view.default, a.permute.default, a.transpose.int,
                     a.expand.default, a.slice.Tensor, a.select.int, a.unsqueeze.default, a.squeeze.dim,
                     a.squeeze.default, a.alias.default, a.as_strided.default, a.detach.default,
                     a.reshape.default}
    return _VIEW_OPS


def saved_param_views(fw_gm, placeholder_fg):
    """Forward-graph outputs that are parameters or views of parameters (AOT autograd may save
    ``t(W)`` instead of W for the backward): {output node name: fetch group}. The backward graph
    receives them as placeholders of the same name, and they read the unit's storage, so the
    backward must gather that group before their first use too."""
    views = _view_ops()
    out = {}
    for a in output_node(fw_gm.graph).args[0]:
        n = a
        while isinstance(n, torch.fx.Node) and n.op == "call_function" and n.target in views:
            n = n.args[0]
        if isinstance(n, torch.fx.Node) and n in placeholder_fg and isinstance(a, torch.fx.Node):
            out[a.name] = placeholder_fg[n]
    return out


def selective_gather(order, fg_bytes, budget_bytes):
    """Groups used last in the forward stay resident for the backward while they fit the budget
    (walking back from the end of the forward)."""
    keep, used = set(), 0
    for fg in reversed(order):
        b = fg_bytes.get(fg, 0)
        if used + b > budget_bytes:
            break
        keep.add(fg)
        used += b
    return keep


class FXZero3Compiler(FXCompiler):
    def __init__(self, engine, cfg):
        super().__init__(engine, cfg)
        self.opt = engine.optimizer
        self.fg_of_pid = {}
        for fg in self.opt.fgroups:
            for u in fg.units:
                if u.persistent:
                    continue
                for p in u.params:
                    self.fg_of_pid[self.pid_of[id(p)]] = fg.idx
        self.prefetch_depth = max(0, int(self.opt.prefetch_depth))
        self.live_budget = int(self.opt.max_live_parameters) * 2  # bytes of bf16 parameters
        self.fg_bytes = {fg.idx: sum(u.padded * u.flat.element_size() for u in fg.units if not u.persistent)
                         for fg in self.opt.fgroups}
        self.stats = {"fetch": 0, "prefetch_launch": 0, "release": 0}

    # ------------------------------------------------------------------------- graph-side ops
    def fetch(self, fg, wait, backward):
        opt = self.opt
        opt._in_bwd = backward
        opt._fetch(opt.fgroups[fg], wait=wait)
        self.stats["fetch" if wait else "prefetch_launch"] += 1

    def release(self, fg, backward):
        opt = self.opt
        opt._in_bwd = backward
        opt._release(opt.fgroups[fg])
        self.stats["release"] += 1

    # ---------------------------------------------------------------------------- the backend
    def compile_graph(self, gm, example_inputs):
        from functorch.compile import make_boxed_func
        from torch._functorch.aot_autograd import aot_module_simplified
        from torch._functorch.partitioners import min_cut_rematerialization_partition

        gid = next(self._gids)
        idx_pid = [(i, self.pid_of[id(t)]) for i, t in enumerate(example_inputs)
                   if torch.is_tensor(t) and id(t) in self.pid_of]
        gp = GraphParams(idx_pid)
        # AOT names the forward placeholder of example input i "primals_{i+1}" and keeps that name for
        # the parameter when the backward graph receives it as a saved tensor
        name_fg = {f"primals_{i + 1}": self.fg_of_pid[pid] for i, pid in idx_pid if pid in self.fg_of_pid}
        rec = self.graphs.setdefault(gid, {"params": len(idx_pid), "reduces": 0, "profile": {}})

        def ph_map(g):
            return {n: name_fg[n.name] for n in g.graph.nodes if n.op == "placeholder" and n.name in name_fg}

        def fw_compiler(g, sample_inputs):
            name_fg.update(saved_param_views(g, ph_map(g)))
            span = _param_groups_of(g, ph_map(g))[1]
            order = sorted(span, key=lambda fg: span[fg][0])
            keep = selective_gather(order, self.fg_bytes, self.live_budget) if torch.is_grad_enabled() else set()
            _, cnt = add_gather_release(g, self.id, ph_map(g), False, keep=keep, prefetch_depth=self.prefetch_depth)
            rec["fw"] = {**cnt, "kept": sorted(keep)}
            return make_boxed_func(g.forward)

        def bw_compiler(g, sample_inputs):
            rec["reduces"] = insert_grad_reduce(g, self.id, gp, torch.ops.sxe_dc.reduce_grad.default)
            sink_reduces(g)
            _, cnt = add_gather_release(g, self.id, ph_map(g), True, prefetch_depth=self.prefetch_depth)
            rec["bw"] = cnt
            rec["order"] = reduce_order(g)
            return make_boxed_func(g.forward)

        return aot_module_simplified(gm, example_inputs, fw_compiler=fw_compiler, bw_compiler=bw_compiler,
                                     partition_fn=min_cut_rematerialization_partition)


def compile_fx_zero3(engine, cfg, compile_kwargs=None):
    """Install the ZeRO-3 graph compiler; returns (compiler, compiled module callable)."""
    opt = engine.optimizer
    assert hasattr(opt, "fgroups"), "compile_fx_zero3 needs the ZeRO-3 optimizer"
    for p in engine.module.parameters():
        for a in ("_sxe_grad_target", "_sxe_grad_done"):
            if hasattr(p, a):
                delattr(p, a)
    if any(p.is_cuda for p in engine.module.parameters()):
        from ..ops import native
        native.require_hip()  # loaded before tracing: the dispatch predicates then stay lock-free
        from ..ops import fake_kernels  # noqa: F401
    opt.enter_graph_mode()
    fx = FXZero3Compiler(engine, cfg)
    kw = {k: v for k, v in (compile_kwargs or {}).items() if k in ("dynamic", "fullgraph")}
    kw.setdefault("dynamic", False)
    # one graph for the whole forward: in graph mode the module hooks are gone, so a module that a
    # graph break leaves to eager execution would read a released (zero-storage) parameter; Dynamo
    # then names the break instead of the step failing somewhere inside it
    if not kw.setdefault("fullgraph", True):
        log_dist("compile: ZeRO-3 with fullgraph=False -- a graph break that leaves a module to eager "
                 "execution reads released parameters", ranks=[0], level=logging.WARNING)
    compiled = torch.compile(engine.module, backend=fx.backend, **kw)
    log_dist(f"compile: FX graph compiler (ZeRO-3): {len(opt.fgroups)} fetch groups, gather/release/prefetch "
             f"(depth {fx.prefetch_depth}) and gradient reduce-scatter placed in the graphs", ranks=[0])
    return fx, compiled
