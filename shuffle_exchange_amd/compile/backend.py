"""Profile-guided schedule compiler for ZeRO-3 -- the MI355X counterpart of DeepCompile
(reference compile/backend.py:217 ``make_backend``, compile/init_z3.py:21, compile/passes/*).

DeepCompile traces the model with Dynamo, inserts ``allgather / release / reduce`` ops into the FX
graph, profiles it, and reorders those ops with passes. This framework's ZeRO-3 already issues
those operations eagerly, per fetch group, on dedicated HIP streams; what the passes add is the
*schedule*. So the "graph" here is the recorded ZeRO-3 schedule (compile/graph.py), the profiler
is the optimizer's own schedule points (compile/profiler.py), and the passes (compile/passes.py)
rewrite which groups stay resident, where each all-gather is issued, and whether optimizer states
leave HBM. Training forward/backward stay eager -- no tracing, no recompiles on shape changes,
custom HIP ops and autograd functions untouched -- and the plan is re-derivable any time from a
fresh trace.

Flow: ``engine.compile()`` (with ``compile.deepcompile``) installs the tracer; after
``profile_steps`` optimizer steps the engine builds the graph, runs the configured passes under
the memory budget and installs the plan (``ZeroStage3Optimizer.apply_compile_plan``)."""
import torch

from ..utils.logging import log_dist
from .config import CompileConfig
from .passes import PASSES, zero3_schedule
from .profiler import ScheduleTracer


def install_profiler(opt):
    opt.tracer = ScheduleTracer(opt)
    return opt.tracer


def _budget_bytes(cfg, graph):
    b = cfg.memory_budget
    if b is None:
        b = 0.9
    if b <= 1.0:
        total = graph.device_bytes
        if not total:  # CPU: no device memory -- the budget is relative to the traced peak
            return int(graph.peak_bytes * (1.0 + b))
        return int(b * total)
    return int(b)


def compile_zero3(opt, cfg: CompileConfig):
    """Build the graph from the tracer, run the passes, install the plan; returns the plan."""
    tracer = opt.tracer
    graph = tracer.graph()
    budget = _budget_bytes(cfg, graph)
    plan = zero3_schedule(graph, {}, budget)
    for name in cfg.passes:
        fn = PASSES[name]
        if name == "prefetch":
            plan = fn(graph, plan, budget, slack=cfg.prefetch_slack)
        else:
            plan = fn(graph, plan, budget)
    plan["budget"] = budget
    plan["graph"] = graph
    opt.tracer = None
    opt.apply_compile_plan(plan)
    log_dist(f"compile: {graph.summary()}; budget {budget / 2**30:.2f} GiB; " + "; ".join(plan["log"]), ranks=[0])
    if cfg.debug_log and torch.distributed.is_initialized() and torch.distributed.get_rank() == 0:
        for n in graph.nodes:
            log_dist(f"  {n.phase} fg{n.fg}: {n.compute_ms:.3f} ms, live {n.live_bytes / 2**20:.1f} MiB, "
                     f"gather {graph.gather_bytes.get(n.fg, 0) / 2**20:.1f} MiB "
                     f"({graph.gather_ms.get(n.fg, 0.0):.3f} ms)", ranks=[0])
    return plan
