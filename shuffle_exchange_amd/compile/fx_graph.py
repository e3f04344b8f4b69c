"""FX-graph utilities and passes of the DeepCompile graph compiler for ZeRO stages 0-2
(reference compile/fx.py, compile/graph_param.py, compile/passes/zero1_compile.py,
compile/profilers/graph_profile.py).

The forward/backward graphs come from AOT autograd (compile/fx_backend.py). A parameter is a
forward placeholder whose example input is one of the engine's parameters; its gradient is the
matching entry of the backward graph's output tuple (AOT returns one gradient per forward input,
in placeholder order).

Passes:
  * ``insert_grad_reduce`` -- for every parameter gradient, a ``sxe_dc.reduce_grad`` node right
    after the node that produces it, and the graph output entry replaced by ``None``: the gradient
    goes straight to the ZeRO optimizer's bucket (which launches its all-reduce / reduce-scatter on
    the comm stream once the bucket is complete) in the middle of the compiled backward, instead of
    after the whole backward graph returns. Without it every gradient of a compiled region would
    reach the optimizer at once, at the end -- no communication/computation overlap.
  * ``sink_reduces`` -- moves each reduce node to the earliest point where its gradient exists
    (a later pass may have moved producers).
  * ``ProfilingInterpreter`` -- runs a graph node by node on real inputs and records per-node
    device time (HIP events) and allocated-memory deltas in ``node.meta`` (reference
    MemoryProfilingInterpreter); the backend logs the summary and keeps it for the passes' log.
"""
import time
from dataclasses import dataclass, field

import torch
from torch.fx import Graph, GraphModule, Interpreter, Node


def output_node(graph: Graph) -> Node:
    for n in reversed(graph.nodes):
        if n.op == "output":
            return n
    raise ValueError("graph has no output node")


def placeholders(graph: Graph):
    return [n for n in graph.nodes if n.op == "placeholder"]


@dataclass
class GraphParams:
    """Which forward inputs are parameters: [(input index, framework param id)]."""
    index_to_pid: list
    names: list = field(default_factory=list)  # forward placeholder names of the parameters


def grad_nodes(bw_graph: Graph, gp: GraphParams):
    """Backward output entries of the parameters: [(pid, node or None, output position)]."""
    outs = output_node(bw_graph).args[0]
    res = []
    for i, pid in gp.index_to_pid:
        g = outs[i] if i < len(outs) else None
        res.append((pid, g if isinstance(g, Node) else None, i))
    return res


def insert_grad_reduce(gm: GraphModule, graph_id: int, gp: GraphParams, reduce_op) -> int:
    """Add reduce_op(grad, graph_id, pid) after each parameter gradient's producer and return
    None for it from the graph. Returns the number of inserted reduces."""
    g = gm.graph
    out = output_node(g)
    outs = list(out.args[0])
    last_ph = placeholders(g)[-1] if placeholders(g) else None
    n_ins = 0
    for pid, node, pos in grad_nodes(g, gp):
        if node is None:
            continue
        anchor = last_ph if node.op == "placeholder" else node
        with g.inserting_after(anchor):
            r = g.call_function(reduce_op, (node, graph_id, pid))
        r.meta["sxe_reduce"] = pid
        outs[pos] = None
        n_ins += 1
    out.args = (tuple(outs),)
    g.lint()
    gm.recompile()
    return n_ins


def sink_reduces(gm: GraphModule) -> int:
    """Move every reduce node directly behind the producer of its gradient (earliest launch)."""
    g = gm.graph
    moved = 0
    for n in list(g.nodes):
        if "sxe_reduce" not in n.meta:
            continue
        src = n.args[0]
        if src.op == "placeholder" or src.next is n:
            continue
        src.append(n)
        moved += 1
    if moved:
        g.lint()
        gm.recompile()
    return moved


def reduce_order(gm: GraphModule):
    """Positions (node index) of the reduce nodes and the graph length -- how early in the backward
    each gradient leaves for the optimizer (logged, and asserted by the tests)."""
    nodes = list(gm.graph.nodes)
    return [i for i, n in enumerate(nodes) if "sxe_reduce" in n.meta], len(nodes)


class ProfilingInterpreter(Interpreter):
    """Run the graph once on real inputs, recording per-node time and memory in node.meta."""

    def __init__(self, gm, cuda):
        super().__init__(gm)
        self.cuda = cuda
        self.records = []

    def run_node(self, n):
        if n.op in ("placeholder", "output", "get_attr"):
            return super().run_node(n)
        if self.cuda:
            m0 = torch.cuda.memory_allocated()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            r = super().run_node(n)
            b.record()
            self.records.append((n, a, b, m0))
        else:
            t0 = time.perf_counter()
            r = super().run_node(n)
            n.meta["device_ms"] = (time.perf_counter() - t0) * 1e3
            n.meta["mem_delta"] = 0
        return r

    def finish(self):
        if self.cuda:
            torch.cuda.synchronize()
            for n, a, b, m0 in self.records:
                n.meta["device_ms"] = a.elapsed_time(b)
            # memory: the allocation high-water deltas are read after the fact per node
            for (n, _, _, m0), nxt in zip(self.records, self.records[1:] + [None]):
                n.meta["mem_delta"] = (nxt[3] if nxt else torch.cuda.memory_allocated()) - m0
        total = sum(n.meta.get("device_ms", 0.0) for n in self.module.graph.nodes)
        comm = sum(n.meta.get("device_ms", 0.0) for n in self.module.graph.nodes if "sxe_reduce" in n.meta)
        top = sorted((n for n in self.module.graph.nodes if "device_ms" in n.meta),
                     key=lambda n: -n.meta["device_ms"])[:5]
        return {"nodes": sum(1 for n in self.module.graph.nodes if "device_ms" in n.meta), "total_ms": total,
                "reduce_ms": comm, "top": [(str(n.target), round(n.meta["device_ms"], 3)) for n in top]}
